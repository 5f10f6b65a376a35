// cg_kernels.hip -- gfx950 kernels for batched cron fire-time expansion.
//
// Pipeline for Expand(specs, zone, T0, T1):
//   k_count      one lane per rule: per plan segment, the first fire (exact
//                Go walk, next_exact) and the closed-form count of the rest,
//                or the walked count inside WALK windows -> run records
//   k_scan_*     exclusive scan of run counts -> run offsets (int64); the
//                last pass also writes the rule-major CSR offsets
//   k_chunk_map  first run touched by each output slice (super_shift(cap))
//   k_write_cf   persistent, output-parallel: each wave walks its slices;
//                long runs are written wave-cooperatively (64 consecutive
//                fires per store instruction, mixed-radix digits + lane rank
//                tables), stretches of short runs lane-parallel via LDS staging
//   k_write_walk re-walks the (rare) WALK-window runs
// Integer and HBM-bound throughout: no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "cg_expand.h"
#ifndef CG_WRITE_BATCH
#define CG_WRITE_BATCH 8
#endif
#ifndef CG_WRITE_LOADER
#define CG_WRITE_LOADER 0  // production writer: k_write_lw (1) or k_write_cf (0)
#endif
#include "cg_kernels.h"

namespace cg {

namespace {

__host__ __device__ inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- plan staging into LDS --------------------------------------------
struct PlanView {
  ZoneView z;
  const Segment* segs;
  const uint32_t* dtab;
};

__device__ PlanView stage_plan(const PlanArgs& p, char* lds) {
  int64_t* w = reinterpret_cast<int64_t*>(lds);
  int32_t* o = reinterpret_cast<int32_t*>(lds + align_up(size_t(p.zn) * 8, 16));
  Segment* s = reinterpret_cast<Segment*>(lds + align_up(size_t(p.zn) * 8, 16) +
                                          align_up(size_t(p.zn) * 4, 16));
  uint32_t* d = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(s) +
                                            align_up(size_t(p.G) * sizeof(Segment), 16));
  for (int i = threadIdx.x; i < p.zn; i += blockDim.x) {
    w[i] = p.zwhen[i];
    o[i] = p.zoff[i];
  }
  const int64_t* sg = reinterpret_cast<const int64_t*>(p.segs);
  int64_t* sd = reinterpret_cast<int64_t*>(s);
  for (int i = threadIdx.x; i < p.G * int(sizeof(Segment) / 8); i += blockDim.x) sd[i] = sg[i];
  if (!p.dtab_global)
    for (int i = threadIdx.x; i < p.nd; i += blockDim.x) d[i] = p.dtab[i];
  __syncthreads();
  PlanView v;
  v.z.when = w;
  v.z.off = o;
  v.z.n = p.zn;
  v.segs = s;
  v.dtab = p.dtab_global ? p.dtab : d;
  return v;
}

__device__ __forceinline__ DSpec load_spec(const DSpec* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  DSpec s;
  s.sec = (uint64_t(a.y) << 32) | a.x;
  s.min = (uint64_t(a.w) << 32) | a.z;
  s.hour = b.x;
  s.dom = b.y;
  s.mondow = b.z;
  s.kind = b.w;
  return s;
}

// ---------------------------------------------------------------- kernels --

__global__ __launch_bounds__(256) void k_next_batch(const DSpec* __restrict__ specs, int64_t n,
                                                     PlanArgs p, const int64_t* __restrict__ t_in,
                                                     int64_t* __restrict__ t_out) {
  extern __shared__ __align__(16) char lds[];
  PlanView v = stage_plan(p, lds);
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    DSpec sp = load_spec(specs + i);
    int64_t t = t_in[i];
    if (sp.kind == KIND_EVERY) t_out[i] = t + int64_t(sp.sec);  // constantdelay.go:25-27
    else t_out[i] = next_exact(sp, v.z, t, INT64_MAX);
  }
}

// Cmd.lockTtl (job.go:194-233) per rule: prev = Next(now), Next(prev), then
// the Kind / AvgTime / LockTtl arithmetic (lock_ttl_of).
__global__ __launch_bounds__(256) void k_lock_ttl(const DSpec* __restrict__ specs, int64_t n,
                                                   PlanArgs p, const int64_t* __restrict__ now,
                                                   const int32_t* __restrict__ kind,
                                                   const int64_t* __restrict__ avg_ms,
                                                   int64_t lock_ttl, int64_t* __restrict__ ttl) {
  extern __shared__ __align__(16) char lds[];
  PlanView v = stage_plan(p, lds);
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    DSpec sp = load_spec(specs + i);
    int64_t prev, nxt;
    if (sp.kind == KIND_EVERY) {  // constantdelay.go:25-27
      prev = now[i] + int64_t(sp.sec);
      nxt = prev + int64_t(sp.sec);
    } else {
      prev = next_exact(sp, v.z, now[i], INT64_MAX);
      nxt = prev == CG_NO_PROGRESS ? prev : next_exact(sp, v.z, prev, INT64_MAX);
    }
    ttl[i] = lock_ttl_of(prev, nxt, kind[i], avg_ms[i], lock_ttl);
  }
}

// ---- GPU-resident dispatcher (Cron.run, node/cron/cron.go:210-275) ----
// Order key of an entry's Next under byTime (cron.go:64-79): the zero time
// sorts after every other time; "never returns" never fires either.
__device__ __forceinline__ unsigned long long next_key(int64_t t) {
  return (t == CG_ZERO_TIME || t == CG_NO_PROGRESS) ? ~0ull
                                                    : (uint64_t(t) ^ (uint64_t(1) << 63));
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}

// One wake of the run loop (cron.go:234-244), in three launches:
//   k_dispatch_scan     every entry whose Next equals `effective` is due: a
//                       bitmap word per 64 entries, a due count per tile, and
//                       the byTime minimum over the entries that stay;
//   k_dispatch_compact  the due slots in ascending order;
//   k_dispatch_advance  dense over the due list: Prev = Next, Next =
//                       Schedule.Next(now), folded into the minimum.
// The scan is a pure 8 B/entry stream; the Next walks run on full waves of
// due entries instead of on the few due lanes of every scanned wave.
__global__ __launch_bounds__(256) void k_dispatch_scan(
    const int64_t* __restrict__ next, int64_t n, int64_t effective,
    unsigned long long* __restrict__ due_bits, uint32_t* __restrict__ tile_cnt,
    unsigned long long* __restrict__ tile_min) {
  __shared__ unsigned long long s_min[4];
  __shared__ uint32_t s_cnt[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t base = int64_t(blockIdx.x) * kDispatchTile;
  constexpr int kIter = kDispatchTile / 256;
  // all loads first: 16 outstanding 512 B wave loads per wave
  int64_t t[kIter];
#pragma unroll
  for (int j = 0; j < kIter; j++) {
    const int64_t i = base + j * 256 + wv * 64 + lane;
    t[j] = i < n ? __builtin_nontemporal_load(next + i) : CG_ZERO_TIME;
  }
  unsigned long long kmin = ~0ull;
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < kIter; j++) {
    const int64_t w0 = base + j * 256 + wv * 64;  // first entry of this wave's word
    const bool due = t[j] == effective;           // (padding lanes hold the zero time)
    const unsigned long long k = due ? ~0ull : next_key(t[j]);
    kmin = k < kmin ? k : kmin;
    const unsigned long long b = __ballot(due);
    if (lane == 0 && w0 < n) due_bits[w0 >> 6] = b;
    cnt += __popcll(b);
  }
  kmin = wave_min_u64(kmin);
  if (lane == 0) {
    s_min[wv] = kmin;
    s_cnt[wv] = cnt;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m = s_min[0];
    uint32_t c = s_cnt[0];
    for (int w = 1; w < 4; w++) {
      m = s_min[w] < m ? s_min[w] : m;
      c += s_cnt[w];
    }
    tile_cnt[blockIdx.x] = c;  // per-tile results: thousands of same-address
    tile_min[blockIdx.x] = m;  // atomics would serialise at one L2 channel
  }
}

__global__ __launch_bounds__(256) void k_dispatch_advance(
    const DSpec* __restrict__ specs, const int32_t* __restrict__ due, PlanArgs p, int64_t now,
    int64_t* __restrict__ next, int64_t* __restrict__ prev, DispatchState* __restrict__ st) {
  extern __shared__ __align__(16) char lds[];
  const int64_t m = int64_t(*(volatile unsigned long long*)&st->n_due);
  if (int64_t(blockIdx.x) * blockDim.x >= m) return;  // uniform: before any barrier
  PlanView v = stage_plan(p, lds);
  unsigned long long kmin = ~0ull;
  for (int64_t j = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; j < m;
       j += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = due[j];
    const DSpec sp = load_spec(specs + i);
    prev[i] = next[i];
    const int64_t t =
        sp.kind == KIND_EVERY ? now + int64_t(sp.sec) : next_exact(sp, v.z, now, INT64_MAX);
    if (t == CG_NO_PROGRESS) atomicMin(&st->stuck, (unsigned long long)i);
    next[i] = t;
    const unsigned long long k = next_key(t);
    kmin = k < kmin ? k : kmin;
  }
  __shared__ unsigned long long s_min[4];
  kmin = wave_min_u64(kmin);
  if ((threadIdx.x & 63) == 0) s_min[threadIdx.x >> 6] = kmin;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long m2 = s_min[0];
    for (int w = 1; w < 4; w++) m2 = s_min[w] < m2 ? s_min[w] : m2;
    if (m2 != ~0ull) atomicMin(&st->min_key, m2);
  }
}

// Due entry indices in ascending order: tile base = sum of the earlier tiles'
// counts, then wave 0 expands the tile's 64 bitmap words in order.
__global__ __launch_bounds__(256) void k_dispatch_compact(
    const unsigned long long* __restrict__ due_bits, const uint32_t* __restrict__ tile_cnt,
    const unsigned long long* __restrict__ tile_min, int64_t n, int32_t* __restrict__ due,
    DispatchState* __restrict__ st) {
  __shared__ unsigned long long s_sum[4], s_min[4];
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (b == int64_t(gridDim.x) - 1) {  // the wake's totals: due count, minimum of the rest
    unsigned long long c = 0, m = ~0ull;
    for (int64_t k = threadIdx.x; k < gridDim.x; k += 256) {
      c += tile_cnt[k];
      m = tile_min[k] < m ? tile_min[k] : m;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    m = wave_min_u64(m);
    if (lane == 0) {
      s_sum[wv] = c;
      s_min[wv] = m;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the whole wake state: no host-side reset needed
      st->stuck = ~0ull;
      st->n_due = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
      unsigned long long mm = s_min[0];
      for (int w = 1; w < 4; w++) mm = s_min[w] < mm ? s_min[w] : mm;
      st->min_key = mm;
    }
    __syncthreads();
  }
  if (tile_cnt[b] == 0) return;
  unsigned long long s = 0;
  for (int64_t k = threadIdx.x; k < b; k += 256) s += tile_cnt[k];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) s_sum[wv] = s;
  __syncthreads();
  if (wv != 0) return;
  const int64_t tile_base = s_sum[0] + s_sum[1] + s_sum[2] + s_sum[3];
  const int64_t w = b * (kDispatchTile / 64) + lane;
  unsigned long long bits = w * 64 < n ? due_bits[w] : 0ull;
  const uint32_t pc = __popcll(bits);
  uint32_t incl = pc;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  int64_t o = tile_base + (incl - pc);
  while (bits) {
    due[o++] = int32_t(w * 64 + __builtin_ctzll(bits));
    bits &= bits - 1;
  }
}

// Entries (re)placed at time now (run start, cron.go:212-215; add, cron.go:246-252):
// Next = Schedule.Next(now), Prev = zero.  idx == nullptr: entries [first, first+k).
__global__ __launch_bounds__(256) void k_dispatch_place(
    DSpec* __restrict__ specs, const int64_t* __restrict__ idx, const DSpec* __restrict__ src,
    int64_t first, int64_t k, PlanArgs p, int64_t now, int64_t* __restrict__ next,
    int64_t* __restrict__ prev, DispatchState* __restrict__ st) {
  extern __shared__ __align__(16) char lds[];
  PlanView v = stage_plan(p, lds);
  for (int64_t j = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; j < k;
       j += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = idx ? idx[j] : first + j;
    DSpec sp;
    if (src) {
      sp = load_spec(src + j);
      specs[i] = sp;
    } else {
      sp = load_spec(specs + i);
    }
    const int64_t t =
        sp.kind == KIND_EVERY ? now + int64_t(sp.sec) : next_exact(sp, v.z, now, INT64_MAX);
    if (t == CG_NO_PROGRESS) atomicMin(&st->stuck, (unsigned long long)i);
    next[i] = t;
    prev[i] = CG_ZERO_TIME;
  }
}

// Entries removed (cron.go:254-262) or slots never filled: Next = Prev = zero,
// which byTime sorts last and no wake ever matches.
__global__ void k_dispatch_clear(const int64_t* __restrict__ idx, int64_t first, int64_t k,
                                 int64_t* __restrict__ next, int64_t* __restrict__ prev) {
  for (int64_t j = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; j < k;
       j += int64_t(gridDim.x) * blockDim.x) {
    const int64_t i = idx ? idx[j] : first + j;
    next[i] = CG_ZERO_TIME;
    prev[i] = CG_ZERO_TIME;
  }
}

// byTime minimum over all entries (after adds / removes).
__global__ __launch_bounds__(256) void k_dispatch_min(const int64_t* __restrict__ next, int64_t n,
                                                       DispatchState* __restrict__ st) {
  unsigned long long m = ~0ull;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const unsigned long long k = next_key(next[i]);
    m = k < m ? k : m;
  }
  __shared__ unsigned long long s_min[4];
  m = wave_min_u64(m);
  if ((threadIdx.x & 63) == 0) s_min[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 4; w++) m = s_min[w] < m ? s_min[w] : m;
    m = s_min[0] < m ? s_min[0] : m;
    if (m != ~0ull) atomicMin(&st->min_key, m);
  }
}

#ifndef CG_COUNT_WPE
#define CG_COUNT_WPE 4  // register budget of k_count: 4 waves per SIMD (walk path 133 -> 128 VGPRs, 24 B spill; DST-day step 2.37 -> 2.12 ms)
#endif
template <bool kWalk>
__global__ __launch_bounds__(256)
#if CG_COUNT_WPE
__attribute__((amdgpu_waves_per_eu(CG_COUNT_WPE)))
#endif
void k_count(const DSpec* __restrict__ specs, int64_t R,
                                                PlanArgs p, int64_t* __restrict__ run_anchor,
                                                int32_t* __restrict__ run_count,
                                                uint32_t* __restrict__ run_dmask,
                                                unsigned long long* __restrict__ stuck_rule) {
  extern __shared__ __align__(16) char lds[];
  PlanView v = stage_plan(p, lds);
  const int G = p.G;
  for (int64_t r = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; r < R;
       r += int64_t(gridDim.x) * blockDim.x) {
    DSpec sp = load_spec(specs + r);
    const int64_t j0 = r * G;
    if (!count_rule<kWalk>(sp, v.z, v.segs, G, v.dtab, p.t0, p.t1, p.flags, run_anchor + j0, run_count + j0,
                    run_dmask + j0))
      atomicMin(stuck_rule, (unsigned long long)r);
  }
}

// ---- scan: int32 counts -> int64 exclusive offsets -----------------------
constexpr int kScanThreads = 256;
#ifndef CG_SCAN_PER_THREAD
#define CG_SCAN_PER_THREAD 4  // A/B (profiles/r02_ab_scan.json): config 2 scan 32 -> 21.5 us at 4 (16 items: 245 blocks, < 1 wave per SIMD)
#endif
constexpr int kScanPerThread = CG_SCAN_PER_THREAD;
constexpr int kScanTile = kScanThreads * kScanPerThread;
constexpr int64_t kScanFuseTiles = 1024;  // up to 4M elements: carries summed per block

__device__ __forceinline__ int64_t wave_incl_scan(int64_t x) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// block-wide exclusive scan of x (256 threads); returns prefix, total in *tot
__device__ int64_t block_excl_scan(int64_t x, int64_t* tot) {
  __shared__ int64_t wsum[kScanThreads / 64];
  int64_t inc = wave_incl_scan(x);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int64_t base = 0, all = 0;
  for (int i = 0; i < kScanThreads / 64; i++) {
    if (i < w) base += wsum[i];
    all += wsum[i];
  }
  __syncthreads();
  *tot = all;
  return base + inc - x;
}

template <class T>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const T* __restrict__ in, int64_t n,
                                                               int64_t* __restrict__ partial) {
  int64_t base = int64_t(blockIdx.x) * kScanTile;
  int64_t acc = 0;
  for (int i = 0; i < kScanPerThread; i++) {
    int64_t idx = base + int64_t(i) * kScanThreads + threadIdx.x;
    if (idx < n) acc += in[idx];
  }
  int64_t tot;
  block_excl_scan(acc, &tot);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_top(int64_t* __restrict__ partial,
                                                            int64_t nb) {
  int64_t carry = 0;
  for (int64_t base = 0; base < nb; base += kScanThreads) {
    int64_t idx = base + threadIdx.x;
    int64_t x = idx < nb ? partial[idx] : 0;
    int64_t tot;
    int64_t pre = block_excl_scan(x, &tot);
    if (idx < nb) partial[idx] = carry + pre;
    carry += tot;
    __syncthreads();
  }
}

// RunTail (expansion scan only, else all null): per-rule CSR offsets
// offsets[r] = out[r*G], the result words res = {E, stuck rule} and the
// stuck flag re-armed for the next call: the host reads E and the stuck rule
// in one 16-B record, with no memset before k_count.
// With chunk_run set it also builds k_write_cf's slice map for an output
// capacity of cap events (what k_chunk_map does, from the run bounds the
// thread already holds) and resets the writer's slice tickets.
struct RunTail {
  int64_t* offsets;
  int64_t* res;
  unsigned long long* stuck;
  int32_t G;
  int64_t* chunk_run;
  int64_t cap;
};

// kFused: the tile's carry is the sum of the earlier tiles' totals, summed by
// the block itself (no k_scan_top launch; used while nb <= kScanFuseTiles)
template <class T, bool kFused>
__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const T* __restrict__ in, int64_t n,
                                                              const int64_t* __restrict__ partial,
                                                              int64_t* __restrict__ out,
                                                              RunTail tail) {
  int64_t carry;
  if (kFused) {
    int64_t x = 0;
    for (int64_t i = threadIdx.x; i < int64_t(blockIdx.x); i += kScanThreads) x += partial[i];
    int64_t all;
    block_excl_scan(x, &all);
    carry = all;
  } else {
    carry = partial[blockIdx.x];
  }
  int64_t base = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanPerThread;
  T v[kScanPerThread];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    int64_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0;
    acc += v[i];
  }
  int64_t tot;
  int64_t run = carry + block_excl_scan(acc, &tot);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = 0;
    if (tail.offsets) tail.offsets[0] = 0;
  }
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    int64_t idx = base + i;
    run += v[i];
    if (idx < n) out[idx + 1] = run;
  }
  if (tail.offsets) {
    const int sh = super_shift(tail.cap);
    const int64_t sup = int64_t(1) << sh;
    const int64_t last_sup = tail.cap >> sh;  // map entries 0 .. last_sup + 1
    if (tail.chunk_run && blockIdx.x == 0)
      for (int i = threadIdx.x; i < kTicketWords + 8; i += kScanThreads)
        tail.chunk_run[last_sup + 2 + i] = 0;
    int64_t r = run;  // out[idx + 1] for the last idx of this thread, walked back
#pragma unroll
    for (int i = kScanPerThread - 1; i >= 0; i--) {
      const int64_t idx = base + i;
      if (idx < n && (tail.G == 1 || (idx + 1) % tail.G == 0))
        tail.offsets[(idx + 1) / tail.G] = r;
      if (tail.chunk_run && idx < n && v[i] > 0) {
        // slices whose first event lies in this (non-empty) run: the largest
        // j with run_off[j] <= c*sup, as k_chunk_map's search finds it
        const int64_t lo = r - v[i];
        for (int64_t c = (lo + sup - 1) >> sh; (c << sh) < r && c <= last_sup; c++)
          tail.chunk_run[c] = idx;
      }
      r -= v[i];
    }
    if (base <= n - 1 && n - 1 < base + kScanPerThread) {
      tail.res[0] = run;  // = out[n]: the thread's values past n - 1 are zeros
      tail.res[1] = int64_t(*tail.stuck);
      *tail.stuck = ~0ull;
      const int64_t nsup = (run + sup - 1) >> sh;
      if (tail.chunk_run && nsup <= last_sup + 1) tail.chunk_run[nsup] = n - 1;
    }
  }
}

// largest j in [lo, hi] with off[j] <= x
__device__ __forceinline__ int64_t search_run(const int64_t* __restrict__ off, int64_t lo,
                                              int64_t hi, int64_t x) {
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Cost-space slice map of a short window (cg_kernels.h, u_mode): per slice c
// {P_c, run holding P_c}, P_c = the position of u = c * 2^s rounded down to a
// 64-event block; entry nsl = {E, last run}.  E is read on the device.
__global__ void k_chunk_map_u(const int64_t* __restrict__ run_off, int64_t nruns, int64_t cap,
                              int64_t* __restrict__ chunk_run) {
  const int64_t E = run_off[nruns];
  if (E > cap || !u_mode(E, cap)) return;
  const int64_t U = E + nruns;
  const int s = u_shift(U);
  const int64_t nsl = (U + (int64_t(1) << s) - 1) >> s;
  int64_t* m = chunk_run + u_map_base(cap);
  for (int64_t c = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; c <= nsl; c += int64_t(gridDim.x) * blockDim.x) {
    int64_t P = E, jr = nruns - 1;
    if (c < nsl) {
      const int64_t u = c << s;
      int64_t lo = 0, hi = nruns - 1;  // the run whose cost range holds u: largest j with off_j + j <= u
      while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (run_off[mid] + mid <= u) lo = mid;
        else hi = mid - 1;
      }
      const int64_t pos = min(run_off[lo] + (u - run_off[lo] - lo), run_off[lo + 1]);
      P = pos & ~int64_t(63);
      jr = search_run(run_off, 0, nruns - 1, P);
    }
    m[2 * c] = P;
    m[2 * c + 1] = jr;
  }
}

// first run touched by each output slice (2^super_shift(cap) events); E is read on the device
// so the launch needs no host sync (grid sized by capacity, extra threads exit)
// (chunk_run holds slice_map_words(cap) entries: the map, then the
// writer's slice ticket counters, reset here)
__global__ void k_chunk_map(const int64_t* __restrict__ run_off, int64_t nruns, int64_t cap,
                            int64_t* __restrict__ chunk_run) {
  const int sh = super_shift(cap);
  const int64_t sup = int64_t(1) << sh;
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < kTicketWords + 8; i += blockDim.x) chunk_run[(cap >> sh) + 2 + i] = 0;
  const int64_t E = run_off[nruns];
  if (E > cap) return;
  const int64_t nsup = (E + sup - 1) >> sh;
  for (int64_t c = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; c <= nsup;
       c += int64_t(gridDim.x) * blockDim.x)
    chunk_run[c] = c == nsup ? nruns - 1 : search_run(run_off, 0, nruns - 1, c << sh);
}


// one run of a wave's 64-run window (lane i holds run jw + i), staged in LDS
// (48 B; the run offset stays in a VGPR of lane i, the plan segment index
// rides in the spec's kind word: kind | seg << 8)
struct WinRun {
  int64_t anchor;  // run_anchor[j]
  DSpec sp;        // specs[j / G]
  int32_t count;   // run_count[j]
  uint32_t dmask;  // run_dmask[j]
};
__device__ __forceinline__ bool win_every(const WinRun& w) { return (w.sp.kind & 0xFFu) == KIND_EVERY; }
__device__ __forceinline__ int win_seg(const WinRun& w) { return int(w.sp.kind >> 8); }

__device__ __forceinline__ int32_t rl32(int32_t v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ int64_t rl64(int64_t v, int i) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), i));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), i));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// Lane k of the result holds unit * (position of the k-th set bit of m), for
// k < popcount(m): each lane pushes its own position to the lane of its rank
// (set bits to 0..n-1, clear bits to n..63 -- a permutation), ds_permute_b32.
// All 64 lanes must be active.
__device__ __forceinline__ int32_t rank_table(uint64_t m, int32_t unit) {
  const int lane = threadIdx.x & 63;
  const bool set = (m >> lane) & 1ull;
  const int32_t below = __popcll(m & ((1ull << lane) - 1ull));
  const int32_t n = __popcll(m);
  const int32_t dst = set ? below : n + (lane - below);
  return __builtin_amdgcn_ds_permute(dst << 2, lane * unit);
}
// entry idx of a rank table (ds_bpermute_b32; idx is taken mod 64)
__device__ __forceinline__ int32_t rank_at(int32_t table, uint32_t idx) {
  return __builtin_amdgcn_ds_bpermute(int(idx << 2), table);
}
// floor(x / n) for x < 2^16, n >= 1, with inv = 1/n (the +0.5 keeps the
// product at least 0.5/n away from an integer, far above the f32 error)
__device__ __forceinline__ uint32_t small_div(uint32_t x, float inv) {
  return uint32_t((float(x) + 0.5f) * inv);
}
// floor(x / n) for x < 2^24, n >= 1, inv = 1/n: the f32 quotient is off by at
// most one, fixed by one remainder test each way (cheaper than a u32 divide)
__device__ __forceinline__ uint32_t fdiv(uint32_t x, uint32_t n, float inv) {
  uint32_t q = uint32_t(float(x) * inv);
  const int32_t r = int32_t(x) - int32_t(q * n);
  q = r < 0 ? q - 1u : (r >= int32_t(n) ? q + 1u : q);
  return q;
}

// Output store.  V (diagnostic variants, CG_WRITE_VARIANT; 0 in production):
// bit 0 = compute only (no store, value kept live), bit 1 = non-temporal store,
// bit 2 = skip the short runs, bit 3 = skip the long runs, bit 4 = static slice
// split instead of tickets, bit 5 = per-phase clock stats, bit 6 = plain fill.
template <int V>
__device__ __forceinline__ void put(int64_t* p, int64_t v) {
  if (V & 1) {
    asm volatile("" ::"v"(v));
  } else if (V & 2) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// cf_seek (cg_expand.h) with the three variable divisions done by fdiv
// (quotients < 2^24); same result, fewer instructions.
__device__ __forceinline__ CFIter cf_seek_fast(const CFRule& c, const Segment& sg, uint32_t dmask,
                                               int64_t uf, int64_t k) {
  if (k == 0) return cf_decode(sg, uf);
  const uint32_t rf = uint32_t(uf - sg.base);
  const uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  uint32_t idx = cf_rank(c, int32_t(tf)) - 1u + uint32_t(k);
  CFIter it;
  it.day = int32_t(jf);
  if (idx >= c.C) {
    idx -= c.C;
    const uint32_t dskip = fdiv(idx, c.C, 1.0f / float(c.C));
    idx -= dskip * c.C;
    const uint64_t above = uint64_t(dmask) & ~((2ull << jf) - 1ull);
    it.day = select64(above, dskip);
  }
  const uint32_t hi = fdiv(idx, c.nMS, 1.0f / float(c.nMS));
  const uint32_t rem = idx - hi * c.nMS;
  const uint32_t mi = fdiv(rem, c.nS, 1.0f / float(c.nS));
  const uint32_t si = rem - mi * c.nS;
  it.h = select64(c.H, hi);
  it.m = select64(c.M, mi);
  it.s = select64(c.S, si);
  return it;
}

// Does mask m (n set bits) hold an arithmetic progression p0 + r*step?
// (rank r -> position is then linear; n <= 1 counts, with step 0)
__device__ __forceinline__ bool ap_level(uint64_t m, uint32_t n, int32_t* p0, int32_t* step) {
  *p0 = m ? __builtin_ctzll(m) : 0;
  *step = 0;
  if (n <= 1) return true;
  const uint64_t rest = m >> *p0;  // bit 0 set
  const int32_t st = __builtin_ctzll(rest >> 1) + 1;
  *step = st;
  // {0, st, 2st, ...} up to the top bit  <=>  ((rest << st) | 1) below the top == rest
  const int32_t top = 63 - __builtin_clzll(rest);
  const uint64_t low = top >= 63 ? ~0ull : ((2ull << top) - 1ull);
  return (((rest << st) | 1ull) & low) == rest;
}

// The aligned 64-fire block holding a run boundary, assembled across runs:
// each run fills its lanes, and the run that completes the block stores it
// with one whole 512 B store (no partially written cache line reaches HBM).
struct Pending {
  int64_t blk;  // block start, or -1 (wave-uniform)
  int64_t val;  // this lane's fire in it
};

// Position offset of this lane's first fire of a piece starting at p0: lane l
// covers p0 + x, x = (floor64(p0) + l - p0) mod 64 -- lanes before p0 in the
// head block belong to earlier runs and start one block later.
__device__ __forceinline__ uint32_t lane_offset(int64_t p0) {
  const int lane = threadIdx.x & 63;
  const int32_t x = int32_t((p0 & ~int64_t(63)) + lane - p0);
  return uint32_t(x < 0 ? x + 64 : x);
}

constexpr int kBatch = CG_WRITE_BATCH;  // blocks computed before their stores are issued
#ifndef CG_WRITE_TAKE
#define CG_WRITE_TAKE 1
#endif
constexpr int kTake = CG_WRITE_TAKE;  // writer slices per ticket atomic
#ifndef CG_WRITE_MIXED
#define CG_WRITE_MIXED 1
#endif
#ifndef CG_WRITE_SPARE_BLOCKS
#define CG_WRITE_SPARE_BLOCKS 0
#endif
constexpr bool kMixedBlocks = CG_WRITE_MIXED;  // blocks holding several runs filled lane-parallel
// 64-bit ds_bpermute (lane src's value; src taken mod 64)
__device__ __forceinline__ int64_t bperm64_w(int64_t v, int src) {
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(v)));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(uint64_t(v) >> 32)));
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

// Runs the piece [p0, p1) through the block protocol: value() is this lane's
// current fire, step() advances it by 64 fires.  Full blocks are stored as
// computed (8 values first, then 8 stores: a wave held back by a full memory
// pipe has no arithmetic queued behind the store); the head block merges the
// pending fires of earlier runs; a partial tail block becomes pending.
// GAP: a walked run -- its fires come from k_write_walk, so only the shared
// blocks are written (placeholders there), never its own full blocks.
template <int V, bool GAP, class Val, class Step>
__device__ __forceinline__ void drive(Val&& value, Step&& step, int64_t p0, int64_t p1,
                                      Pending& pd, int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63;
  const int64_t b0 = p0 & ~int64_t(63);
  const bool mine0 = b0 + lane >= p0;
  {
    int64_t v = GAP ? 0 : value();
    if (!mine0) v = pd.val;
    if (b0 + 64 > p1) {  // the run ends inside its head block
      pd.blk = b0;
      pd.val = v;
      return;
    }
    put<V>(times + b0 + lane, v);
    pd.blk = -1;
    if (!GAP && mine0) step();
  }
  int64_t b = b0 + 64;
  if (GAP) {
    b += (p1 - b) & ~int64_t(63);
  } else {
    for (; b + kBatch * 64 <= p1; b += kBatch * 64) {
      int64_t vv[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        vv[u] = value();
        step();
      }
#pragma unroll
      for (int u = 0; u < kBatch; u++) asm volatile("" : "+v"(vv[u]));
#pragma unroll
      for (int u = 0; u < kBatch; u++) put<V>(times + b + 64 * u + lane, vv[u]);
    }
    for (; b + 64 <= p1; b += 64) {
      put<V>(times + b + lane, value());
      step();
    }
  }
  if (b < p1) {
    pd.blk = b;
    pd.val = GAP ? 0 : value();
  }
}

// Fires [p0, p1) of closed-form run w (run start roff), wave-cooperatively.
// A fire's index g = rank(anchor) - 1 + (p - roff) counts (day, hour, minute,
// second) combinations from the anchor's local day, so it is carried as
// mixed-radix digits (matching-day rank, hour/minute/second ranks; radices -,
// nH, nM, nS) and stepped by the constant 64.  Same enumeration as
// cf_seek/cf_next.  Rank -> seconds, cheapest form first:
//   linear   every level an arithmetic progression and the sequence has one
//            stride (e.g. */10 s with every minute/hour/day): t += 64*stride;
//   affine   every level an arithmetic progression: t = C0 + sum r_i * w_i;
//   tables   otherwise: per-level lane tables read with ds_bpermute.
template <int V>
__device__ void coop_cf(const WinRun& w, int64_t roff, const Segment& sg, int64_t p0, int64_t p1,
                        Pending& pd, int64_t* __restrict__ times) {
  const CFRule c = cf_rule(w.sp);
  const uint32_t nS = c.nS, nM = c.nM, nH = uint32_t(__builtin_popcount(c.H));
  const uint32_t rf = uint32_t(w.anchor - sg.base);
  const uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  const uint32_t dmask = w.dmask >> jf;  // matching days from the anchor's (bit 0)
  const float iS = 1.0f / float(nS), iM = 1.0f / float(nM), iH = 1.0f / float(nH);
  // g < 31 * 86400 < 2^24
  uint32_t g = cf_rank(c, int32_t(tf)) - 1u + uint32_t(p0 - roff);
  uint32_t d = fdiv(g, c.C, 1.0f / float(c.C));
  g -= d * c.C;
  uint32_t h = fdiv(g, c.nMS, 1.0f / float(c.nMS));
  g -= h * c.nMS;
  uint32_t m = fdiv(g, nS, iS);
  uint32_t s = g - m * nS;
  // + this lane's offset (< 128)
  uint32_t q;
  s += lane_offset(p0);
  q = small_div(s, iS);
  s -= q * nS;
  m += q;
  q = small_div(m, iM);
  m -= q * nM;
  h += q;
  q = small_div(h, iH);
  h -= q * nH;
  d += q;
  // digits of 64
  uint32_t a = small_div(64, iS);
  const uint32_t a0 = 64 - a * nS;
  uint32_t a_ = small_div(a, iM);
  const uint32_t a1 = a - a_ * nM;
  a = small_div(a_, iH);
  const uint32_t a2 = a_ - a * nH;
  const uint32_t a3 = a;
  auto step = [&]() {
    s += a0;
    const uint32_t cs = s >= nS;
    s -= cs ? nS : 0u;
    m += a1 + cs;
    const uint32_t cm = m >= nM;
    m -= cm ? nM : 0u;
    h += a2 + cm;
    const uint32_t ch = h >= nH;
    h -= ch ? nH : 0u;
    d += a3 + ch;
  };
  int32_t s0, ss, m0, ms, h0, hs, d0, ds;
  const uint32_t nD = uint32_t(__builtin_popcount(dmask));
  const bool apS = ap_level(c.S, nS, &s0, &ss), apM = ap_level(c.M, nM, &m0, &ms);
  const bool apH = ap_level(c.H, nH, &h0, &hs), apD = ap_level(dmask, nD, &d0, &ds);
  if (apS && apM && apH && apD) {
    const int64_t C0 = sg.base + s0 + 60 * m0 + 3600 * h0 + 86400 * int32_t(jf);  // d0 == 0
    const uint32_t ws = uint32_t(ss), wm = 60u * uint32_t(ms), wh = 3600u * uint32_t(hs),
                   wd = 86400u * uint32_t(ds);
    auto value = [&]() -> int64_t {
      // every product < 2^24 x 2^24 operands: v_mul_u32_u24 (full rate)
      return C0 + int64_t(__umul24(s, ws) + __umul24(m, wm) + __umul24(h, wh) + __umul24(d, wd));
    };
    // one stride: the lowest level with > 1 value wraps evenly into the next
    // unit, and every level above it takes every value (days: consecutive)
    const bool days_full = nD <= 1 || ds == 1;
    int32_t stride = 0;
    if (nS > 1) {
      if (uint32_t(ss) * nS == 60 && s0 < ss && nM == 60 && nH == 24 && days_full) stride = ss;
    } else if (nM > 1) {
      if (uint32_t(ms) * nM == 60 && m0 < ms && nH == 24 && days_full) stride = 60 * ms;
    } else if (nH > 1) {
      if (uint32_t(hs) * nH == 24 && h0 < hs && days_full) stride = 3600 * hs;
    } else {
      stride = 86400 * ds;
    }
    if (stride > 0) {
      int64_t v = value();
      const int64_t st = 64 * int64_t(stride);
      drive<V, false>([&]() { return v; }, [&]() { v += st; }, p0, p1, pd, times);
    } else {
      drive<V, false>(value, step, p0, p1, pd, times);
    }
    return;
  }
  const int32_t ts = rank_table(c.S, 1);
  const int32_t tm = rank_table(c.M, 60);
  const int32_t th = rank_table(c.H, 3600);
  const int32_t td = rank_table(uint64_t(dmask), 86400) + int32_t(jf) * 86400;
  const int64_t base = sg.base;
  auto value = [&]() -> int64_t {  // all lanes active: the table reads are cross-lane
    return base + int64_t(rank_at(td, d) + rank_at(th, h) + rank_at(tm, m) + rank_at(ts, s));
  };
  drive<V, false>(value, step, p0, p1, pd, times);
}

// Fires [p0, p1) of a short closed-form run: each lane seeks its own fire
// (the anchor itself, its successor, or cf_seek).
template <int V>
__device__ void tiny_cf(const WinRun& w, int64_t roff, const Segment& sg, int64_t p0, int64_t p1,
                        Pending& pd, int64_t* __restrict__ times) {
  int32_t k = int32_t(p0 - roff) + int32_t(lane_offset(p0));
  const CFRule c = cf_rule(w.sp);
  auto value = [&]() -> int64_t {
    if (k == 0) return w.anchor;
    if (int64_t(k) >= p1 - roff) return 0;  // not this run's (a later run's lane)
    if (k == 1) {
      CFIter it = cf_decode(sg, w.anchor);
      cf_next(c, w.dmask, it);
      return cf_value(sg, it);
    }
    return cf_value(sg, cf_seek_fast(c, sg, w.dmask, w.anchor, k));
  };
  drive<V, false>(value, [&]() { k += 64; }, p0, p1, pd, times);
}

// Fires [p0, p1) of @every run w: anchor + (k + 1) * D (constantdelay.go:25-27)
template <int V>
__device__ void coop_every(const WinRun& w, int64_t roff, int64_t p0, int64_t p1, Pending& pd,
                           int64_t* __restrict__ times) {
  const int64_t D = int64_t(w.sp.sec);
  int64_t t = w.anchor + (p0 - roff + int64_t(lane_offset(p0)) + 1) * D;
  const int64_t st = 64 * D;
  drive<V, false>([&]() { return t; }, [&]() { t += st; }, p0, p1, pd, times);
}

// Fire k (>= 0) of window run w, for one lane (the per-lane form of
// coop_every / tiny_cf): @every anchor + (k + 1) D (constantdelay.go:25-27),
// a walked run's placeholder 0 (k_write_walk writes it), else the k-th
// closed-form fire from the anchor.
__device__ __forceinline__ int64_t run_fire(const WinRun& w, const Segment& sg, int64_t k) {
  if (win_every(w)) return w.anchor + (k + 1) * int64_t(w.sp.sec);
  if (run_is_walked(sg, w.dmask)) return 0;
  if (k == 0) return w.anchor;
  const CFRule c = cf_rule(w.sp);
  if (k == 1) {
    CFIter it = cf_decode(sg, w.anchor);
    cf_next(c, w.dmask, it);
    return cf_value(sg, it);
  }
  return cf_value(sg, cf_seek_fast(c, sg, w.dmask, w.anchor, k));
}

// Persistent closed-form writer.  Waves work independently on 2^super_shift(cap)-event
// output slices, handed out by ticket.  A wave keeps a window of 64
// consecutive runs (one coalesced round of loads, staged in its LDS slice;
// only the runs the slice can touch are loaded) and walks its slice run by
// run, in aligned 64-fire blocks: every store instruction writes one whole
// 512 B block (a block shared by several runs is assembled across them, see
// Pending), so no partially written cache line reaches HBM.  Long runs are
// generated wave-cooperatively from mixed-radix digits (coop_cf) or the
// @every progression (coop_every); short runs by per-lane seeks (tiny_cf).
// Walked runs' own blocks are left to k_write_walk, which runs after this
// kernel.
template <int V>
__global__ __launch_bounds__(kWriteWaves * 64, kWriteBlocksPerCU) void k_write_cf(
    const DSpec* __restrict__ specs, PlanArgs p, const int64_t* __restrict__ run_anchor,
    const int32_t* __restrict__ run_count, const uint32_t* __restrict__ run_dmask,
    const int64_t* __restrict__ run_off, int64_t nruns, int64_t* __restrict__ chunk_run,
    int64_t cap, int64_t* __restrict__ times) {
  __shared__ WinRun win_all[kWriteWaves][64];
  extern __shared__ __align__(16) char dyn[];  // the plan's G segments
  Segment* segs = reinterpret_cast<Segment*>(dyn);
  for (int i = threadIdx.x; i < p.G * int(sizeof(Segment) / 8); i += blockDim.x)
    reinterpret_cast<int64_t*>(segs)[i] = reinterpret_cast<const int64_t*>(p.segs)[i];
  __syncthreads();

  const int G = p.G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  WinRun* win = win_all[wave];
  const int64_t E = run_off[nruns];
  if (E > cap) return;  // output buffer too small: host grows it and relaunches
  const int sh = super_shift(cap);
  const int64_t sup = int64_t(1) << sh;
  // short windows: slices from the cost-space map (k_chunk_map_u)
  const bool um = u_mode(E, cap);
  const int64_t* umap = chunk_run + u_map_base(cap);
  const int64_t nsup = um ? ((E + nruns + (int64_t(1) << u_shift(E + nruns)) - 1) >> u_shift(E + nruns))
                          : (E + sup - 1) >> sh;
  int64_t woff = INT64_MAX;  // this lane's window run: offset, count
  int32_t wcnt = 0;
  int64_t jend = nruns;  // runs the current slice can touch: [.., jend)
  auto load_window = [&](int64_t j0) {
    __syncwarp();  // every lane is done with the previous window
    const int64_t jl = j0 + lane;
    WinRun w;
    int64_t off = INT64_MAX;
    if (jl < jend) {  // only the runs this slice needs: no over-fetch into the write stream
      const int64_t r = G == 1 ? jl : jl / G;
      off = run_off[jl];
      w.anchor = run_anchor[jl];
      w.count = run_count[jl];
      w.dmask = run_dmask[jl];
      w.sp = load_spec(specs + r);
      w.sp.kind |= uint32_t(jl - r * G) << 8;
    } else {
      w.anchor = 0;
      w.count = 0;
      w.dmask = 0;
      w.sp = DSpec{};
    }
    win[lane] = w;
    woff = off;
    wcnt = w.count;
    __syncwarp();
  };
  // Slices are handed out dynamically (the cost per slice varies with the
  // spec mix; a static split leaves a long tail).  kTicketGroups counters,
  // 128 B apart, one per group of blocks (blocks go round-robin over the
  // groups): group g's counter hands out slices g, g + ng, g + 2 ng, ..., so
  // the atomics spread over ng addresses.  With large slices a wave whose
  // group has run out moves on to the next group's counter (no group's tail
  // waits on its own waves alone).  Tickets are taken one slice ahead so the atomic's latency
  // hides under the current slice.
  const int ng = gridDim.x < kTicketGroups ? int(gridDim.x) : kTicketGroups;
  const int grp = int(blockIdx.x % unsigned(ng));
  unsigned int* tickets = reinterpret_cast<unsigned int*>(chunk_run + (cap >> sh) + 2);
  int cur = grp, hops = 0;  // the group whose slices this wave takes, groups left behind
  // (same-box A/B, profiles/r02_ab_steal.json: config 4 with 16384-event
  // slices 23.7 vs 24.5 ms; config 2 with 2048-event slices 1.03 vs 0.99 ms:
  // moving on only pays with the large slices)
  const bool steal = sh == CG_SUPER_SHIFT_LARGE;
  int64_t static_next = int64_t(blockIdx.x) * kWriteWaves + wave;
  // kTake consecutive tickets of the group per atomic (the atomic's result is
  // waited for behind every store the wave has issued).  Same-box A/B,
  // profiles/r02_ab_writer_lw.json: 1 is best -- 2/4/8 lose more to the
  // coarser tail than the fewer atomics save
  uint32_t tk_next = 0, tk_left = 0;
  auto take = [&]() -> int64_t {
    if (V & 16) {  // diagnostic: static grid-stride split
      const int64_t t = static_next;
      static_next += int64_t(gridDim.x) * kWriteWaves;
      return t;
    }
    for (;;) {
      if (tk_left == 0) {
        unsigned int t = 0;
        if (lane == 0) t = atomicAdd(tickets + cur * kTicketStride, unsigned(kTake));
        tk_next = uint32_t(__builtin_amdgcn_readfirstlane(int(t)));
        tk_left = kTake;
      }
      const int64_t c = cur + int64_t(ng) * int64_t(tk_next);
      tk_next++;
      tk_left--;
      if (c < nsup || !steal || ++hops >= ng) return c;
      cur = cur + 1 == ng ? 0 : cur + 1;
      tk_left = 0;
    }
  };
  // V & 32 (diagnostic): per-phase shader-clock totals and counts
  uint64_t st_win = 0, st_long = 0, st_all = 0, n_win = 0, n_long = 0, st_mix = 0, n_mix = 0;
  auto clk = [&]() -> uint64_t { return (V & 32) ? __builtin_amdgcn_s_memtime() : 0; };
  const uint64_t k_start = clk();
  for (int64_t c = take(); c < nsup;) {
    const int64_t c_next = take();
    // slice start: a multiple of 64, so every store below is a whole 512 B block
    int64_t pos = um ? umap[2 * c] : c << sh;
    const int64_t S1 = um ? umap[2 * c + 2] : (E - pos < sup ? E : pos + sup);
    if (pos >= S1) {  // a cost-space slice of empty runs only
      c = c_next;
      continue;
    }
    uint64_t t_a = clk();
    if (V & 64) {  // diagnostic: plain fill of the slice (with bit 3: + the skeleton's reads)
      for (int64_t b = pos + lane; b < S1; b += 64) put<V>(times + b, b);
    }
    int64_t jw = um ? umap[2 * c + 1] : chunk_run[c];  // run_off[jw] <= pos
    jend = (um ? umap[2 * c + 3] : chunk_run[c + 1]) + 1;  // the run holding S1 (or the last run)
    load_window(jw);
    if (V & 32) {
      st_win += clk() - t_a;
      n_win++;
    }
    Pending pd;
    pd.blk = -1;
    pd.val = 0;
    int i = 63 - __builtin_clzll(__ballot(woff <= pos));  // the run holding pos
    while (pos < S1) {
      if (i == 64) {  // past the window (the slice's runs continue: jw + 64 < jend)
        jw += 64;
        t_a = clk();
        load_window(jw);
        if (V & 32) {
          st_win += clk() - t_a;
          n_win++;
        }
        i = 0;
      }
      const int32_t cnt = rl32(wcnt, i);
      if (cnt == 0) {
        i++;
        continue;
      }
      const int64_t roff = rl64(woff, i);
      const int64_t p1 = roff + cnt < S1 ? roff + cnt : S1;
      const int64_t b = pos & ~int64_t(63);
      if (kMixedBlocks && !(V & 8) && p1 < b + 64 && p1 < S1) {
        // The run ends inside this block and the slice goes on: the block
        // holds several runs.  Fill it lane-parallel -- each lane finds its
        // run among the window's (largest j with woff[j] <= q) and computes
        // that run's fire -- instead of run by run.  Needs every run up to
        // the block's end in this window.
        const int64_t be = b + 64 < S1 ? b + 64 : S1;
        const int jl = 63 - __builtin_clzll(__ballot(woff <= be - 1));
        if (rl64(woff, jl) + rl32(wcnt, jl) >= be) {
          const int64_t q = b + lane;
          int j = 0;
          for (int st = 32; st; st >>= 1) {
            const int64_t wj = bperm64_w(woff, j + st);
            if (wj <= q) j += st;
          }
          const int64_t rj = bperm64_w(woff, j);
          int64_t v = 0;
          if (q >= pos && q < be) {
            const WinRun& wr = win[j];
            v = run_fire(wr, segs[win_seg(wr)], q - rj);
          } else if (q < pos) {
            v = pd.val;  // earlier runs' fires of this block
          }
          if (be == b + 64) {
            put<V>(times + q, v);
            pd.blk = -1;
            pos = be;
            i = 63 - __builtin_clzll(__ballot(woff <= pos));  // the run holding pos
          } else {  // the slice ends inside the block
            pd.blk = b;
            pd.val = v;
            pos = be;
          }
          continue;
        }
      }
      const WinRun& w = win[i];
      const Segment& sg = segs[win_seg(w)];
      t_a = clk();
      if (V & 8) {
      } else if (win_every(w)) {
        coop_every<V>(w, roff, pos, p1, pd, times);
      } else if (run_is_walked(sg, w.dmask)) {
        drive<V, true>([]() { return int64_t(0); }, []() {}, pos, p1, pd, times);
      } else if (p1 - pos >= 64) {
        coop_cf<V>(w, roff, sg, pos, p1, pd, times);
      } else {
        tiny_cf<V>(w, roff, sg, pos, p1, pd, times);
      }
      if (V & 32) {
        const uint64_t dt = clk() - t_a;
        if (p1 - pos >= 64) {
          st_long += dt;
          n_long++;
        } else {
          st_mix += dt;
          n_mix++;
        }
      }
      pos = p1;
      i++;
    }
    // the last slice ends inside a block
    if (pd.blk >= 0 && pd.blk + lane < S1 && !(V & 8)) put<V>(times + pd.blk + lane, pd.val);
    c = c_next;
  }
  if (V & 32) {
    st_all = clk() - k_start;
    unsigned long long* dbg =
        reinterpret_cast<unsigned long long*>(chunk_run + (cap >> sh) + 2 + kTicketWords);
    if (lane == 0) {
      atomicAdd(dbg + 0, st_all);
      atomicAdd(dbg + 1, st_win);
      atomicAdd(dbg + 2, st_long);
      atomicAdd(dbg + 3, st_mix);
      atomicAdd(dbg + 4, n_win);
      atomicAdd(dbg + 5, n_long);
      atomicAdd(dbg + 6, n_mix);
      atomicAdd(dbg + 7, 1ull);
    }
  }
}

// ---- k_write_lw: the closed-form writer with its loads split off ----------
// On gfx9 a wave's vector loads and stores retire in issue order (one vmcnt),
// so every load a writer wave waits for -- its slice ticket, the slice's run
// window -- also waits for every store it issued before: in k_write_cf each
// slice drains the wave's store queue one to three times.  Here each block
// has kLwWriters writer waves that issue no vector loads and one loader wave
// that issues them all: it takes the tickets, reads the slice map and copies
// each slice's 64-run windows (run offsets, anchors, counts, day masks and
// the runs' rule specs) into one LDS slot per writer with global->LDS DMA
// (no registers; one wait for every writer's copies).  A writer turns its
// slot into its own window (as k_write_cf's) and hands the slot back at once,
// so the next window is copied while it writes.  Writers wait on LDS flags
// only (lgkmcnt): their stores stream without drains.  Every wait is
// bounded: a wave that waits ~2 s (the other side gone) sets an error word
// and leaves, so the grid always drains.
#ifndef CG_LW_WRITERS
#define CG_LW_WRITERS 7
#endif
constexpr int kLwWriters = CG_LW_WRITERS;
#ifndef CG_LW_WPE
#define CG_LW_WPE 4  // waves per SIMD the register allocation must allow
#endif
constexpr uint32_t kLwSpin = 1u << 25;  // polls of ~64 clocks each before giving up

struct LwSlot {  // one window, as copied: structure of arrays
  int64_t off[64];     // run_off
  int64_t anchor[64];  // run_anchor
  int32_t count[64];   // run_count
  uint32_t dmask[64];  // run_dmask
  DSpec spec[65];      // specs of rules jw / G .. (jw + 63) / G
  int64_t c, jw, jend;  // slice (-1: no more slices for this writer), first run, runs end
  int32_t k, nw;        // window k of the slice's nw windows
  int32_t seg0;         // jw % G (the first run's segment; spec[0] is rule jw / G)
};

__device__ __forceinline__ uint32_t lds_flag_get(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_set(uint32_t* f, uint32_t v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads/writes are done
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// global -> LDS copy of `bytes` (a multiple of 4) by the whole wave, 256 B a round
__device__ __forceinline__ void lds_copy(void* lds, const void* g, int bytes) {
  const int lane = threadIdx.x & 63;
  for (int b = 0; b < bytes; b += 256)
    if (b + 4 * lane < bytes)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(g) + b + 4 * lane,
                                       (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(lds) + b),
                                       4, 0, 0);
}

template <int V>
__global__ __launch_bounds__((kLwWriters + 1) * 64) __attribute__((amdgpu_waves_per_eu(CG_LW_WPE)))
void k_write_lw(
    const DSpec* __restrict__ specs, PlanArgs p, const int64_t* __restrict__ run_anchor,
    const int32_t* __restrict__ run_count, const uint32_t* __restrict__ run_dmask,
    const int64_t* __restrict__ run_off, int64_t nruns, int64_t* __restrict__ chunk_run,
    int64_t cap, int64_t* __restrict__ times) {
  __shared__ LwSlot slots[kLwWriters];
  __shared__ WinRun win_all[kLwWriters][64];
  __shared__ uint32_t flags[kLwWriters];  // 1: filled by the loader, 0: free
  extern __shared__ __align__(16) char dyn[];  // the plan's G segments
  Segment* segs = reinterpret_cast<Segment*>(dyn);
  for (int i = threadIdx.x; i < p.G * int(sizeof(Segment) / 8); i += blockDim.x)
    reinterpret_cast<int64_t*>(segs)[i] = reinterpret_cast<const int64_t*>(p.segs)[i];
  for (int i = threadIdx.x; i < kLwWriters; i += blockDim.x) flags[i] = 0u;
  __syncthreads();

  const int G = p.G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t E = run_off[nruns];
  if (E > cap) return;  // output buffer too small: host grows it and relaunches
  const int sh = super_shift(cap);
  const int64_t sup = int64_t(1) << sh;
  const int64_t nsup = (E + sup - 1) >> sh;
  unsigned long long* dbg =
      reinterpret_cast<unsigned long long*>(chunk_run + (cap >> sh) + 2 + kTicketWords);

  if (wave == kLwWriters) {
    // ---- loader.  Lane w < kLwWriters keeps writer w's state, three stages
    // deep: a ticket (the slice after next), the next slice's map entries,
    // and the slice being copied window by window.  Each round issues every
    // stage's loads for every writer at once -- atomics, slice-map reads,
    // window copies -- and waits once.
    const int ng = gridDim.x < kTicketGroups ? int(gridDim.x) : kTicketGroups;
    unsigned int* tickets = reinterpret_cast<unsigned int*>(chunk_run + (cap >> sh) + 2);
    const bool steal = sh == CG_SUPER_SHIFT_LARGE;
    int cur = int(blockIdx.x % unsigned(ng)), hops = 0;
    int64_t c = 0, jw0 = 0, jend = 0;   // the slice being copied
    int32_t k = 0, nw = 0;              // its next window, its windows
    int64_t nc = 0, njw0 = 0, njend = 0;  // the next slice (has_nx)
    int64_t tk = 0;                       // a ticket's slice (has_tk)
    bool has_nx = false, has_tk = false, no_more = false;
    bool fin = lane >= kLwWriters;  // writer `lane` has been sent its end item
    uint32_t idle = 0, idle_total = 0;
    while (__ballot(!fin)) {
      const bool live = !fin;
      const bool ready = live && lds_flag_get(&flags[lane]) == 0u;  // writer's slot free
      if (live && k == nw && has_nx) {  // the next slice becomes current
        c = nc;
        jw0 = njw0;
        jend = njend;
        nw = int32_t((jend - jw0 + 63) >> 6);
        k = 0;
        has_nx = false;
      }
      const bool go = ready && k < nw;
      if (ready && k == nw && !has_nx && no_more) {  // nothing left: the end item
        slots[lane].c = -1;
        lds_flag_set(&flags[lane], 1u);
        fin = true;
      }
      bool busy = go;
      // slice map of the ticket taken last round
      if (live && !has_nx && has_tk) {
        has_tk = false;
        busy = true;
        if (tk < nsup) {
          nc = tk;
          njw0 = chunk_run[tk];           // run_off[njw0] <= tk << sh
          njend = chunk_run[tk + 1] + 1;  // the run holding the slice's end (or the last run)
          has_nx = true;
        } else if (steal && ++hops < ng) {  // this group is used up: move to the next one
          cur = cur + 1 == ng ? 0 : cur + 1;
        } else {
          no_more = true;
        }
      }
      // a ticket, one slice ahead of the slice map
      if (live && !has_tk && !no_more) {
        const unsigned int t = atomicAdd(tickets + cur * kTicketStride, 1u);
        tk = cur + int64_t(ng) * int64_t(t);
        has_tk = true;
        busy = true;
      }
      // window copies, every writer's, then one wait for everything above
      for (uint64_t m = __ballot(go); m; m &= m - 1) {
        const int w = __builtin_ctzll(m);
        const int64_t jw = rl64(jw0, w) + 64 * int64_t(rl32(k, w));
        const int64_t je = rl64(jend, w);
        const int n = int(je - jw < 64 ? je - jw : 64);
        const int64_t r0 = G == 1 ? jw : jw / G, r1 = G == 1 ? jw + n - 1 : (jw + n - 1) / G;
        LwSlot& s = slots[w];
        lds_copy(s.off, run_off + jw, 8 * n);
        lds_copy(s.anchor, run_anchor + jw, 8 * n);
        lds_copy(s.count, run_count + jw, 4 * n);
        lds_copy(s.dmask, run_dmask + jw, 4 * n);
        lds_copy(s.spec, specs + r0, int(sizeof(DSpec)) * int(r1 - r0 + 1));
        if (lane == 0) {
          s.c = rl64(c, w);
          s.jw = jw;
          s.jend = je;
          s.seg0 = int32_t(jw - r0 * G);
          s.k = rl32(k, w);
          s.nw = rl32(nw, w);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // copies, map reads and tickets have landed
      if (go) {
        lds_flag_set(&flags[lane], 1u);
        k++;
      }
      if (!__ballot(busy)) {
        if (++idle > kLwSpin) {
          if (lane == 0) atomicOr(dbg, 1ull);
          break;
        }
        if (V & 32) idle_total++;
        __builtin_amdgcn_s_sleep(1);
      } else {
        idle = 0;
      }
    }
    if ((V & 32) && lane == 0) atomicAdd(dbg + 1, (unsigned long long)idle_total);
    return;
  }

  // ---- writer wave: its slices' windows, in order
  WinRun* win = win_all[wave];
  uint32_t* f = &flags[wave];
  const LwSlot& s = slots[wave];
  Pending pd;
  pd.blk = -1;
  pd.val = 0;
  int64_t pos = 0, S1 = 0;
  uint32_t waits = 0;
  for (;;) {
    for (uint32_t n = 0; lds_flag_get(f) != 1u; n++) {
      if (n > kLwSpin) {
        if (lane == 0) atomicOr(dbg, 2ull);
        return;
      }
      if (V & 32) waits++;
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    const int64_t c = s.c;
    if (c < 0) break;
    const int32_t k = s.k, nw = s.nw;
    const int64_t jw = s.jw, jend = s.jend;
    // the slot -> this wave's window (k_write_cf's layout), then the slot is free
    // lane index re-derived each window: addresses built from it are not
    // hoisted out of the loop (and spilled: scratch reloads wait on vmcnt)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int64_t j = jw + ln;
    int64_t woff = INT64_MAX;
    int32_t wcnt = 0;
    // field by field (a WinRun temporary lands in scratch: vector-memory
    // traffic the writer would wait for behind its stores)
    WinRun& r = win[ln];
    if (j < jend) {
      // run j = rule (jw / G + q), segment x - q G with x = jw % G + lane
      const uint32_t x = uint32_t(s.seg0 + ln);
      uint32_t q = x;
      if (G > 1) {  // x < G + 64 < 2^24: f32 quotient, one correction each way
        const float inv = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(1.0f / float(G))));
        q = uint32_t(float(x) * inv);
        const int32_t rem = int32_t(x) - int32_t(q * uint32_t(G));
        q = rem < 0 ? q - 1u : (rem >= G ? q + 1u : q);
      }
      const DSpec& sp = s.spec[q];
      const uint32_t seg = x - q * uint32_t(G);
      woff = s.off[ln];
      wcnt = s.count[ln];
      r.anchor = s.anchor[ln];
      r.count = wcnt;
      r.dmask = s.dmask[ln];
      r.sp.sec = sp.sec;
      r.sp.min = sp.min;
      r.sp.hour = sp.hour;
      r.sp.dom = sp.dom;
      r.sp.mondow = sp.mondow;
      r.sp.kind = sp.kind | (seg << 8);
    } else {
      r.anchor = 0;
      r.count = 0;
      r.dmask = 0;
      r.sp.sec = 0;
      r.sp.min = 0;
      r.sp.hour = 0;
      r.sp.dom = 0;
      r.sp.mondow = 0;
      r.sp.kind = 0;
    }
    lds_flag_set(f, 0u);  // also waits for this lane's window write
    int i = 0;
    if (k == 0) {
      pos = c << sh;  // multiple of 64: every store below is a whole 512 B block
      S1 = E - pos < sup ? E : pos + sup;
      pd.blk = -1;
      pd.val = 0;
      i = 63 - __builtin_clzll(__ballot(woff <= pos));  // the run holding pos
    }
    while (pos < S1 && i < 64) {
      const int32_t cnt = rl32(wcnt, i);
      if (cnt == 0) {
        i++;
        continue;
      }
      const int64_t roff = rl64(woff, i);
      const int64_t p1 = roff + cnt < S1 ? roff + cnt : S1;
      const WinRun& w = win[i];
      const Segment& sg = segs[win_seg(w)];
      if (V & 8) {
      } else if (win_every(w)) {
        coop_every<V>(w, roff, pos, p1, pd, times);
      } else if (run_is_walked(sg, w.dmask)) {
        drive<V, true>([]() { return int64_t(0); }, []() {}, pos, p1, pd, times);
      } else if (p1 - pos >= 64) {
        coop_cf<V>(w, roff, sg, pos, p1, pd, times);
      } else {
        tiny_cf<V>(w, roff, sg, pos, p1, pd, times);
      }
      pos = p1;
      i++;
    }
    if (k == nw - 1) {
      // the slice ends inside a block
      if (pd.blk >= 0 && pd.blk + lane < S1 && !(V & 8)) put<V>(times + pd.blk + lane, pd.val);
      pd.blk = -1;
    }
    // every lane is done with this window before the next one overwrites it
    __builtin_amdgcn_wave_barrier();
  }
  if ((V & 32) && lane == 0) atomicAdd(dbg + 2, (unsigned long long)waits);
}

// diagnostic store ceiling (CG_WRITE_PROBE): fill the writer's slices of the
// output with W*8-byte-per-lane stores, 64 lanes contiguous
template <int W>
__global__ __launch_bounds__(kWriteWaves * 64) void k_fill_probe(const int64_t* __restrict__ run_off,
                                                                 int64_t nruns, int64_t cap,
                                                                 int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t E = run_off[nruns];
  if (E > cap) return;
  const int64_t kSup = int64_t(1) << super_shift(cap);
  if (W == 6 || W == 7) {  // per-wave streams with a pause (s_sleep) after every 24 stores
    const int64_t nsup = (E + kSup - 1) / kSup;
    const int64_t nwaves = int64_t(gridDim.x) * kWriteWaves;
    for (int64_t c = int64_t(blockIdx.x) * kWriteWaves + wave; c < nsup; c += nwaves) {
      const int64_t p0 = c * kSup, p1 = E - p0 < kSup ? E : p0 + kSup;
      int k = 0;
      for (int64_t b = p0 + lane; b < p1; b += 64) {
        times[b] = b;
        if (++k == 24) {
          k = 0;
          if (W == 6) __builtin_amdgcn_s_sleep(16);
          else __builtin_amdgcn_s_sleep(64);
        }
      }
    }
    return;
  }
  if (W == 4) {  // block-wide streams: the 4 waves interleave 512 B pieces of one slice
    const int64_t nsup = (E + kSup - 1) / kSup;
    for (int64_t c = blockIdx.x; c < nsup; c += gridDim.x) {
      const int64_t p0 = c * kSup, p1 = E - p0 < kSup ? E : p0 + kSup;
      for (int64_t b = p0 + wave * 64 + lane; b < p1; b += 64 * kWriteWaves) times[b] = b;
    }
    return;
  }
  const int64_t nsup = (E + kSup - 1) / kSup;
  const int64_t nwaves = int64_t(gridDim.x) * kWriteWaves;
  for (int64_t c = int64_t(blockIdx.x) * kWriteWaves + wave; c < nsup; c += nwaves) {
    const int64_t p0 = c * kSup + (W == 3 ? 8 : 0), p1 = E - c * kSup < kSup ? E : c * kSup + kSup;
    for (int64_t b = p0 + lane * (W == 3 ? 1 : W); b < p1; b += 64 * (W == 3 ? 1 : W)) {
      if (W == 2 && b + 1 < p1) {
        longlong2 v;
        v.x = b;
        v.y = b + 1;
        *reinterpret_cast<longlong2*>(times + b) = v;
      } else {
        times[b] = b;
      }
    }
  }
}

#ifndef CG_WALK_WPE
#define CG_WALK_WPE 5  // register budget of k_write_walk: 5 waves per SIMD (98 -> 96 VGPRs, 12 B spill; 0.41 -> 0.37 ms on a DST day)
#endif
__global__ __launch_bounds__(256)
#if CG_WALK_WPE
__attribute__((amdgpu_waves_per_eu(CG_WALK_WPE)))
#endif
void k_write_walk(const DSpec* __restrict__ specs, int64_t R,
                                                     PlanArgs p,
                                                     const int64_t* __restrict__ run_anchor,
                                                     const int32_t* __restrict__ run_count,
                                                     const uint32_t* __restrict__ run_dmask,
                                                     const int64_t* __restrict__ run_off,
                                                     int64_t cap, int64_t* __restrict__ times) {
  extern __shared__ __align__(16) char lds[];
  PlanView v = stage_plan(p, lds);
  const int G = p.G;
  if (run_off[int64_t(R) * G] > cap) return;
  for (int64_t r = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; r < R;
       r += int64_t(gridDim.x) * blockDim.x) {
    DSpec sp;
    bool loaded = false;
    for (int s = 0; s < G; s++) {
      const int64_t j = r * G + s;
      int32_t n = run_count[j];
      if (n == 0 || !run_is_walked(v.segs[s], run_dmask[j])) continue;
      if (!loaded) {
        sp = load_spec(specs + r);
        loaded = true;
      }
      if (sp.kind == KIND_EVERY) break;
      int64_t t = run_anchor[j];
      int64_t o = run_off[j];
      for (int32_t q = 0; q < n; q++) {
        t = next_exact(sp, v.z, t, p.t1);
        times[o + q] = t;
      }
    }
  }
}

// Order-sensitive checksum of a device array: sum over i of
// mix(first + i, v[i] + add) mod 2^64 (splitmix64 finaliser), so checksums of
// consecutive ranges add up and a shard's output can be compared with its
// range of an unsharded result without moving either.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

template <class T>
__global__ __launch_bounds__(256) void k_checksum(const T* __restrict__ v, int64_t n, int64_t first,
                                                   int64_t add, unsigned long long* __restrict__ out) {
  uint64_t acc = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t x = uint64_t(int64_t(v[i]) + add);
    acc += mix64(x ^ mix64(uint64_t(first + i) * 0x9E3779B97F4A7C15ull));
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __shared__ uint64_t s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(s[0] + s[1] + s[2] + s[3]));
}

// *out += number of elements of v equal to x (cg_count_value_device)
template <class T>
__global__ __launch_bounds__(256) void k_count_eq(const T* __restrict__ v, int64_t n, T x,
                                                   unsigned long long* __restrict__ out) {
  uint64_t c = 0;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    c += v[i] == x;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ uint64_t s[4];
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, (unsigned long long)(s[0] + s[1] + s[2] + s[3]));
}

int grid_for(int64_t n, int threads, int max_blocks) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  return int(b < max_blocks ? b : max_blocks);
}

}  // namespace

size_t plan_lds_bytes(const PlanArgs& p) {
  return align_up(size_t(p.zn) * 8, 16) + align_up(size_t(p.zn) * 4, 16) +
         align_up(size_t(p.G) * sizeof(Segment), 16) +
         (p.dtab_global ? 0 : align_up(size_t(p.nd) * 4, 16));
}

void launch_checksum(const void* v, int64_t n, int elem_bytes, int64_t first, int64_t add,
                     unsigned long long* out, hipStream_t st) {
  if (n <= 0) return;
  const int grid = grid_for(n, 256 * 8, 256 * 32);
  if (elem_bytes == 8)
    hipLaunchKernelGGL(k_checksum<int64_t>, dim3(grid), dim3(256), 0, st,
                       static_cast<const int64_t*>(v), n, first, add, out);
  else
    hipLaunchKernelGGL(k_checksum<int32_t>, dim3(grid), dim3(256), 0, st,
                       static_cast<const int32_t*>(v), n, first, add, out);
}

void launch_count_eq(const void* v, int64_t n, int elem_bytes, int64_t x, unsigned long long* out,
                     hipStream_t st) {
  if (n <= 0) return;
  const int grid = grid_for(n, 256 * 8, 256 * 32);
  if (elem_bytes == 8)
    hipLaunchKernelGGL(k_count_eq<int64_t>, dim3(grid), dim3(256), 0, st, static_cast<const int64_t*>(v), n, x,
                       out);
  else
    hipLaunchKernelGGL(k_count_eq<int32_t>, dim3(grid), dim3(256), 0, st, static_cast<const int32_t*>(v), n,
                       int32_t(x), out);
}

void launch_next_batch(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* t_in,
                       int64_t* t_out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_next_batch, dim3(grid_for(n, 256, 256 * 16)), dim3(256),
                     plan_lds_bytes(p), st, specs, n, p, t_in, t_out);
}

void launch_lock_ttl(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* now,
                     const int32_t* kind, const int64_t* avg_ms, int64_t lock_ttl, int64_t* ttl,
                     hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_lock_ttl, dim3(grid_for(n, 256, 256 * 16)), dim3(256), plan_lds_bytes(p),
                     st, specs, n, p, now, kind, avg_ms, lock_ttl, ttl);
}

void launch_dispatch_scan(const int64_t* next, int64_t n, int64_t effective,
                          unsigned long long* due_bits, uint32_t* tile_cnt,
                          unsigned long long* tile_min, hipStream_t s) {
  if (n <= 0) return;
  const int64_t tiles = (n + kDispatchTile - 1) / kDispatchTile;
  hipLaunchKernelGGL(k_dispatch_scan, dim3(unsigned(tiles)), dim3(256), 0, s, next, n, effective,
                     due_bits, tile_cnt, tile_min);
}

void launch_dispatch_advance(const DSpec* specs, const int32_t* due, int64_t n, const PlanArgs& p,
                             int64_t now, int64_t* next, int64_t* prev, DispatchState* st,
                             hipStream_t s) {
  if (n <= 0) return;
  // sized for the largest possible due list; blocks past the device-side
  // count exit before staging the zone table
  hipLaunchKernelGGL(k_dispatch_advance, dim3(grid_for(n, 256, 4096)), dim3(256),
                     plan_lds_bytes(p), s, specs, due, p, now, next, prev, st);
}

void launch_dispatch_compact(const unsigned long long* due_bits, const uint32_t* tile_cnt,
                             const unsigned long long* tile_min, int64_t n, int32_t* due,
                             DispatchState* st, hipStream_t s) {
  if (n <= 0) return;
  const int64_t tiles = (n + kDispatchTile - 1) / kDispatchTile;
  hipLaunchKernelGGL(k_dispatch_compact, dim3(unsigned(tiles)), dim3(256), 0, s, due_bits, tile_cnt,
                     tile_min, n, due, st);
}

void launch_dispatch_place(DSpec* specs, const int64_t* idx, const DSpec* src, int64_t first,
                           int64_t k, const PlanArgs& p, int64_t now, int64_t* next, int64_t* prev,
                           DispatchState* st, hipStream_t s) {
  if (k <= 0) return;
  hipLaunchKernelGGL(k_dispatch_place, dim3(grid_for(k, 256, 256 * 16)), dim3(256), plan_lds_bytes(p),
                     s, specs, idx, src, first, k, p, now, next, prev, st);
}

void launch_dispatch_clear(const int64_t* idx, int64_t first, int64_t k, int64_t* next, int64_t* prev,
                           hipStream_t s) {
  if (k <= 0) return;
  hipLaunchKernelGGL(k_dispatch_clear, dim3(grid_for(k, 256, 4096)), dim3(256), 0, s, idx, first, k,
                     next, prev);
}

void launch_dispatch_min(const int64_t* next, int64_t n, DispatchState* st, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_dispatch_min, dim3(grid_for(n, 256 * 8, 1024)), dim3(256), 0, s, next, n, st);
}

#ifndef CG_COUNT_MAX_BLOCKS
#define CG_COUNT_MAX_BLOCKS 4096  // k_count grid cap (rules beyond it loop grid-stride)
#endif
void launch_count(const DSpec* specs, int64_t R, const PlanArgs& p, int64_t* run_anchor,
                  int32_t* run_count, uint32_t* run_dmask, unsigned long long* stuck_rule,
                  hipStream_t st) {
  if (R <= 0) return;
  // the plan's walked parts (flags: WALK segments, an exact Next from T0, a
  // final walk); without them k_count needs no exact walk
  if (p.flags != 0)
    hipLaunchKernelGGL(k_count<true>, dim3(grid_for(R, 256, CG_COUNT_MAX_BLOCKS)), dim3(256), plan_lds_bytes(p), st,
                       specs, R, p, run_anchor, run_count, run_dmask, stuck_rule);
  else
    hipLaunchKernelGGL(k_count<false>, dim3(grid_for(R, 256, CG_COUNT_MAX_BLOCKS)), dim3(256), plan_lds_bytes(p),
                       st, specs, R, p, run_anchor, run_count, run_dmask, stuck_rule);
}

size_t scan_temp_bytes(int64_t n) {
  int64_t nb = (n + kScanTile - 1) / kScanTile;
  return size_t(nb + 1) * sizeof(int64_t);
}

template <class T>
static void scan_impl(const T* in, int64_t* out, int64_t n, void* temp, RunTail tail, hipStream_t st) {
  int64_t nb = (n + kScanTile - 1) / kScanTile;
  int64_t* partial = static_cast<int64_t*>(temp);
  hipLaunchKernelGGL(k_scan_reduce<T>, dim3(nb), dim3(kScanThreads), 0, st, in, n, partial);
  if (nb <= kScanFuseTiles) {
    hipLaunchKernelGGL((k_scan_apply<T, true>), dim3(nb), dim3(kScanThreads), 0, st, in, n, partial, out,
                       tail);
    return;
  }
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanThreads), 0, st, partial, nb);
  hipLaunchKernelGGL((k_scan_apply<T, false>), dim3(nb), dim3(kScanThreads), 0, st, in, n, partial, out,
                     tail);
}

void launch_scan(const int32_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st) {
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int64_t), st);
    return;
  }
  scan_impl(in, out, n, temp, RunTail{nullptr, nullptr, nullptr, 1, nullptr, 0}, st);
}

void launch_scan64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st) {
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int64_t), st);
    return;
  }
  scan_impl(in, out, n, temp, RunTail{nullptr, nullptr, nullptr, 1, nullptr, 0}, st);
}

void launch_scan_runs(const int32_t* run_count, int64_t* run_off, int64_t R, int32_t G, void* temp,
                      int64_t* offsets, int64_t* res, unsigned long long* stuck,
                      int64_t* chunk_run, int64_t cap, hipStream_t st) {
  scan_impl(run_count, run_off, R * G, temp, RunTail{offsets, res, stuck, G, chunk_run, cap}, st);
  if (chunk_run) launch_chunk_map_u(run_off, R * G, cap, chunk_run, st);
}

void launch_chunk_map_u(const int64_t* run_off, int64_t nruns, int64_t cap, int64_t* chunk_run,
                        hipStream_t st) {
  if (nruns <= 0) return;
  hipLaunchKernelGGL(k_chunk_map_u, dim3(unsigned((kUSlices + 1 + 255) / 256)), dim3(256), 0, st, run_off,
                     nruns, cap, chunk_run);
}

void launch_chunk_map(const int64_t* run_off, int64_t nruns, int64_t cap, int64_t* chunk_run,
                      hipStream_t st) {
  int64_t max_sup = (cap >> super_shift(cap)) + 1;
  hipLaunchKernelGGL(k_chunk_map, dim3(grid_for(max_sup + 1, 256, 4096)), dim3(256), 0, st,
                     run_off, nruns, cap, chunk_run);
  launch_chunk_map_u(run_off, nruns, cap, chunk_run, st);
}

void launch_write_cf(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor,
                     const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                     int64_t nruns, int64_t* chunk_run, int64_t cap, int64_t* times,
                     int n_blocks, hipStream_t st) {
  const size_t lds = size_t(p.G) * sizeof(Segment);
#ifndef CG_DIAG
  // production build: the writer, nothing else (the probes and store-dropping
  // variants below exist only in the diagnostic library, `make diag`)
#if CG_WRITE_LOADER
  // persistent k_write_lw grid: as many blocks per CU as its registers and
  // LDS (slots + the plan's segments) let run at once
  static int lw_per_cu[2] = {0, 0};  // by whether the segments fit the small-LDS case
  const int key = lds <= 4096 ? 0 : 1;
  if (!lw_per_cu[key]) {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_write_lw<0>, (kLwWriters + 1) * 64,
                                                     key ? kMaxSegments * sizeof(Segment) : 4096) != hipSuccess ||
        n < 1)
      n = 1;
    lw_per_cu[key] = n;
  }
  const int cus = std::max(1, n_blocks / kWriteBlocksPerCU);
  hipLaunchKernelGGL(k_write_lw<0>, dim3(cus * lw_per_cu[key]), dim3((kLwWriters + 1) * 64), lds, st, specs,
                     p, run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
#else
  // CG_WRITE_SPARE_BLOCKS block slots left to the next pipelined call's
  // count and scan (they run beside the persistent writer instead of after it)
  const int nb = std::max(1, n_blocks - CG_WRITE_SPARE_BLOCKS);
  hipLaunchKernelGGL(k_write_cf<0>, dim3(nb), dim3(kWriteWaves * 64), lds, st, specs, p,
                     run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
#endif
#else
  // CG_WRITE_PROBE (diagnostic build only): replace the
  // writer by a plain fill of the same E*8 output bytes, same grid and slices,
  // with 8 B (1) or 16 B (2) per lane per store -- the store ceiling the
  // writer is compared against.
  static const int probe = [] {
    const char* e = getenv("CG_WRITE_PROBE");
    return e ? atoi(e) : 0;
  }();
  if (probe == 1) {
    hipLaunchKernelGGL(k_fill_probe<1>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  if (probe == 4) {
    hipLaunchKernelGGL(k_fill_probe<4>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  if (probe == 6) {
    hipLaunchKernelGGL(k_fill_probe<6>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  if (probe == 7) {
    hipLaunchKernelGGL(k_fill_probe<7>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  if (probe == 5) {  // hipMemsetAsync of the capacity (>= the E*8 bytes)
    (void)hipMemsetAsync(times, 0, size_t(cap) * 8, st);
    return;
  }
  if (probe == 3) {  // 8 B per lane, every store instruction 64 B off a 512 B boundary
    hipLaunchKernelGGL(k_fill_probe<3>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  if (probe == 2) {
    hipLaunchKernelGGL(k_fill_probe<2>, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, run_off,
                       nruns, cap, times);
    return;
  }
  static const int variant = [] {
    const char* e = getenv("CG_WRITE_VARIANT");  // diagnostic only (see put<V>)
    return e ? atoi(e) : 0;
  }();
#define CG_WCF(V)                                                                             \
  hipLaunchKernelGGL(k_write_cf<V>, dim3(n_blocks), dim3(kWriteWaves * 64), lds, st, specs, p, \
                     run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times)
  if (variant == 256) {  // k_write_lw with wait counters
    int n = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_write_lw<32>, (kLwWriters + 1) * 64, lds);
    const int blocks = std::max(1, n_blocks / kWriteBlocksPerCU) * std::max(n, 1);
    hipLaunchKernelGGL(k_write_lw<32>, dim3(blocks), dim3((kLwWriters + 1) * 64), lds, st, specs, p,
                       run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
    unsigned long long d[8];
    (void)hipMemcpyAsync(d, chunk_run + (cap >> super_shift(cap)) + 2 + kTicketWords, sizeof d,
                         hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    fprintf(stderr, "[k_write_lw stats] blocks=%d err=%llu loader idle rounds=%llu writer waits=%llu\n", blocks,
            d[0], d[1], d[2]);
    return;
  }
  switch (variant) {
    case 1: CG_WCF(1); break;
    case 2: CG_WCF(2); break;
    case 4: CG_WCF(4); break;
    case 8: CG_WCF(8); break;
    case 12: CG_WCF(12); break;
    case 16: CG_WCF(16); break;
    case 32: CG_WCF(32); break;
    case 76: CG_WCF(76); break;
    case 128: CG_WCF(128); break;
    default: CG_WCF(0); break;
  }
#undef CG_WCF
  if (variant & 32) {
    unsigned long long d[8];
    (void)hipMemcpyAsync(d, chunk_run + (cap >> super_shift(cap)) + 2 + kTicketWords, sizeof d,
                         hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    fprintf(stderr,
            "[k_write_cf stats] waves=%llu cycles/wave: all=%.0f window=%.0f coop=%.0f tiny=%.0f | "
            "per wave: windows=%.1f coop_pieces=%.1f tiny_pieces=%.1f\n",
            d[7], double(d[0]) / d[7], double(d[1]) / d[7], double(d[2]) / d[7], double(d[3]) / d[7],
            double(d[4]) / d[7], double(d[5]) / d[7], double(d[6]) / d[7]);
  }
#endif  // CG_DIAG
}

void launch_write_walk(const DSpec* specs, int64_t R, const PlanArgs& p, const int64_t* run_anchor,
                       const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                       int64_t cap, int64_t* times, hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_write_walk, dim3(grid_for(R, 256, 256 * 16)), dim3(256),
                     plan_lds_bytes(p), st, specs, R, p, run_anchor, run_count, run_dmask, run_off,
                     cap, times);
}


}  // namespace cg
