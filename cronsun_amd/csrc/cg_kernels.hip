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
#include "cg_kernels.h"
#include "cg_write.h"

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


// The second launch bound is the minimum waves per SIMD (HIP/AMDGPU: it caps
// the VGPRs).  The grid runs 3 waves per SIMD; a bound of 6 caps the writer at
// 80 VGPRs (148 B/lane of spills) and is the fastest measured: k_write_cf
// 0.978-0.985 ms vs 1.004-1.019 at the grid's own 3 (122 VGPRs, no spills),
// 0.985-0.991 at 5 (96 VGPRs), 1.027-1.029 at 8 (64 VGPRs), two boxes
// (profiles/r04_ab_writer_regcap.txt).  The spills hold per-slice state that
// the inner block loops do not touch; the tighter allocation changes where
// the compiler puts the waits of the window and spec loads.
#ifndef CG_WRITE_WPE
#define CG_WRITE_WPE 6
#endif
// Ticket groups across the XCDs (1) or one XCD per group (0: blocks go
// round-robin over the XCDs, so group blockIdx % 32 lived on XCD
// blockIdx % 8).  With one XCD per group the groups ran dry up to 120 us
// apart on config 2 (the XCDs' rates differ), and a dry group's waves idled:
// 5-9 % of the wave-time (per-wave stamps, profiles/r06_writer_tail_*.json).
// Across the XCDs: dry within 40 us, idle 3.3 %, k_write_cf 0.980 -> 0.946 ms
// (same box, profiles/r06_ab_writer_groups.txt; moving on to other groups
// when dry, CG_WRITE_STEAL_SMALL, gains nothing on top).
#ifndef CG_WRITE_GROUPS_SMALL
#define CG_WRITE_GROUPS_SMALL 8
#endif
constexpr int kWriteGroupsSmall = CG_WRITE_GROUPS_SMALL < kTicketGroups ? CG_WRITE_GROUPS_SMALL : kTicketGroups;
#ifndef CG_WRITE_GRP_XCD
#define CG_WRITE_GRP_XCD 1
#endif
#ifndef CG_WRITE_STEAL_SMALL
#define CG_WRITE_STEAL_SMALL 0
#endif
#ifdef CG_DIAG
// diagnostic build only (CG_WRITE_STAMPS=1): per wave of the last k_write_cf
// launch {start, end, slices written, the wall clock when its ticket group
// ran dry}, wall_clock64() units (100 MHz) -- the launch's ramp and tail
__device__ int64_t* cg_write_stamps = nullptr;
#endif
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
__global__ __launch_bounds__(kWriteWaves * 64, CG_WRITE_WPE) void k_write_cf(
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
#ifdef CG_DIAG
  int64_t* const stamp = cg_write_stamps ? cg_write_stamps + 4 * (int64_t(blockIdx.x) * kWriteWaves + wave) : nullptr;
  const int64_t st_start = stamp ? int64_t(wall_clock64()) : 0;
  int64_t st_slices = 0;
#endif
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
  // 8 ticket groups for small slices, 32 for large ones (same-box A/B,
  // profiles/r06_ab_ticket_groups.txt and r06_ab_ticket_groups_pn.txt: config 2
  // writer 0.957 -> 0.941 ms with 8 instead of 32; config 4's large slices,
  // which move on to other groups, 26.0 -> 26.6 ms with 8).  Fewer groups of
  // more blocks each progress at closer rates, so they run dry closer together.
  const int groups = sh == CG_SUPER_SHIFT_LARGE ? kTicketGroups : kWriteGroupsSmall;
  const int ng = int(gridDim.x) < groups ? int(gridDim.x) : groups;
#if CG_WRITE_GRP_XCD
  // every group spans the 8 XCDs (blocks b..b+7 of one dispatch round share a
  // group): a group's slices then advance at the chip's average rate
  // (only when the grid gives every group a block that way)
  const int grp = int(gridDim.x >= 8u * unsigned(ng) ? (blockIdx.x >> 3) % unsigned(ng) : blockIdx.x % unsigned(ng));
#else
  const int grp = int(blockIdx.x % unsigned(ng));
#endif
  unsigned int* tickets = reinterpret_cast<unsigned int*>(chunk_run + (cap >> sh) + 2);
  int cur = grp, hops = 0;  // the group whose slices this wave takes, groups left behind
  // (same-box A/B, profiles/r02_ab_steal.json: config 4 with 16384-event
  // slices 23.7 vs 24.5 ms; config 2 with 2048-event slices 1.03 vs 0.99 ms:
  // moving on only pays with the large slices)
  const bool steal = CG_WRITE_STEAL_SMALL || sh == CG_SUPER_SHIFT_LARGE;
  // One ticket per atomic (same-box A/B, profiles/r02_ab_writer_lw.json:
  // taking 2/4/8 per atomic loses more to the coarser tail than it saves).
  auto take = [&]() -> int64_t {
    for (;;) {
      unsigned int t = 0;
      if (lane == 0) t = atomicAdd(tickets + cur * kTicketStride, 1u);
      const int64_t c = cur + int64_t(ng) * int64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(t))));
      if (c < nsup || !steal || ++hops >= ng) return c;
      cur = cur + 1 == ng ? 0 : cur + 1;
    }
  };
  for (int64_t c = take(); c < nsup;) {
    const int64_t c_next = take();
#ifdef CG_DIAG
    st_slices++;
    if (stamp && c_next >= nsup && lane == 0) stamp[3] = int64_t(wall_clock64());
#endif
    // slice start: a multiple of 64, so every store below is a whole 512 B block
    int64_t pos = um ? umap[2 * c] : c << sh;
    const int64_t S1 = um ? umap[2 * c + 2] : (E - pos < sup ? E : pos + sup);
    if (pos >= S1) {  // a cost-space slice of empty runs only
      c = c_next;
      continue;
    }
    int64_t jw = um ? umap[2 * c + 1] : chunk_run[c];  // run_off[jw] <= pos
    jend = (um ? umap[2 * c + 3] : chunk_run[c + 1]) + 1;  // the run holding S1 (or the last run)
    load_window(jw);
    Pending pd;
    pd.blk = -1;
    pd.val = 0;
    int i = 63 - __builtin_clzll(__ballot(woff <= pos));  // the run holding pos
    while (pos < S1) {
      if (i == 64) {  // past the window (the slice's runs continue: jw + 64 < jend)
        jw += 64;
        load_window(jw);
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
      if (p1 < b + 64 && p1 < S1) {
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
            put(times + q, v);
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
      if (win_every(w)) {
        coop_every(w, roff, pos, p1, pd, times);
      } else if (run_is_walked(sg, w.dmask)) {
        drive<true>([]() { return int64_t(0); }, []() {}, pos, p1, pd, times);
      } else if (p1 - pos >= 64) {
        coop_cf(w, roff, sg, pos, p1, pd, times);
      } else {
        tiny_cf(w, roff, sg, pos, p1, pd, times);
      }
      pos = p1;
      i++;
    }
    // the last slice ends inside a block
    if (pd.blk >= 0 && pd.blk + lane < S1) put(times + pd.blk + lane, pd.val);
    c = c_next;
  }
#ifdef CG_DIAG
  if (stamp && lane == 0) {
    stamp[0] = st_start;
    stamp[1] = int64_t(wall_clock64());
    stamp[2] = st_slices;
  }
#endif
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

// Store ceiling (cg_fill_rate_device): every lane writes 16 B per store, a
// wave 1 KB of consecutive bytes, four stores in flight per lane per round;
// the grid strides over the whole buffer.  No loads: nothing ever drains.
typedef int v4i32 __attribute__((ext_vector_type(4)));
template <bool kNT>
__global__ __launch_bounds__(256) void k_fill_stream(v4i32* __restrict__ p, int64_t n16) {
  const int64_t stride = int64_t(gridDim.x) * blockDim.x;
  int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const v4i32 v = {int(0x5EED0000u), 0x5EED, int(0x5EED0000u), 0x5EED};
  for (; i + 3 * stride < n16; i += 4 * stride) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      if (kNT) __builtin_nontemporal_store(v, p + i + u * stride);
      else p[i + u * stride] = v;
    }
  }
  for (; i < n16; i += stride) {
    if (kNT) __builtin_nontemporal_store(v, p + i);
    else p[i] = v;
  }
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

void launch_fill_stream(void* p, int64_t n16, int nt, hipStream_t st) {
  if (n16 <= 0) return;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  // one 4-wave block per CU: the fastest plain streaming fill on this part
  // (profiles/r03_fill_patterns_box*.jsonl: 6.3-6.5 TB/s, the rate of
  // hipMemsetAsync; 2-8 blocks per CU 5.2-5.7 TB/s)
  const int grid = grid_for((n16 + 3) / 4, 256, cus);
  if (nt)
    hipLaunchKernelGGL(k_fill_stream<true>, dim3(grid), dim3(256), 0, st, static_cast<v4i32*>(p), n16);
  else
    hipLaunchKernelGGL(k_fill_stream<false>, dim3(grid), dim3(256), 0, st, static_cast<v4i32*>(p), n16);
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

#ifdef CG_DIAG
int64_t* g_stamp_buf = nullptr;
int g_stamp_waves = 0;
#endif

void launch_write_cf(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor,
                     const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                     int64_t nruns, int64_t* chunk_run, int64_t cap, int64_t* times,
                     int n_blocks, hipStream_t st) {
  const size_t lds = size_t(p.G) * sizeof(Segment);
#ifdef CG_DIAG
  static const bool stamps = getenv("CG_WRITE_STAMPS") != nullptr;
  if (stamps) {  // the per-wave stamps of this launch (read by cg_diag_write_stamps)
    static int64_t* buf = nullptr;
    static int cap_waves = 0;
    const int waves = n_blocks * kWriteWaves;
    if (waves > cap_waves) {
      if (buf) (void)hipFree(buf);
      (void)hipMalloc(&buf, size_t(waves) * 32);
      cap_waves = waves;
      (void)hipMemcpyToSymbol(HIP_SYMBOL(cg_write_stamps), &buf, sizeof buf);
    }
    (void)hipMemsetAsync(buf, 0, size_t(waves) * 32, st);
    g_stamp_buf = buf;
    g_stamp_waves = waves;
  }
  // the diagnostic library only (`make diag`): store-ceiling probes and the
  // experimental loader/writer split replace the writer when asked for
  // (CG_WRITE_PROBE / CG_WRITE_VARIANT, cg_diag.hip)
  if (launch_write_diag(specs, p, run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times, n_blocks,
                        lds, st))
    return;
#endif
  hipLaunchKernelGGL(k_write_cf, dim3(n_blocks), dim3(kWriteWaves * 64), lds, st, specs, p, run_anchor, run_count,
                     run_dmask, run_off, nruns, chunk_run, cap, times);
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

#ifdef CG_DIAG
// the diagnostic library's per-wave stamps of the last k_write_cf launch
// (CG_WRITE_STAMPS=1): 4 int64 per wave {start, end, slices, dry}; returns the
// number of waves (0 when stamps are off), after a device sync
extern "C" int cg_diag_write_stamps(int64_t* out, int64_t max_waves) {
  if (!cg::g_stamp_buf) return 0;
  (void)hipDeviceSynchronize();
  const int64_t n = std::min<int64_t>(cg::g_stamp_waves, max_waves);
  (void)hipMemcpy(out, cg::g_stamp_buf, size_t(n) * 32, hipMemcpyDeviceToHost);
  return int(n);
}
#endif
