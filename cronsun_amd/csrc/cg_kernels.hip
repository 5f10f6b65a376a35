// cg_kernels.hip -- gfx950 kernels for batched cron fire-time expansion.
//
// Pipeline for Expand(specs, zone, T0, T1):
//   k_count      one lane per rule: per plan segment, the first fire (exact
//                Go walk, next_exact) and the closed-form count of the rest,
//                or the walked count inside WALK windows -> run records
//   k_scan_*     exclusive scan of run counts -> run offsets (int64)
//   k_chunk_map  first run touched by each 16384-event output slice
//   k_write_cf   persistent, output-parallel: each wave walks its slices;
//                long runs are written wave-cooperatively (64 consecutive
//                fires per store instruction, mixed-radix digits + lane rank
//                tables), stretches of short runs lane-parallel via LDS staging
//   k_write_walk re-walks the (rare) WALK-window runs
//   k_rule_offs  rule-major CSR offsets
// Integer and HBM-bound throughout: no MFMA.
#include <hip/hip_runtime.h>

#include "cg_expand.h"
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
  for (int i = threadIdx.x; i < p.nd; i += blockDim.x) d[i] = p.dtab[i];
  __syncthreads();
  PlanView v;
  v.z.when = w;
  v.z.off = o;
  v.z.n = p.zn;
  v.segs = s;
  v.dtab = d;
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

__global__ __launch_bounds__(256) void k_count(const DSpec* __restrict__ specs, int64_t R,
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
    if (!count_rule(sp, v.z, v.segs, G, v.dtab, p.t0, p.t1, run_anchor + j0, run_count + j0,
                    run_dmask + j0))
      atomicMin(stuck_rule, (unsigned long long)r);
  }
}

// ---- scan: int32 counts -> int64 exclusive offsets -----------------------
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 16;
constexpr int kScanTile = kScanThreads * kScanPerThread;

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

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const int32_t* __restrict__ in,
                                                               int64_t n,
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

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const int32_t* __restrict__ in,
                                                              int64_t n,
                                                              const int64_t* __restrict__ partial,
                                                              int64_t* __restrict__ out) {
  int64_t base = int64_t(blockIdx.x) * kScanTile + int64_t(threadIdx.x) * kScanPerThread;
  int32_t v[kScanPerThread];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    int64_t idx = base + i;
    v[i] = idx < n ? in[idx] : 0;
    acc += v[i];
  }
  int64_t tot;
  int64_t run = partial[blockIdx.x] + block_excl_scan(acc, &tot);
  if (blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; i++) {
    int64_t idx = base + i;
    run += v[i];
    if (idx < n) out[idx + 1] = run;
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

// first run touched by each kSuper-event output slice; E is read on the device
// so the launch needs no host sync (grid sized by capacity, extra threads exit)
__global__ void k_chunk_map(const int64_t* __restrict__ run_off, int64_t nruns, int64_t cap,
                            int64_t* __restrict__ chunk_run) {
  const int64_t E = run_off[nruns];
  if (E > cap) return;  // chunk_run holds cap / kSuper + 2 entries
  const int64_t nsup = (E + kSuper - 1) / kSuper;
  for (int64_t c = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; c <= nsup;
       c += int64_t(gridDim.x) * blockDim.x)
    chunk_run[c] = c == nsup ? nruns - 1 : search_run(run_off, 0, nruns - 1, c * int64_t(kSuper));
}

constexpr int kStageStride = kLaneEvents + 1;  // pad: conflict-free ds_write_b64 / ds_read_b64
// run pieces at least this long are written wave-cooperatively
constexpr int64_t kCoopMin = 64;

// one run of a wave's 64-run window (lane i holds run jw + i), staged in LDS
struct WinRun {
  int64_t off;     // run_off[j]
  int64_t anchor;  // run_anchor[j]
  DSpec sp;        // specs[j / G]
  int32_t count;   // run_count[j]
  uint32_t dmask;  // run_dmask[j]
  int32_t seg;     // j % G
  int32_t pad;
};

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

// Fires [p0, p1) of closed-form run w, wave-cooperatively: lane l writes
// p0 + l + 64u.  A fire's index g = rank(anchor) - 1 + (p - run start) counts
// (day, hour, minute, second) combinations from the anchor's local day, so it
// is carried as mixed-radix digits (matching-day rank, hour/minute/second
// ranks; radices -, nH, nM, nS) and stepped by the constant 64; rank -> seconds
// comes from per-run lane tables.  Same enumeration as cf_seek/cf_next.
__device__ void coop_cf(const WinRun& w, const Segment& sg, int64_t p0, int64_t p1,
                        int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63;
  const CFRule c = cf_rule(w.sp);
  const uint32_t nS = c.nS, nM = c.nM, nH = c.C / c.nMS;
  const uint32_t rf = uint32_t(w.anchor - sg.base);
  const uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  const int32_t ts = rank_table(c.S, 1);
  const int32_t tm = rank_table(c.M, 60);
  const int32_t th = rank_table(c.H, 3600);
  const int32_t td = rank_table(uint64_t(w.dmask >> jf), 86400) + int32_t(jf) * 86400;
  uint32_t g = cf_rank(c, int32_t(tf)) - 1u + uint32_t(p0 - w.off);
  uint32_t d = g / c.C;
  g -= d * c.C;
  uint32_t h = g / c.nMS;
  g -= h * c.nMS;
  uint32_t m = g / nS;
  uint32_t s = g - m * nS;
  // + lane
  const float iS = 1.0f / float(nS), iM = 1.0f / float(nM), iH = 1.0f / float(nH);
  uint32_t q;
  s += uint32_t(lane);
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
  uint32_t a = 64;
  const uint32_t a0 = a % nS;
  a /= nS;
  const uint32_t a1 = a % nM;
  a /= nM;
  const uint32_t a2 = a % nH;
  const uint32_t a3 = a / nH;
  const int64_t base = sg.base;
  auto value = [&]() -> int64_t {
    return base + int64_t(rank_at(td, d) + rank_at(th, h) + rank_at(tm, m) + rank_at(ts, s));
  };
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
  int64_t* out = times + p0 + lane;
  const int64_t n = p1 - p0;
  int64_t b = 0;
  for (; b + 8 * 64 <= n; b += 8 * 64) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      out[b + 64 * u] = value();
      step();
    }
  }
  for (; b < n; b += 64) {
    const int64_t v = value();  // all lanes: the table reads are cross-lane
    if (b + lane < n) out[b] = v;
    step();
  }
}

// Fires [p0, p1) of @every run w: anchor + (k + 1) * D (constantdelay.go:25-27)
__device__ void coop_every(const WinRun& w, int64_t p0, int64_t p1, int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63;
  const int64_t D = int64_t(w.sp.sec);
  int64_t t = w.anchor + (p0 - w.off + lane + 1) * D;
  const int64_t st = 64 * D;
  int64_t* out = times + p0 + lane;
  const int64_t n = p1 - p0;
  int64_t b = 0;
  for (; b + 8 * 64 <= n; b += 8 * 64) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      out[b + 64 * u] = t;
      t += st;
    }
  }
  for (; b < n; b += 64) {
    if (b + lane < n) out[b] = t;
    t += st;
  }
}

// Fires [pos, rend) spread over many short runs of the window (all inside it):
// per kChunk piece lane l materialises events [8l, 8l+8) (seek once, then the
// branch-free iterator), stages them in LDS, and the wave stores the piece
// with coalesced 512 B wave-instructions.  Walked runs get placeholders that
// k_write_walk overwrites.
__device__ void lane_region(const WinRun* win, int64_t woff, const Segment* segs, int64_t pos,
                            int64_t rend, int64_t* stage, int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63;
  for (int64_t p = pos; p < rend; p += kChunk) {
    const int64_t i = p + int64_t(lane) * kLaneEvents;
    // window lane of the run holding event i: the last lane with off <= i
    int j = 0;
#pragma unroll
    for (int st = 32; st > 0; st >>= 1) {
      const int64_t v = __shfl(woff, (j + st) & 63, 64);
      if (j + st < 64 && v <= i) j += st;
    }
    if (i < rend) {
      const int32_t qmax = int32_t(rend - i < kLaneEvents ? rend - i : kLaneEvents);
      int kind = 0;  // 0 closed form, 1 @every, 2 walked (k_write_walk)
      CFRule cr;
      CFIter it;
      const Segment* sg = &segs[0];
      uint32_t dm = 0;
      int64_t anchor = 0, D = 0;
      int32_t k = int32_t(i - win[j].off), n = 0;
      // enter window run j at its k-th fire
      auto load_run = [&]() {
        const WinRun& w = win[j];
        n = w.count;
        anchor = w.anchor;
        dm = w.dmask;
        sg = &segs[w.seg];
        if (w.sp.kind == KIND_EVERY) {
          kind = 1;
          D = int64_t(w.sp.sec);
        } else if (run_is_walked(*sg, dm)) {
          kind = 2;
        } else {
          kind = 0;
          cr = cf_rule(w.sp);
          it = cf_seek(cr, *sg, dm, anchor, k);
        }
      };
      load_run();
#pragma unroll 1
      for (int q = 0; q < qmax; q++) {
        if (k >= n) {  // next non-empty run, entered at its first fire
          do {
            j++;
            n = win[j].count;
          } while (n == 0);
          k = 0;
          load_run();
        }
        const int64_t val =
            kind == 0 ? cf_value(*sg, it) : (kind == 1 ? anchor + int64_t(k + 1) * D : 0);
        stage[lane * kStageStride + q] = val;
        if (kind == 0) cf_next(cr, dm, it);
        k++;
      }
    }
    __syncwarp();
    const int64_t lim = rend - p < kChunk ? rend - p : kChunk;
#pragma unroll
    for (int u = 0; u < kLaneEvents; u++) {
      const int t = u * 64 + lane;
      if (t < lim) times[p + t] = stage[(t / kLaneEvents) * kStageStride + t % kLaneEvents];
    }
    __syncwarp();
  }
}

// Persistent closed-form writer.  Waves work independently on kSuper-event
// output slices (grid-stride).  A wave keeps a window of 64 consecutive runs
// (one coalesced round of loads, staged in its LDS slice) and walks its slice:
//   * a run piece of >= kCoopMin events is written by the whole wave, 64
//     consecutive events per store instruction, from mixed-radix digits
//     (coop_cf) or the @every progression (coop_every);
//   * a stretch of shorter runs is written lane-parallel (lane_region).
// Walked runs are left to k_write_walk, which runs after this kernel.
__global__ __launch_bounds__(kWriteWaves * 64) void k_write_cf(
    const DSpec* __restrict__ specs, PlanArgs p, const int64_t* __restrict__ run_anchor,
    const int32_t* __restrict__ run_count, const uint32_t* __restrict__ run_dmask,
    const int64_t* __restrict__ run_off, int64_t nruns, const int64_t* __restrict__ chunk_run,
    int64_t cap, int64_t* __restrict__ times) {
  __shared__ int64_t stage_all[kWriteWaves][64 * kStageStride];
  __shared__ WinRun win_all[kWriteWaves][64];
  __shared__ Segment segs[64];
  for (int i = threadIdx.x; i < p.G * int(sizeof(Segment) / 8); i += blockDim.x)
    reinterpret_cast<int64_t*>(segs)[i] = reinterpret_cast<const int64_t*>(p.segs)[i];
  __syncthreads();

  const int G = p.G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int64_t* stage = stage_all[wave];
  WinRun* win = win_all[wave];
  const int64_t E = run_off[nruns];
  if (E > cap) return;  // output buffer too small: host grows it and relaunches
  const int64_t nsup = (E + kSuper - 1) / kSuper;
  const int64_t nwaves = int64_t(gridDim.x) * kWriteWaves;
  int64_t woff = INT64_MAX;  // this lane's window run: offset, count
  int32_t wcnt = 0;
  auto load_window = [&](int64_t j0) {
    __syncwarp();  // every lane is done with the previous window
    const int64_t jl = j0 + lane;
    WinRun w;
    if (jl < nruns) {
      const int64_t r = G == 1 ? jl : jl / G;
      w.off = run_off[jl];
      w.anchor = run_anchor[jl];
      w.count = run_count[jl];
      w.dmask = run_dmask[jl];
      w.seg = int32_t(jl - r * G);
      w.sp = load_spec(specs + r);
    } else {
      w.off = INT64_MAX;
      w.anchor = 0;
      w.count = 0;
      w.dmask = 0;
      w.seg = 0;
      w.sp = DSpec{};
    }
    w.pad = 0;
    win[lane] = w;
    woff = w.off;
    wcnt = w.count;
    __syncwarp();
  };
  for (int64_t c = int64_t(blockIdx.x) * kWriteWaves + wave; c < nsup; c += nwaves) {
    int64_t pos = c * kSuper;
    const int64_t S1 = E - pos < kSuper ? E : pos + kSuper;
    int64_t jw = chunk_run[c];  // run_off[jw] <= pos
    load_window(jw);
    while (pos < S1) {
      // the run holding pos: the last window lane with off <= pos (lane 0 qualifies)
      const int i = 63 - __builtin_clzll(__ballot(woff <= pos));
      if (i == 63 && jw + 64 < nruns) {  // may continue past the window: slide it
        jw += 63;
        load_window(jw);
        continue;
      }
      const int64_t roff = rl64(woff, i);
      const int64_t rend_run = roff + rl32(wcnt, i);
      const int64_t piece_end = rend_run < S1 ? rend_run : S1;
      if (piece_end - pos >= kCoopMin) {
        const WinRun& w = win[i];
        const Segment& sg = segs[w.seg];
        if (w.sp.kind == KIND_EVERY) coop_every(w, pos, piece_end, times);
        else if (!run_is_walked(sg, w.dmask)) coop_cf(w, sg, pos, piece_end, times);
        pos = piece_end;
        continue;
      }
      // a stretch of short runs: up to the next long run of the window
      const uint64_t big = __ballot(lane > i && wcnt >= kCoopMin);
      int64_t rend;
      if (big) {
        rend = rl64(woff, __builtin_ctzll(big));
      } else {
        const int L = 63 - __builtin_clzll(__ballot(woff != INT64_MAX));
        rend = rl64(woff, L) + rl32(wcnt, L);
      }
      if (rend > S1) rend = S1;
      lane_region(win, woff, segs, pos, rend, stage, times);
      pos = rend;
    }
  }
}

__global__ __launch_bounds__(256) void k_write_walk(const DSpec* __restrict__ specs, int64_t R,
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

__global__ void k_rule_offsets(const int64_t* __restrict__ run_off, int64_t R, int32_t G,
                               int64_t* __restrict__ offsets) {
  int64_t r = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (r <= R) offsets[r] = run_off[r * G];
}

int grid_for(int64_t n, int threads, int max_blocks) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  return int(b < max_blocks ? b : max_blocks);
}

}  // namespace

size_t plan_lds_bytes(const PlanArgs& p) {
  return align_up(size_t(p.zn) * 8, 16) + align_up(size_t(p.zn) * 4, 16) +
         align_up(size_t(p.G) * sizeof(Segment), 16) + align_up(size_t(p.nd) * 4, 16);
}

void launch_next_batch(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* t_in,
                       int64_t* t_out, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_next_batch, dim3(grid_for(n, 256, 256 * 16)), dim3(256),
                     plan_lds_bytes(p), st, specs, n, p, t_in, t_out);
}

void launch_count(const DSpec* specs, int64_t R, const PlanArgs& p, int64_t* run_anchor,
                  int32_t* run_count, uint32_t* run_dmask, unsigned long long* stuck_rule,
                  hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_count, dim3(grid_for(R, 256, 256 * 16)), dim3(256), plan_lds_bytes(p), st,
                     specs, R, p, run_anchor, run_count, run_dmask, stuck_rule);
}

size_t scan_temp_bytes(int64_t n) {
  int64_t nb = (n + kScanTile - 1) / kScanTile;
  return size_t(nb + 1) * sizeof(int64_t);
}

void launch_scan(const int32_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st) {
  if (n <= 0) {
    (void)hipMemsetAsync(out, 0, sizeof(int64_t), st);
    return;
  }
  int64_t nb = (n + kScanTile - 1) / kScanTile;
  int64_t* partial = static_cast<int64_t*>(temp);
  hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(kScanThreads), 0, st, in, n, partial);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanThreads), 0, st, partial, nb);
  hipLaunchKernelGGL(k_scan_apply, dim3(nb), dim3(kScanThreads), 0, st, in, n, partial, out);
}

void launch_chunk_map(const int64_t* run_off, int64_t nruns, int64_t cap, int64_t* chunk_run,
                      hipStream_t st) {
  int64_t max_sup = cap / kSuper + 1;
  hipLaunchKernelGGL(k_chunk_map, dim3(grid_for(max_sup + 1, 256, 4096)), dim3(256), 0, st,
                     run_off, nruns, cap, chunk_run);
}

void launch_write_cf(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor,
                     const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                     int64_t nruns, const int64_t* chunk_run, int64_t cap, int64_t* times,
                     int n_blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_write_cf, dim3(n_blocks), dim3(kWriteWaves * 64), 0, st, specs, p,
                     run_anchor, run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
}

void launch_write_walk(const DSpec* specs, int64_t R, const PlanArgs& p, const int64_t* run_anchor,
                       const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                       int64_t cap, int64_t* times, hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(k_write_walk, dim3(grid_for(R, 256, 256 * 16)), dim3(256),
                     plan_lds_bytes(p), st, specs, R, p, run_anchor, run_count, run_dmask, run_off,
                     cap, times);
}

void launch_rule_offsets(const int64_t* run_off, int64_t R, int32_t G, int64_t* offsets,
                         hipStream_t st) {
  hipLaunchKernelGGL(k_rule_offsets, dim3(grid_for(R + 1, 256, 1 << 30)), dim3(256), 0, st,
                     run_off, R, G, offsets);
}

}  // namespace cg
