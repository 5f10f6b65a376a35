// cg_node_order.hip -- time-ordered view of the per-node fire lists.
//
// The reference's runtime consumer keeps a node's entries ordered by their
// next fire time (Cron.run: sort.Sort(byTime(c.entries)) every wake,
// node/cron/cron.go:64-79,220).  k_node_write leaves each node's list
// rule-major (rules ascending, times ascending within a rule), so this pass
// reorders every node's list by (time, rule): a stable LSD radix sort on the
// time offset (t - T0 - 1, 6 bits per pass) that never moves an event out of
// its node.  The input order inside a node is rule-ascending, so ties keep
// rule order.  (The reference's sort is unstable for equal times; (time,
// rule) is one of the orders it may produce.)
//
// Windows of at most 4096 s (a scheduler's tick windows; config 3's 1-h
// windows): one pass, k_to_node -- one workgroup per node (nodes by ticket),
// a stable counting sort on the whole 12-bit time offset: the node's four
// wave chunks are histogrammed into LDS (read 8 B per event), turned into
// per-(wave, second) destinations by one workgroup scan, and re-read (12 B,
// mostly from the Infinity Cache) and placed: every event is read twice and
// written once, against 2 x (8 + 12 + 12) B for the two radix passes below.
//
// Longer windows: a stable LSD radix sort, 6 bits a pass.
// Node-aligned tiles of up to kTsTile events (a tile never spans two nodes):
//   k_ts_tiles     per node: its tiles' node index (tile bases from a scan)
// per pass (digit = (toff >> shift) & 63):
//   k_ts_hist      per tile: 64-bin histogram (LDS), tile-major
//   k_ts_offsets   one wave per node: digit totals over the node's tiles,
//                  exclusive scan over digits, then per (tile, digit) the
//                  destination of the tile's first event with that digit
//   k_ts_scatter   per tile: stable wave multisplit (6 ballots), running
//                  counts per wave in LDS, time (8 B) + rule (4 B) moved
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

constexpr int kTsItems = 16;
constexpr int kTsTile = 256 * kTsItems;  // events per tile (4 waves x 16 items x 64 lanes)
constexpr int kTsBits = 6;
constexpr int kTsDigits = 1 << kTsBits;

__global__ void k_ts_tile_count(const int64_t* __restrict__ node_off, int32_t N, int32_t* __restrict__ cnt) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n >= N) return;
  cnt[n] = int32_t((node_off[n + 1] - node_off[n] + kTsTile - 1) / kTsTile);
}

__global__ void k_ts_tiles(const int64_t* __restrict__ tile_base, int32_t N, int32_t* __restrict__ tile_node) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n >= N) return;
  for (int64_t t = tile_base[n]; t < tile_base[n + 1]; t++) tile_node[t] = int32_t(n);
}

struct TileRange {
  int64_t lo, hi;
};
__device__ __forceinline__ TileRange tile_range(int64_t t, const int32_t* tile_node, const int64_t* tile_base,
                                                const int64_t* node_off) {
  const int32_t n = tile_node[t];
  TileRange r;
  r.lo = node_off[n] + (t - tile_base[n]) * kTsTile;
  r.hi = min(r.lo + int64_t(kTsTile), node_off[n + 1]);
  return r;
}

__device__ __forceinline__ uint32_t ts_digit(int64_t time, int64_t t0, int shift) {
  return uint32_t(uint64_t(time - t0 - 1) >> shift) & (kTsDigits - 1);
}

__global__ __launch_bounds__(256) void k_ts_hist(const int64_t* __restrict__ time, const int32_t* __restrict__ tile_node,
                                                  const int64_t* __restrict__ tile_base,
                                                  const int64_t* __restrict__ node_off, int64_t t0, int shift,
                                                  int32_t* __restrict__ hist) {
  __shared__ uint32_t h[kTsDigits];
  if (threadIdx.x < kTsDigits) h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t t = blockIdx.x;
  const TileRange r = tile_range(t, tile_node, tile_base, node_off);
  for (int64_t i = r.lo + threadIdx.x; i < r.hi; i += 256) atomicAdd(&h[ts_digit(time[i], t0, shift)], 1u);
  __syncthreads();
  if (threadIdx.x < kTsDigits) hist[t * kTsDigits + threadIdx.x] = int32_t(h[threadIdx.x]);
}

// one wave per node, lane d = digit
__global__ __launch_bounds__(64) void k_ts_offsets(const int32_t* __restrict__ hist,
                                                    const int64_t* __restrict__ tile_base,
                                                    const int64_t* __restrict__ node_off, int32_t N,
                                                    int64_t* __restrict__ off) {
  const int32_t n = blockIdx.x;
  if (n >= N) return;
  const int d = threadIdx.x;
  const int64_t ta = tile_base[n], tb = tile_base[n + 1];
  int64_t tot = 0;
  for (int64_t t = ta; t < tb; t++) tot += hist[t * kTsDigits + d];
  int64_t inc = tot;  // inclusive scan over the 64 digits
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(inc, o, 64);
    if (d >= o) inc += y;
  }
  int64_t run = node_off[n] + inc - tot;
  for (int64_t t = ta; t < tb; t++) {
    off[t * kTsDigits + d] = run;
    run += hist[t * kTsDigits + d];
  }
}

// Stable scatter of one tile.  Input order inside the tile: wave w owns
// events [lo + w*1024, +1024), item j the 64 events [j*64, j*64 + 64) of
// those.  Rank among equal digits = earlier items of its wave (running counts
// in LDS) + earlier lanes of its item (6-ballot multisplit) + earlier waves
// (prefix per digit) + earlier tiles of the node (k_ts_offsets).
__global__ __launch_bounds__(256) void k_ts_scatter(const int64_t* __restrict__ tin, const int32_t* __restrict__ rin,
                                                     const int32_t* __restrict__ tile_node,
                                                     const int64_t* __restrict__ tile_base,
                                                     const int64_t* __restrict__ node_off,
                                                     const int64_t* __restrict__ off, int64_t t0, int shift,
                                                     int64_t* __restrict__ tout, int32_t* __restrict__ rout) {
  __shared__ int32_t run[4][kTsDigits];
  __shared__ int64_t base_of[4][kTsDigits];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  run[w][lane] = 0;
  const int64_t t = blockIdx.x;
  const TileRange r = tile_range(t, tile_node, tile_base, node_off);
  __syncthreads();
  const int64_t base = r.lo + int64_t(w) * (64 * kTsItems);
  const uint64_t lt = (1ull << lane) - 1ull;
  int64_t tv[kTsItems];
  int32_t rv[kTsItems], rk[kTsItems];
  uint32_t dg[kTsItems];
#pragma unroll
  for (int j = 0; j < kTsItems; j++) {
    const int64_t i = base + j * 64 + lane;
    tv[j] = i < r.hi ? tin[i] : t0 + 1;
    rv[j] = i < r.hi ? rin[i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kTsItems; j++) {
    const bool valid = base + j * 64 + lane < r.hi;
    const uint32_t d = ts_digit(tv[j], t0, shift);
    dg[j] = d;
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < kTsBits; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    // every lane reads the running count before the group's first lane adds
    // the group size (a wave's LDS operations complete in program order)
    const int32_t r0 = run[w][d];
    rk[j] = r0 + __popcll(peers & lt);
    if (valid && (peers & lt) == 0) run[w][d] = r0 + __popcll(peers);
  }
  __syncthreads();
  if (threadIdx.x < kTsDigits) {
    const int d = threadIdx.x;
    int64_t acc = off[t * kTsDigits + d];
    for (int ww = 0; ww < 4; ww++) {
      base_of[ww][d] = acc;
      acc += run[ww][d];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kTsItems; j++) {
    if (base + j * 64 + lane >= r.hi) continue;
    const int64_t pos = base_of[w][dg[j]] + rk[j];
    tout[pos] = tv[j];
    rout[pos] = rv[j];
  }
}

// ---- windows <= 4096 s: the ordered lists straight from the segment records
//
// k_node_timed writes every node's list in (time, rule) order directly from
// the per-node writer's segment records (k_seg_records: per (node, rule band)
// segment, one record per non-empty pair {rule, first position, x, stride}),
// without reading the rule-major per-node lists: one workgroup per node
// (nodes by ticket), NW waves, each owning a contiguous range of the node's
// segments (so the waves' records are in rule order, wave after wave).
//   hist    every fire's second (t - t0 - 1) counted into an LDS histogram;
//           a progression's fires are t0 + f0 + i * stride, other records'
//           come from the rule-major fire lists (L2)
//   slabs   prefix over the seconds -> each second's first output position;
//           the window is cut into slabs of <= kTwC events and <= kTwSlabKeys
//           seconds (a second holding more than kTwC events is a slab alone)
//   per slab  each wave expands its records' fires inside the slab (fire
//           indices by one division per slab bound) into LDS in rule order
//           (the waves' bases from the previous slab's visit, which also
//           counted this slab), then a stable LDS counting sort by second
//           places them and the slab is stored with coalesced writes; a
//           single heavy second is written in rule order directly
// HBM traffic is the output (12 B per event) plus the records (16 B per
// pair, re-read per slab from L2): the rule-major per-node lists are not read.
constexpr int kTwWaves = 8;
constexpr int kTwC = 2048;        // events per slab staged in LDS
constexpr int kTwKeys = 4096;     // window seconds
constexpr int kTwSlabKeys = 1024; // seconds per slab
constexpr int kTwMaxSegs = 1024;  // (node, band) segments per node

struct TwArgs {
  const int64_t* seg_pair;
  const int32_t* seg_nrec;
  const int64_t* seg_pos;
  const PairRec* recs;
  const int64_t* rule_off;
  const int64_t* times;
  int64_t t0;
  int32_t N, K, B, H;
  int32_t* ctl;  // [0] node ticket, [1] error (a node list of 2^31 events or more)
  int64_t* out_time;
  int32_t* out_rule;
};

// floor(a / b) for |a| < 2^24, b >= 1 (f32 quotient, corrected)
__device__ __forceinline__ int32_t fdiv_floor(int32_t a, int32_t b) {
  int32_t q = int32_t(floorf(float(a) / float(b)));
  const int32_t r = a - q * b;
  q += r < 0 ? -1 : (r >= b ? 1 : 0);
  return q;
}

// A wave's view of one record: fires i in [0, cnt), second of fire i =
// f0 - 1 + i * st (progression), or from the rule-major list g[i] - t0 - 1.
struct TwRec {
  int32_t rule, cnt, f0, st;
  const int64_t* g;  // gathered: the record's first fire in the rule-major list (st == 0)
};

// number of the record's fires with second < k (k in [0, H])
__device__ __forceinline__ int32_t tw_before(const TwRec& r, int64_t t0, int32_t k) {
  if (r.cnt <= 0) return 0;
  if (r.st != 0) {
    // i with f0 - 1 + i*st < k  <=>  i < (k + 1 - f0) / st
    const int32_t num = k + 1 - r.f0;
    if (num <= 0) return 0;
    const int32_t i = fdiv_floor(num + r.st - 1, r.st);
    return i < r.cnt ? i : r.cnt;
  }
  int32_t lo = 0, hi = r.cnt;  // first i with g[i] - t0 - 1 >= k
  while (lo < hi) {
    const int32_t mid = (lo + hi) >> 1;
    if (r.g[mid] - t0 - 1 < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t tw_fire(const TwRec& r, int64_t t0, int32_t i) {
  return r.st != 0 ? t0 + int64_t(r.f0) + int64_t(i) * r.st : r.g[i];
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void k_node_timed(TwArgs a) {
  __shared__ int32_t start[kTwKeys + 1];        // histogram, then first relative output position per second
  __shared__ int16_t slab_lo[kTwKeys + 1];      // first second of slab j; slab_lo[nslabs] = H
  __shared__ int32_t hw[NW][kTwSlabKeys];       // per-wave counts, then destinations, per slab second
  __shared__ int64_t At[kTwC], Bt[kTwC];
  __shared__ int32_t Ar[kTwC], Br[kTwC];
  __shared__ int64_t s_recb[kTwMaxSegs];        // segment: first record
  __shared__ int32_t s_nrec[kTwMaxSegs], s_size[kTwMaxSegs];
  __shared__ int64_t s_glo[kTwMaxSegs];         // segment: rule-major index of its band's first fire
  __shared__ int32_t wseg[NW + 1];              // wave w owns segments [wseg[w], wseg[w+1])
  __shared__ int32_t wtot[2][NW];               // per-wave fires in a slab (double-buffered)
  __shared__ int32_t s_misc[4];                 // node, nslabs
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const int32_t H = a.H, K = a.K;
  for (;;) {
    if (tid == 0) s_misc[0] = atomicAdd(a.ctl, 1);
    __syncthreads();
    const int32_t n = s_misc[0];
    if (n >= a.N) break;
    const int64_t s0 = int64_t(n) * K;
    const int64_t lo = a.seg_pos[s0], L = a.seg_pos[s0 + K] - lo;
    if (L == 0 || L > INT32_MAX) {
      if (L > INT32_MAX && tid == 0) a.ctl[1] = 1;
      __syncthreads();
      continue;
    }
    // segments, histogram reset
    for (int k = tid; k < K; k += NW * 64) {
      s_recb[k] = a.seg_pair[s0 + k];
      s_nrec[k] = a.seg_nrec[s0 + k];
      s_size[k] = int32_t(a.seg_pos[s0 + k + 1] - a.seg_pos[s0 + k]);
      s_glo[k] = a.rule_off[int64_t(k) * a.B];
    }
    for (int k = tid; k <= H; k += NW * 64) start[k] = 0;
    __syncthreads();
    // waves' segment ranges: about equal record counts (thread 0; K is small)
    if (tid == 0) {
      int64_t tot = 0;
      for (int k = 0; k < K; k++) tot += s_nrec[k];
      int64_t run = 0;
      int ww = 0;
      wseg[0] = 0;
      for (int k = 0; k < K && ww < NW - 1; k++) {
        run += s_nrec[k];
        while (ww < NW - 1 && run * NW >= tot * (ww + 1)) wseg[++ww] = k + 1;
      }
      while (ww < NW - 1) wseg[++ww] = K;
      wseg[NW] = K;
    }
    __syncthreads();
    const int32_t ka_w = wseg[w], kb_w = wseg[w + 1];

    // Visit every record of this wave, 64 at a time: lane i holds record i of
    // the batch as a TwRec.  fn(rec, valid) is called once per batch with all
    // lanes active.
    auto visit = [&](auto&& fn) {
      for (int32_t k = ka_w; k < kb_w; k++) {
        const int32_t nr = s_nrec[k];
        const int64_t rb = s_recb[k];
        const int64_t* tb = a.times + s_glo[k];
        for (int32_t q = 0; q < nr; q += 64) {
          const int32_t qi = q + lane;
          const bool valid = qi < nr;
          const PairRec pr = a.recs[rb + (valid ? qi : nr - 1)];
          // this record's count: the next record's first position, or the segment's end
          int32_t nd = __shfl_down(pr.dst, 1, 64);
          if (lane == 63 || qi + 1 >= nr) nd = qi + 1 < nr ? a.recs[rb + qi + 1].dst : s_size[k];
          TwRec r;
          r.rule = pr.rule;
          r.cnt = valid ? nd - pr.dst : 0;
          r.st = pr.st;
          r.f0 = pr.st != 0 ? int32_t(int64_t(pr.x) + int64_t(pr.dst) * pr.st) : 0;
          r.g = tb + (int64_t(pr.dst) + pr.x);
          fn(r, valid);
        }
      }
    };
    // fires [i0, i0 + c) of each lane's record, expanded over the wave's lanes:
    // emit(rec lane j, fire index i, flattened index f)
    auto expand = [&](const TwRec& r, int32_t i0, int32_t c, auto&& emit) {
      int32_t inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      const int32_t total = __shfl(inc, 63, 64);
      const int32_t pre = inc - c;
      for (int32_t f = lane; f - lane < total; f += 64) {
        // the record holding fire f: the largest j with pre_j <= f (lanes with
        // c = 0 share their successor's pre; the largest one is the holder)
        int j = 0;
#pragma unroll
        for (int st = 32; st; st >>= 1) {
          const int32_t pj = __shfl(pre, j + st, 64);
          if (pj <= f && j + st < 64) j += st;
        }
        const int32_t pj = __shfl(pre, j, 64), i0j = __shfl(i0, j, 64);
        TwRec rj;
        rj.rule = __shfl(r.rule, j, 64);
        rj.cnt = __shfl(r.cnt, j, 64);
        rj.f0 = __shfl(r.f0, j, 64);
        rj.st = __shfl(r.st, j, 64);
        rj.g = reinterpret_cast<const int64_t*>(
            (uint64_t(uint32_t(__shfl(int(uint64_t(r.g) >> 32), j, 64))) << 32) |
            uint32_t(__shfl(int(uint64_t(r.g)), j, 64)));
        if (f < total) emit(rj, i0j + (f - pj), f);
      }
      return total;
    };

    // 1. histogram of the node's fire seconds
    visit([&](const TwRec& r, bool) {
      expand(r, 0, r.cnt, [&](const TwRec& rj, int32_t i, int32_t) {
        atomicAdd(&start[int32_t(tw_fire(rj, a.t0, i) - a.t0 - 1)], 1);
      });
    });
    __syncthreads();
    // 2. exclusive prefix over the seconds (16 per thread at 512 threads)
    {
      constexpr int PER = (kTwKeys + NW * 64 - 1) / (NW * 64);
      int32_t loc[PER], sum = 0;
#pragma unroll
      for (int j = 0; j < PER; j++) {
        const int k = tid * PER + j;
        const int32_t v = k < H ? start[k] : 0;
        loc[j] = sum;
        sum += v;
      }
      int32_t inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
      }
      if (lane == 63) wtot[0][w] = inc;
      __syncthreads();
      int32_t base = inc - sum;
      for (int ww = 0; ww < w; ww++) base += wtot[0][ww];
      __syncthreads();
#pragma unroll
      for (int j = 0; j < PER; j++) {
        const int k = tid * PER + j;
        if (k < H) start[k] = base + loc[j];
      }
      if (tid == 0) start[H] = int32_t(L);
    }
    __syncthreads();
    // 3. slabs: greedy, <= kTwC events and <= kTwSlabKeys seconds (a heavier
    // single second is a slab alone)
    if (tid == 0) {
      int32_t ns = 0, k = 0;
      while (k < H) {
        slab_lo[ns++] = int16_t(k);
        int32_t l = k + 1, h = min(H, k + kTwSlabKeys);  // largest e in [k+1, h] with start[e] - start[k] <= kTwC
        while (l < h) {
          const int32_t m = (l + h + 1) >> 1;
          if (start[m] - start[k] <= kTwC) l = m;
          else h = m - 1;
        }
        k = l;
      }
      slab_lo[ns] = int16_t(H);
      s_misc[1] = ns;
    }
    __syncthreads();
    const int32_t nslabs = s_misc[1];
    // this wave's fires in slab 0
    {
      const int32_t e0 = slab_lo[1];
      int32_t acc = 0;
      visit([&](const TwRec& r, bool) { acc += tw_before(r, a.t0, e0); });
      for (int o = 32; o; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (lane == 0) wtot[0][w] = acc;
    }
    __syncthreads();
    for (int32_t j = 0; j < nslabs; j++) {
      const int32_t kx = slab_lo[j], ky = slab_lo[j + 1];
      const int32_t kz = j + 1 < nslabs ? slab_lo[j + 2] : H;
      const int32_t p0 = start[kx], nj = start[ky] - p0;
      const bool heavy = nj > kTwC;  // one second, more events than the staging holds
      const int cb = j & 1;
      int32_t base = 0;
      for (int ww = 0; ww < w; ww++) base += wtot[cb][ww];
      // expand this slab's fires (and count the next slab's)
      int32_t nxt = 0;
      visit([&](const TwRec& r, bool) {
        const int32_t ia = tw_before(r, a.t0, kx), ib = tw_before(r, a.t0, ky);
        if (j + 1 < nslabs) nxt += tw_before(r, a.t0, kz) - ib;
        const int32_t tot = expand(r, ia, ib - ia, [&](const TwRec& rj, int32_t i, int32_t f) {
          const int64_t t = tw_fire(rj, a.t0, i);
          if (heavy) {  // rule order is the order within one second
            a.out_time[lo + p0 + base + f] = t;
            a.out_rule[lo + p0 + base + f] = rj.rule;
          } else {
            At[base + f] = t;
            Ar[base + f] = rj.rule;
          }
        });
        base += tot;
      });
      for (int o = 32; o; o >>= 1) nxt += __shfl_xor(nxt, o, 64);
      if (lane == 0) wtot[cb ^ 1][w] = nxt;
      __syncthreads();
      if (heavy) continue;
      // stable counting sort of A (rule-major) by second into B: wave ww
      // takes A[ww*Q, (ww+1)*Q)
      const int32_t nk = ky - kx;
      int kbits = 0;
      while ((1 << kbits) < nk) kbits++;
      const int32_t Q = (((nj + NW - 1) / NW) + 63) & ~63;
      const int32_t qa = min(w * Q, nj), qb = min(qa + Q, nj);
      for (int k = lane; k < nk; k += 64) hw[w][k] = 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int32_t i = qa + lane; i < qb; i += 64) atomicAdd(&hw[w][int32_t(At[i] - a.t0 - 1) - kx], 1);
      __syncthreads();
      for (int k = tid; k < nk; k += NW * 64) {
        int32_t run = start[kx + k] - p0;
#pragma unroll
        for (int ww = 0; ww < NW; ww++) {
          const int32_t c = hw[ww][k];
          hw[ww][k] = run;
          run += c;
        }
      }
      __syncthreads();
      for (int32_t i0 = qa; i0 < qb; i0 += 64) {
        const int32_t i = i0 + lane;
        const bool valid = i < qb;
        const int64_t t = valid ? At[i] : a.t0 + 1 + kx;
        const int32_t rl = valid ? Ar[i] : 0;
        const uint32_t k = uint32_t(int32_t(t - a.t0 - 1) - kx);
        uint64_t peers = __ballot(valid);
        for (int bit = 0; bit < kbits; bit++) {
          const bool on = (k >> bit) & 1u;
          const uint64_t m = __ballot(on);
          peers &= on ? m : ~m;
        }
        const int32_t r0 = hw[w][k];
        if (valid && (peers & lt) == 0) hw[w][k] = r0 + __popcll(peers);
        if (valid) {
          const int32_t pos = r0 + __popcll(peers & lt);
          Bt[pos] = t;
          Br[pos] = rl;
        }
      }
      __syncthreads();
      for (int32_t i = tid; i < nj; i += NW * 64) {
        a.out_time[lo + p0 + i] = Bt[i];
        a.out_rule[lo + p0 + i] = Br[i];
      }
      // (the next slab writes A and hw only after its visit; B after a barrier)
    }
    __syncthreads();  // every wave is done with this node's LDS
  }
}

int gridn(int64_t n, int threads) { return int(std::max<int64_t>(1, (n + threads - 1) / threads)); }

}  // namespace

extern "C" int cg_node_result_order_by_time(cg_ctx* c) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_order_by_time: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  const int64_t En = c->pn_E;
  const int32_t N = int32_t(c->pn_N);
  if (En == 0 || N == 0) return CG_OK;
  const int64_t H = c->pn_t1 - c->pn_t0;  // time offsets in [0, H - 1]
  int bits = 0;
  while (bits < 63 && (int64_t(1) << bits) < H) bits++;
  const int passes = std::max(1, (bits + kTsBits - 1) / kTsBits);
  hipStream_t st = c->st;
  // windows <= 4096 s, straight from the last per-node call's segment records
  // (valid until another expansion reuses the context's buffers)
  if (H <= kTwKeys && c->pn_recs_valid && c->pn_K > 0 && c->pn_K <= kTwMaxSegs) {
    if ((rc = c->ts_cnt.ensure(std::max<int64_t>(N, 2))) || (rc = c->node_time2.ensure(En)) ||
        (rc = c->node_rule2.ensure(En)))
      return rc;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipEventRecord(c->pev[0], st);
    if ((rc = cg_hip_check(hipMemsetAsync(c->ts_cnt.p, 0, 8, st), "memset"))) return rc;
    TwArgs ta{c->seg_pair.p, c->seg_nrec.p, c->seg_pos.p, c->recs.p, c->offsets.p, c->times.p, c->pn_t0,
              N, c->pn_K, c->pn_B, int32_t(H), c->ts_cnt.p, c->node_time2.p, c->node_rule2.p};
    hipLaunchKernelGGL(k_node_timed<kTwWaves>, dim3(unsigned(std::min<int64_t>(N, cus))), dim3(kTwWaves * 64), 0,
                       st, ta);
    (void)hipEventRecord(c->pev[1], st);
    if ((rc = cg_hip_check(hipGetLastError(), "k_node_timed"))) return rc;
    int32_t ctl[2] = {0, 0};
    if ((rc = cg_hip_check(hipMemcpyAsync(ctl, c->ts_cnt.p, 8, hipMemcpyDeviceToHost, st), "ctl")) ||
        (rc = cg_hip_check(hipStreamSynchronize(st), "sync")))
      return rc;
    if (ctl[1] == 0) {
      std::swap(c->node_time, c->node_time2);
      std::swap(c->node_rule, c->node_rule2);
      (void)hipEventElapsedTime(&c->kt[12], c->pev[0], c->pev[1]);
      c->pn_recs_valid = false;  // the records describe the rule-major lists, no longer the result
      return CG_OK;
    }
    // a node list of 2^31 events or more: the radix passes below
  }
  if ((rc = c->ts_cnt.ensure(N)) || (rc = c->ts_base.ensure(int64_t(N) + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(N))))) return rc;
  hipLaunchKernelGGL(k_ts_tile_count, dim3(gridn(N, 256)), dim3(256), 0, st, c->node_off.p, N, c->ts_cnt.p);
  launch_scan(c->ts_cnt.p, c->ts_base.p, N, c->scan_tmp.p, st);
  int64_t T = 0;
  if ((rc = cg_hip_check(hipMemcpyAsync(&T, c->ts_base.p + N, 8, hipMemcpyDeviceToHost, st), "tiles")) ||
      (rc = cg_hip_check(hipStreamSynchronize(st), "sync")))
    return rc;
  if ((rc = c->ts_tile_node.ensure(T)) || (rc = c->ts_hist.ensure(T * kTsDigits)) ||
      (rc = c->ts_off.ensure(T * kTsDigits)) || (rc = c->node_time2.ensure(En)) || (rc = c->node_rule2.ensure(En)))
    return rc;
  (void)hipEventRecord(c->pev[0], st);
  hipLaunchKernelGGL(k_ts_tiles, dim3(gridn(N, 256)), dim3(256), 0, st, c->ts_base.p, N, c->ts_tile_node.p);
  int64_t* tin = c->node_time.p;
  int32_t* rin = c->node_rule.p;
  int64_t* tout = c->node_time2.p;
  int32_t* rout = c->node_rule2.p;
  for (int p = 0; p < passes; p++) {
    const int shift = p * kTsBits;
    hipLaunchKernelGGL(k_ts_hist, dim3(unsigned(T)), dim3(256), 0, st, tin, c->ts_tile_node.p, c->ts_base.p,
                       c->node_off.p, c->pn_t0, shift, c->ts_hist.p);
    hipLaunchKernelGGL(k_ts_offsets, dim3(unsigned(N)), dim3(64), 0, st, c->ts_hist.p, c->ts_base.p,
                       c->node_off.p, N, c->ts_off.p);
    hipLaunchKernelGGL(k_ts_scatter, dim3(unsigned(T)), dim3(256), 0, st, tin, rin, c->ts_tile_node.p,
                       c->ts_base.p, c->node_off.p, c->ts_off.p, c->pn_t0, shift, tout, rout);
    std::swap(tin, tout);
    std::swap(rin, rout);
  }
  (void)hipEventRecord(c->pev[1], st);
  if ((rc = cg_hip_check(hipGetLastError(), "time-order kernels"))) return rc;
  if (passes % 2 == 1) {  // the ordered lists are in the second buffers: make them the result
    std::swap(c->node_time, c->node_time2);
    std::swap(c->node_rule, c->node_rule2);
  }
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  (void)hipEventElapsedTime(&c->kt[12], c->pev[0], c->pev[1]);
  return CG_OK;
}
