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
#include <cstdlib>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

constexpr int kTsItems = 16;
constexpr int kTsTile = 256 * kTsItems;  // events per tile (4 waves x 16 items x 64 lanes)
constexpr int kTsBits = 6;
constexpr int kTsDigits = 1 << kTsBits;

// tiles per node; none at all when the lists' total exceeds the buffers' capacity
// cap (a pipelined window whose writer wrote nothing: CG_ECAPACITY at the wait),
// so no later kernel of the pass touches an event past cap
__global__ void k_ts_tile_count(const int64_t* __restrict__ node_off, int32_t N, int tile, int64_t cap,
                                int32_t* __restrict__ cnt) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n >= N) return;
  cnt[n] = node_off[N] > cap ? 0 : int32_t((node_off[n + 1] - node_off[n] + tile - 1) / tile);
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
                                                const int64_t* node_off, int tile = kTsTile) {
  const int32_t n = tile_node[t];
  TileRange r;
  r.lo = node_off[n] + (t - tile_base[n]) * tile;
  r.hi = min(r.lo + int64_t(tile), node_off[n + 1]);
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

// ---- windows <= 4096 s (12-bit time offsets): tile sort + per-node merge ----
//
//   k_ot_tile   per tile (<= kOtTile events of one node, rule-major): a
//               stable LDS counting partition of packed (offset << 12 |
//               index) words by slab (offset >> 6: 64 s; one 6-bit pass), the
//               tile written back slab by slab with coalesced stores, and its
//               slab prefix pre[t][0..64].  A node of one tile is sorted by
//               the whole offset instead (a second pass) and is done.
//   k_ot_merge  one workgroup per node: runs of whole slabs holding <= a
//               chunk are gathered from every tile (one contiguous range per
//               tile: its events of those slabs, in rule order; tile order =
//               rule order), sorted by offset - the run's first second in LDS
//               (one 8-bit pass for a run of <= 4 slabs) and stored
//               contiguously; a larger slab, or every slab of a node of more
//               than kOtMaxTiles tiles, is queued for k_ot_big
//   k_ot_big    per queued slab: the histogram of its 64 seconds over all its
//               portions, then its chunks in order, each sorted in LDS and
//               stored at its seconds' running bases
// Every sort is stable and the gathered order is (tile, rule order inside
// the tile), so equal seconds stay in rule order.  The partitioned tiles are
// kept as 16-bit offsets + rules (6 B per event), so the two passes move
// 12 + 6 + 6 + 12 = 36 B per event, every store coalesced, where the LSD
// passes above scatter each event to its own address per pass and read the
// times again for every histogram.
constexpr int kOtItems = 16;                  // per thread
constexpr int kOtTile = 4 * 64 * kOtItems;    // 4096 events: the tile sort's 4-wave chunk
#ifndef CG_OT_MERGE_WAVES
#define CG_OT_MERGE_WAVES 4
#endif
constexpr int kOtMergeWaves = CG_OT_MERGE_WAVES;  // k_ot_merge: waves per node
#ifndef CG_OT_MERGE_ITEMS
#define CG_OT_MERGE_ITEMS 16
#endif
constexpr int kOtMergeItems = CG_OT_MERGE_ITEMS;  // k_ot_merge: events per thread of a chunk
// the merge's packed words when every rule index is below 2^20: offset << 20 |
// rule (the word order is the (time, rule) order; no rule array in LDS)
constexpr int kOtRuleBits = 20;
// chunk index bits of a packed word (offset << kOtIdxBits | index): up to
// 16384 events (k_ot_mid's 16-wave chunk: 16 waves x 64 x 16)
constexpr int kOtIdxBits = 14;
constexpr int kOtMidWaves = 8;    // k_ot_mid: waves per slab (slabs of <= 8192 events)
constexpr int kOtMid2Waves = 16;  // its 16-wave form (slabs of <= 16384 events; one block per CU)
#ifndef CG_OT_DENSE_WAVES
#define CG_OT_DENSE_WAVES 8
#endif
constexpr int kOtDenseWaves = CG_OT_DENSE_WAVES;  // the dense nodes' merge: waves per block (8 or 16)
constexpr int kOtDenseWavesHx = 16;                // its form past 2^20 rules (order_tail)
#ifndef CG_OT_DENSE_ITEMS
#define CG_OT_DENSE_ITEMS 16
#endif
constexpr int kOtDenseItems = CG_OT_DENSE_ITEMS;  // its events per thread of a chunk
static_assert(64 * kOtMid2Waves * kOtItems <= (1 << kOtIdxBits) && 64 * kOtDenseWaves * kOtDenseItems <= (1 << kOtIdxBits) &&
                  64 * kOtDenseWavesHx * kOtDenseItems <= (1 << kOtIdxBits),
              "every chunk's element index fits the packed words' index bits");
static_assert(kOtMergeWaves <= 8 && 12 + kOtIdxBits <= 32, "packed words");
constexpr uint32_t kOtIdxMask = (1u << kOtIdxBits) - 1u;
constexpr int kOtSlabBits = 6;               // slab = offset >> kOtSlabBits (64 s): one 6-bit digit
constexpr int kOtSlabs = 4096 >> kOtSlabBits;
constexpr int kOtPre = kOtSlabs + 1;          // pre row per tile
constexpr int kOtMaxTiles = 256;              // portion list capacity
// rule indices up to 2^24 in the packed words: the words hold rule & 0xFFFFF
// and every tile's rules share rule >> 20 (ts_hi); the merges rebuild the
// rule from its tile
constexpr int kOtHiBits = 4;
constexpr uint32_t kOtLowMask = (1u << kOtRuleBits) - 1u;

// The tiles of the tile sort: every node's list cut into kOtTile-event tiles,
// restarting at each multiple of 2^20 in rule index (the lists are
// rule-major, so those are H - 1 cut positions per node, found from the
// (node, band) segment offsets: bph bands of 2^20 / bph rules per block).
struct OtCut {
  const int64_t* seg_pos;  // null: no cuts (H = 1)
  int32_t K, bph, H;
};
// the first position of node n's events with rule >= h << 20 (0 <= h <= H)
__device__ __forceinline__ int64_t ot_cut_pos(const OtCut& c, const int64_t* node_off, int32_t n, int h) {
  if (c.H <= 1) return h == 0 ? node_off[n] : node_off[n + 1];
  const int64_t k = int64_t(h) * c.bph;
  return c.seg_pos[int64_t(n) * c.K + (k < c.K ? k : c.K)];
}
// tiles per node; none at all when the lists exceed the buffers' capacity
__global__ void k_ot_tile_count(const int64_t* __restrict__ node_off, int32_t N, int64_t cap, OtCut cut,
                                int32_t* __restrict__ cnt) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n >= N) return;
  int32_t t = 0;
  if (node_off[N] <= cap) {
    int64_t a = ot_cut_pos(cut, node_off, int32_t(n), 0);
    for (int h = 0; h < cut.H; h++) {
      const int64_t b = ot_cut_pos(cut, node_off, int32_t(n), h + 1);
      t += int32_t((b - a + kOtTile - 1) / kOtTile);
      a = b;
    }
  }
  cnt[n] = t;
}
// per tile: its node, first position and rule >> 20; ts_start[T] = the end
__global__ void k_ot_tiles(const int64_t* __restrict__ tile_base, const int64_t* __restrict__ node_off, int32_t N,
                           OtCut cut, int32_t* __restrict__ tile_node, int64_t* __restrict__ ts_start,
                           int32_t* __restrict__ ts_hi) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n >= N) return;
  int64_t t = tile_base[n];
  if (n == N - 1) ts_start[tile_base[N]] = node_off[N];
  if (tile_base[n + 1] == t) return;
  int64_t a = ot_cut_pos(cut, node_off, int32_t(n), 0);
  for (int h = 0; h < cut.H; h++) {
    const int64_t b = ot_cut_pos(cut, node_off, int32_t(n), h + 1);
    for (int64_t p = a; p < b; p += kOtTile, t++) {
      tile_node[t] = int32_t(n);
      ts_start[t] = p;
      ts_hi[t] = h;
    }
    a = b;
  }
}

template <int NW>
__device__ __forceinline__ void ot_sync() {
  if constexpr (NW > 1) {
    __syncthreads();
  } else {  // one wave: its LDS operations complete in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

#ifndef CG_OT_RUN_SLOTS
#define CG_OT_RUN_SLOTS 1  // RUNS ranks: a run's position handed to its lanes through LDS by run ordinal (mbcnt), not ds_bpermute from the head lane
#endif
template <int NW, int D>  // D digits: 64 or 256
struct OtRank {
  int32_t run[NW][D];  // per wave: its events of each digit, then their first position
  int32_t head[CG_OT_RUN_SLOTS ? NW : 1][64];  // RUNS, CG_OT_RUN_SLOTS: per wave, run k's first position - its head lane
  int32_t dbase[65];   // D == 64: exclusive prefix of the digit totals; [64] = events
  int32_t wtot[4];     // CG_OT_SCAN_ALL: the digit-scan waves' totals
};
#ifndef CG_OT_SCAN_ALL
#define CG_OT_SCAN_ALL 1  // a 256-digit scan by 256 threads, one digit each (fewer live VGPRs: no merge spills)
#endif

// Stable positions of the n valid items (item j of wave w, lane l = element
// w*64*kOtItems + j*64 + l) by the digit dg[j] < D: earlier elements with
// the same digit keep their order.  The rank inside the wave is the value an
// LDS atomic add on the digit's counter returns: a wave's LDS operations
// complete in program order, and the lanes of one ds_add_rtn that hit the
// same address are served in ascending lane order on gfx950
// (tools/lds_atomic_order.hip: 0 of 6.3 M ranks out of order over random and
// adversarial digit patterns; the GPU tests check every ordered list against
// the oracle's).  It replaces a 6-ballot multisplit per element (~40 VALU
// instructions; the sorts were VALU-bound, profiles/r03_ab_time_order.json).
// Each wave only touches its own counter row outside the two barriers.
// RUNS: lanes holding the same digit as their left neighbour join its run and
// only the run's first lane adds (the run's length): a digit shared by long
// runs of neighbouring elements (slabs of a rule-major tile: one rule's
// events sit in neighbouring seconds) would otherwise serialise its lanes on
// one LDS address.  Ends synchronised.
template <int NW, int D, bool RUNS = false, int IT = kOtItems>
__device__ __forceinline__ void ot_rank(const uint32_t (&dg)[IT], int n, int32_t (&pos)[IT],
                                        OtRank<NW, D>& s) {
  static_assert(D == 64 || D == 256, "digits");
  constexpr int P = D / 64;  // digits per lane in the scan
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t* run = reinterpret_cast<uint32_t*>(s.run[w]);
#pragma unroll
  for (int i = 0; i < P; i++) run[lane + 64 * i] = 0;
  const int ebase = w * (64 * IT);
  const uint64_t upto = ~0ull >> (63 - lane);  // lanes 0 .. lane
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const bool valid = ebase + j * 64 + lane < n;
    if constexpr (RUNS) {
      const uint32_t d = valid ? dg[j] : uint32_t(D);  // invalid lanes (the tail) add nothing
      // the left neighbour's digit by DPP wave_shr:1 (no LDS round trip;
      // lane 0 is a head whatever it reads)
      const uint32_t left = uint32_t(__builtin_amdgcn_update_dpp(0, int(d), 0x138, 0xf, 0xf, false));
      const bool head = lane == 0 || left != d;
      const uint64_t hm = __ballot(head);
      const uint64_t after = hm & ~upto;
      const int end = after ? __builtin_ctzll(after) : 64;
      if constexpr (CG_OT_RUN_SLOTS) {
        // run ordinal k = heads before this lane (mbcnt), minus one off a head;
        // the head leaves its run's first position - its lane in slot k (a
        // wave's LDS operations complete in order)
        const int before = int(__builtin_amdgcn_mbcnt_hi(uint32_t(hm >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(hm), 0u)));
        const int k = head ? before : before - 1;
        int32_t* slot = s.head[w];
        if (head && valid) slot[k] = int32_t(atomicAdd(run + d, uint32_t(end - lane))) - lane;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pos[j] = valid ? slot[k] + lane : 0;
      } else {
        const int h = 63 - __builtin_clzll(hm & upto);  // this lane's run starts at lane h
        uint32_t r = 0;
        if (head && valid) r = atomicAdd(run + d, uint32_t(end - lane));
        r = __shfl(r, h, 64);
        pos[j] = valid ? int32_t(r) + (lane - h) : 0;
      }
    } else {
      pos[j] = valid ? int32_t(atomicAdd(run + dg[j], 1u)) : 0;
    }
  }
  ot_sync<NW>();
  if constexpr (CG_OT_SCAN_ALL && D == 256 && NW >= 4) {  // thread d < 256: digit d
    const int d = threadIdx.x;
    int32_t c[NW], sum = 0;
#pragma unroll
    for (int ww = 0; ww < NW; ww++) {
      c[ww] = d < D ? s.run[ww][d] : 0;
      sum += c[ww];
    }
    int32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63 && w < 4) s.wtot[w] = inc;
    ot_sync<NW>();
    int32_t acc = inc - sum;
    for (int ww = 0; ww < w && ww < 4; ww++) acc += s.wtot[ww];
    if (d < D) {
#pragma unroll
      for (int ww = 0; ww < NW; ww++) {
        s.run[ww][d] = acc;
        acc += c[ww];
      }
    }
  } else if (NW * P > 16 && threadIdx.x < 64) {  // many waves: the counts re-read from LDS, not held in registers
    const int d0 = threadIdx.x * P;
    int32_t sum = 0;
#pragma unroll
    for (int i = 0; i < P; i++)
#pragma unroll
      for (int ww = 0; ww < NW; ww++) sum += s.run[ww][d0 + i];
    int32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(inc, o, 64);
      if (threadIdx.x >= o) inc += y;
    }
    int32_t acc = inc - sum;
    if constexpr (D == 64) {
      s.dbase[d0] = acc;
      if (d0 == 63) s.dbase[64] = inc;
    }
#pragma unroll
    for (int i = 0; i < P; i++)
#pragma unroll
      for (int ww = 0; ww < NW; ww++) {
        const int32_t v = s.run[ww][d0 + i];
        s.run[ww][d0 + i] = acc;
        acc += v;
      }
  } else if (threadIdx.x < 64) {  // lane d: digits d*P .. d*P + P - 1
    const int d0 = threadIdx.x * P;
    int32_t r[P][NW], sum = 0;
#pragma unroll
    for (int i = 0; i < P; i++)
#pragma unroll
      for (int ww = 0; ww < NW; ww++) {
        r[i][ww] = s.run[ww][d0 + i];
        sum += r[i][ww];
      }
    int32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(inc, o, 64);
      if (threadIdx.x >= o) inc += y;
    }
    int32_t acc = inc - sum;
    if constexpr (D == 64) {
      s.dbase[d0] = acc;
      if (d0 == 63) s.dbase[64] = inc;
    }
#pragma unroll
    for (int i = 0; i < P; i++)
#pragma unroll
      for (int ww = 0; ww < NW; ww++) {
        s.run[ww][d0 + i] = acc;
        acc += r[i][ww];
      }
  }
  ot_sync<NW>();
#pragma unroll
  for (int j = 0; j < IT; j++) pos[j] += s.run[w][dg[j]];
}

// Stable sort of n packed words (offset << 12 | index) held as items by
// digits of rel = offset - lo: `passes` (1 or 2) passes of log2(D) bits from
// bit sh of rel up (the second from bit sh2 when given: overlapping digits
// still sort by rel, the last pass deciding); the sorted words end in
// pk[0..n).  Ends synchronised.
template <int NW, int D, bool RUNS = false, int IB = kOtIdxBits, int IT = kOtItems>  // IB: bits below the offset; IT: items per thread
__device__ __forceinline__ void ot_sort(uint32_t (&key)[IT], int n, uint32_t lo, int sh, int passes,
                                        uint32_t* pk, OtRank<NW, D>& s, int sh2 = -1) {
  constexpr int B = D == 64 ? 6 : 8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ebase = w * (64 * IT);
  uint32_t dg[IT];
  int32_t pos[IT];
#pragma unroll
  for (int j = 0; j < IT; j++) dg[j] = (((key[j] >> IB) - lo) >> sh) & uint32_t(D - 1);
  ot_rank<NW, D, RUNS, IT>(dg, n, pos, s);
#pragma unroll
  for (int j = 0; j < IT; j++)
    if (ebase + j * 64 + lane < n) pk[pos[j]] = key[j];
  ot_sync<NW>();
  if (passes == 1) return;
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int e = ebase + j * 64 + lane;
    key[j] = e < n ? pk[e] : 0u;
    dg[j] = (((key[j] >> IB) - lo) >> (sh2 >= 0 ? sh2 : sh + B)) & uint32_t(D - 1);
  }
  ot_rank<NW, D, false, IT>(dg, n, pos, s);  // its first barrier orders the reloads before the stores below
#pragma unroll
  for (int j = 0; j < IT; j++)
    if (ebase + j * 64 + lane < n) pk[pos[j]] = key[j];
  ot_sync<NW>();
}

// pk[p - 1] for the element p this lane holds, where a wave's lanes hold
// consecutive elements: the left lane's v by DPP (wave_shr:1, no LDS access),
// lane 0 reads LDS (p > 0)
__device__ __forceinline__ uint32_t ot_prev(const uint32_t* pk, int p, uint32_t v) {
  uint32_t u = uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x138, 0xf, 0xf, false));  // wave_shr:1
  if ((threadIdx.x & 63) == 0 && p > 0) u = pk[p - 1];
  return u;
}

// two neighbours u, v of a sorted chunk (packed offset << 12 | index, rules in
// rl by index) out of (time, rule) order: a rule fires once per second, so
// equal offsets need strictly ascending rules
__device__ __forceinline__ bool ot_out_of_order(uint32_t u, uint32_t v, const int32_t* rl) {
  const uint32_t a = u >> kOtIdxBits, b = v >> kOtIdxBits;
  return a > b || (a == b && rl[u & kOtIdxMask] >= rl[v & kOtIdxMask]);
}

#ifndef CG_OT_TILE_WPE
#define CG_OT_TILE_WPE 6  // min waves per SIMD of the packed tile sort (its LDS allows 9 blocks per CU)
#endif
// PACK (rule indices < 2^kOtRuleBits): the sorted words are offset << 20 |
// rule, so no rule array in LDS (17 KB per block instead of 34: more blocks
// per CU); the sorts are stable, so the rule-major order inside a slab (and
// the rule order of equal offsets) carries through without the index.
// IN: 0 int64 times (their low words read) + rules, 1 16-bit offsets
// t - t0 - 1 + rules, 2 packed words offset << 20 | rule (in `rule`).
// PACK: the output is the packed words too (in rule_out; toff_out unused).
template <int IN, bool PACK>
__global__ __launch_bounds__(256, PACK ? CG_OT_TILE_WPE : 4) void k_ot_tile(const int64_t* __restrict__ time, const int32_t* __restrict__ rule,
                                                  const int32_t* __restrict__ tile_node,
                                                  const int64_t* __restrict__ tile_base,
                                                  const int64_t* __restrict__ node_off, int64_t t0,
                                                  uint16_t* __restrict__ toff_out, int32_t* __restrict__ rule_out,
                                                  int32_t* __restrict__ pre, const int64_t* __restrict__ n_tiles,
                                                  int64_t* __restrict__ err, int sb,
                                                  const int64_t* __restrict__ ts_start) {
  constexpr int IB = PACK ? kOtRuleBits : kOtIdxBits;
  constexpr uint32_t kLow = (1u << IB) - 1u;
  __shared__ OtRank<4, 64> s;
  __shared__ uint32_t pk[kOtTile];
  __shared__ int32_t rl[PACK ? 1 : kOtTile];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t t = blockIdx.x;
  if (t >= *n_tiles) return;  // the grid may be an upper bound (pipelined windows)
  const TileRange r{ts_start[t], ts_start[t + 1]};  // never more than kOtTile events
  const int n = int(r.hi - r.lo);
  const int ebase = w * (64 * kOtItems);
  const uint32_t* __restrict__ tlo = reinterpret_cast<const uint32_t*>(time);  // low words: offsets < 4096
  const uint32_t b = uint32_t(t0 + 1);
  uint32_t key[kOtItems], tv[kOtItems];
  int32_t rv[kOtItems];
#pragma unroll
  for (int j = 0; j < kOtItems; j++) {  // every load issued before any is used
    const int e = ebase + j * 64 + lane;
    const int64_t i = r.lo + (e < n ? e : n - 1);
    if constexpr (IN == 1) tv[j] = uint32_t(reinterpret_cast<const uint16_t*>(time)[i]) + b;
    else if constexpr (IN == 0) tv[j] = tlo[2 * i];
    rv[j] = rule[i];
  }
  if constexpr (IN == 2) {
#pragma unroll
    for (int j = 0; j < kOtItems; j++) {
      tv[j] = (uint32_t(rv[j]) >> kOtRuleBits) + b;
      rv[j] = int32_t(uint32_t(rv[j]) & ((1u << kOtRuleBits) - 1u));
    }
  }
#pragma unroll
  for (int j = 0; j < kOtItems; j++) {
    const int e = ebase + j * 64 + lane;
    if constexpr (PACK) {
      key[j] = e < n ? ((tv[j] - b) << IB) | uint32_t(rv[j]) : 0u;
    } else {
      key[j] = e < n ? ((tv[j] - b) << IB) | uint32_t(e) : 0u;
      if (e < n) rl[e] = rv[j];
    }
  }
  // by slab (offset >> sb); a node's only tile by the whole offset: bits 0..5,
  // then its last pass by the slab (offset >> sb: the pre row's digits)
  const int32_t nd = tile_node[t];
  const bool one = tile_base[nd + 1] - tile_base[nd] == 1;
  if (one) ot_sort<4, 64, false, IB>(key, n, 0u, 0, 2, pk, s, sb);
  else ot_sort<4, 64, true, IB>(key, n, 0u, sb, 1, pk, s);
  int32_t* __restrict__ pt = pre + t * kOtPre;
  if (threadIdx.x <= 64) pt[threadIdx.x] = s.dbase[threadIdx.x];  // slabs = the last pass's digits
  auto rule_of = [&](uint32_t v) { return PACK ? int32_t(v & kLow) : rl[v & kLow]; };
  bool bad = false;
  for (int p = threadIdx.x; p < n; p += 256) {
    const uint32_t v = pk[p];
    if constexpr (PACK) {
      __builtin_nontemporal_store(int32_t(v), rule_out + r.lo + p);  // the word itself: offset << 20 | rule
    } else {
      toff_out[r.lo + p] = uint16_t(v >> IB);
      __builtin_nontemporal_store(rule_of(v), rule_out + r.lo + p);
    }
    // the ranks rest on lane-ordered LDS atomics (ot_rank): check the order
    // they produced -- a node's only tile is final: (offset, rule) ascending;
    // a partitioned tile keeps rule order inside each slab
    const uint32_t u = ot_prev(pk, p, v);
    if (p > 0) {
      const int32_t ru = rule_of(u), rv2 = rule_of(v);
      const uint32_t ou = u >> IB, ov = v >> IB;
      if (one) bad |= ou > ov || (ou == ov && ru >= rv2);
      else if ((ou >> sb) == (ov >> sb)) bad |= ru > rv2 || (ru == rv2 && ou >= ov);  // rule-major
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull);
}

// Exclusive scan of cnt(q) for q in [0, Q) (Q <= kOtMaxTiles) into ps[0..Q]
// (ps[Q] = total); src(q) into psrc.  Ends synchronised.
template <int NW, class Portion>
__device__ __forceinline__ void ot_portions(int Q, Portion&& portion, int32_t* ps, int32_t* psrc, int32_t* wsum) {
  constexpr int PER = (kOtMaxTiles + 64 * NW - 1) / (64 * NW);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t c[PER], sum = 0;
#pragma unroll
  for (int i = 0; i < PER; i++) {
    const int q = threadIdx.x * PER + i;
    c[i] = 0;
    if (q < Q) {
      int32_t src;
      c[i] = portion(q, &src);
      psrc[q] = src;
    }
    sum += c[i];
  }
  int32_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  int32_t run = inc - sum;
  if constexpr (NW > 1) {
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    for (int ww = 0; ww < w; ww++) run += wsum[ww];
  }
#pragma unroll
  for (int i = 0; i < PER; i++) {
    const int q = threadIdx.x * PER + i;
    if (q < Q) ps[q] = run;
    run += c[i];
  }
  if (threadIdx.x == 64 * NW - 1) ps[Q] = run;
  ot_sync<NW>();
}

// the portion holding element e of the list (ps ascending, ps[0] = 0)
__device__ __forceinline__ int ot_find(const int32_t* ps, int Q, int32_t e) {
  int lo = 0, hi = Q - 1;  // the last q with ps[q] <= e
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (ps[mid] <= e) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// own[i] = the portion holding element c0 + i of the list, i < n_el <= the
// chunk: every non-empty portion marks its first element and an inclusive
// max-scan fills the rest (portion indices grow with position), so no
// element searches.  own is padded (element i at i + i / 32) so the scan's
// per-thread runs of kOtItems do not collide in the LDS banks.  Ends
// synchronised.
__device__ __forceinline__ int ot_pad(int i) { return i + (i >> 5); }
template <int NW, int IT = kOtItems>
__device__ __forceinline__ void ot_owners(const int32_t* ps, int Q, int32_t c0, int n_el, int32_t* own,
                                          int32_t* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < n_el; i += 64 * NW) own[ot_pad(i)] = -1;
  ot_sync<NW>();
  for (int q = threadIdx.x; q < Q; q += 64 * NW) {
    const int32_t a = ps[q];
    if (a < ps[q + 1] && a >= c0 && a < c0 + n_el) own[ot_pad(a - c0)] = q;
  }
  if (threadIdx.x == 0) own[0] = ot_find(ps, Q, c0);  // the portion the chunk starts in (the same q if it starts at c0)
  ot_sync<NW>();
  int32_t v[IT], m = -1;
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const int idx = threadIdx.x * IT + i;
    v[i] = idx < n_el ? own[ot_pad(idx)] : -1;
    m = v[i] > m ? v[i] : m;
    v[i] = m;
  }
  int32_t inc = m;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc = y > inc ? y : inc;
  }
  int32_t prev = __shfl_up(inc, 1, 64);
  if (lane == 0) prev = -1;
  if constexpr (NW > 1) {
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    for (int ww = 0; ww < w; ww++) prev = wsum[ww] > prev ? wsum[ww] : prev;
  }
#pragma unroll
  for (int i = 0; i < IT; i++) {
    const int idx = threadIdx.x * IT + i;
    if (idx < n_el) own[ot_pad(idx)] = v[i] > prev ? v[i] : prev;
  }
  ot_sync<NW>();
}

// Items of elements c0 .. c0 + n_el of the portion list (sources relative
// to tin / rin, < 2^31; tin = the tile sort's 16-bit offsets): key =
// (offset << 12 | chunk index), rule into rl[chunk index] (RULES).  All loads
// issued before any is used (clamped indices).
// SEARCH: each element finds its portion by a binary search of ps (Q
// portions) instead of reading the owner map (no ot_owners pass)
// PACK: key = offset << kOtRuleBits | rule (rules < 2^kOtRuleBits), no rl
// SEARCH 2: the lane's first element finds its portion by a binary search,
// each later item (64 elements on) walks forward from there (portions are
// consecutive, so a few steps at most)
// BUF: the loads as raw buffer loads (32-bit offsets against a descriptor
// over n_src elements; an index past it reads 0): one VGPR per address
// instead of two, and no 64-bit address arithmetic per item
// PIN: the source is one array of packed words offset << 20 | rule (rin; tin
// unused), 4 B per event instead of 2 + 4
// HX (with PIN; rule indices past 2^20): the words hold rule & 0xFFFFF and
// portion q's tile adds ph[q] << 20.  PACK keys become (offset - hx_lo) << 24
// | rule (a run of at most 256 s: the key order is still the (time, rule)
// order); otherwise rl[] gets the whole rule
template <bool RULES, int SEARCH = 0, bool PACK = false, int IT = kOtItems, bool BUF = false, bool PIN = false,
          bool HX = false>
__device__ __forceinline__ void ot_gather(const uint16_t* __restrict__ tin, const int32_t* __restrict__ rin,
                                          const int32_t* ps, const int32_t* psrc, const int32_t* own,
                                          int32_t c0, int n_el, uint32_t (&key)[IT], int32_t* rl, int Q = 0,
                                          uint32_t n_src = 0, const int32_t* ph = nullptr, uint32_t hx_lo = 0) {
  static_assert(!HX || PIN, "high rule bits come with packed words");
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ebase = w * (64 * IT);
  uint32_t tv[IT];
  int32_t rv[IT];
  uint32_t hq[HX ? IT : 1];  // HX: the element's tile's rule >> 20, shifted
  __amdgpu_buffer_rsrc_t ra, rb;
  if constexpr (BUF) {
    constexpr int kRsrcWord3 = 0x00020000;  // gfx9 raw buffer: 32-bit data format, no swizzle
    ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(tin), 0, int(n_src * 2u), kRsrcWord3);
    rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<int32_t*>(rin), 0, int(n_src * 4u), kRsrcWord3);
  }
  int qw = 0, qa = 0, qb = 0, qs = 0;  // SEARCH 2: the current portion, its bounds ps[qw], ps[qw + 1], psrc[qw]
  if (SEARCH == 2) {
    const int e0 = ebase + lane < n_el ? ebase + lane : n_el - 1;
    qw = ot_find(ps, Q, c0 + e0);
    qa = ps[qw];
    qb = ps[qw + 1];
    qs = psrc[qw];
  }
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int e = ebase + j * 64 + lane;
    const int ec = e < n_el ? e : n_el - 1;
    int q;
    if (SEARCH == 2) {
      while (qb <= c0 + ec && qw + 1 < Q) {
        qw++;
        qa = qb;
        qb = ps[qw + 1];
        qs = psrc[qw];
      }
      q = qw;
    } else {
      q = SEARCH ? ot_find(ps, Q, c0 + ec) : own[ot_pad(ec)];
    }
    const uint32_t src = SEARCH == 2 ? uint32_t(qs + (c0 + ec - qa)) : uint32_t(psrc[q] + (c0 + ec - ps[q]));
    if constexpr (HX) hq[j] = uint32_t(ph[q]) << kOtRuleBits;
    if constexpr (PIN) {  // one word: split below
      rv[j] = BUF ? __builtin_amdgcn_raw_buffer_load_b32(rb, int(src * 4u), 0, 0) : rin[src];
    } else if constexpr (BUF) {
      tv[j] = __builtin_amdgcn_raw_buffer_load_b16(ra, int(src * 2u), 0, 0);
      if (RULES) rv[j] = __builtin_amdgcn_raw_buffer_load_b32(rb, int(src * 4u), 0, 0);
    } else {
      tv[j] = tin[src];
      if (RULES) rv[j] = rin[src];
    }
  }
  if constexpr (PIN) {
#pragma unroll
    for (int j = 0; j < IT; j++) {
      tv[j] = uint32_t(rv[j]) >> kOtRuleBits;
      rv[j] = int32_t(uint32_t(rv[j]) & ((1u << kOtRuleBits) - 1u));
    }
  }
#pragma unroll
  for (int j = 0; j < IT; j++) {
    const int e = ebase + j * 64 + lane;
    if constexpr (HX) {
      if (PACK) {
        key[j] = e < n_el ? ((tv[j] - hx_lo) << (kOtRuleBits + kOtHiBits)) | hq[j] | uint32_t(rv[j]) : 0u;
      } else {
        key[j] = e < n_el ? (tv[j] << kOtIdxBits) | uint32_t(e) : 0u;
        if (RULES && e < n_el) rl[e] = int32_t(hq[j] | uint32_t(rv[j]));
      }
    } else if (PACK) {
      key[j] = e < n_el ? (tv[j] << kOtRuleBits) | uint32_t(rv[j]) : 0u;
    } else {
      key[j] = e < n_el ? (tv[j] << kOtIdxBits) | uint32_t(e) : 0u;
      if (RULES && e < n_el) rl[e] = rv[j];
    }
  }
}

// Per node: the first node-relative position of each slab (events of the
// earlier slabs over all its tiles), slab_off[n][0..kOtSlabs].  One wave per
// node, kOtSlabs / 64 slabs per lane.
__global__ __launch_bounds__(64) void k_ot_slabs(const int64_t* __restrict__ tile_base,
                                                  const int32_t* __restrict__ pre, int32_t N,
                                                  int64_t* __restrict__ slab_off) {
  constexpr int kSpl = kOtSlabs / 64;
  const int lane = threadIdx.x;
  const int32_t n = blockIdx.x;
  if (n >= N) return;
  const int64_t ta = tile_base[n], M = tile_base[n + 1] - ta;
  int64_t c[kSpl];
#pragma unroll
  for (int i = 0; i < kSpl; i++) c[i] = 0;
  for (int64_t t = ta; t < ta + M; t++) {
    const int32_t* pt = pre + t * kOtPre + kSpl * lane;
    int32_t p[kSpl + 1];
#pragma unroll
    for (int i = 0; i <= kSpl; i++) p[i] = pt[i];
#pragma unroll
    for (int i = 0; i < kSpl; i++) c[i] += p[i + 1] - p[i];
  }
  int64_t sum = 0;
#pragma unroll
  for (int i = 0; i < kSpl; i++) sum += c[i];
  int64_t inc = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  int64_t run = inc - sum;
  int64_t* so = slab_off + int64_t(n) * kOtPre;
#pragma unroll
  for (int i = 0; i < kSpl; i++) {
    so[kSpl * lane + i] = run;
    run += c[i];
  }
  if (lane == 63) so[kOtSlabs] = run;
}

#ifndef CG_OT_MID_WPE
#define CG_OT_MID_WPE 4  // min waves per SIMD of k_ot_mid (8-wave blocks: 2 per SIMD each)
#endif
#ifndef CG_OT_MERGE_WPE
#define CG_OT_MERGE_WPE 4  // min waves per SIMD of the packed merge (its LDS allows 6 blocks per CU)
#endif
#ifndef CG_OT_DENSE_WPE
#define CG_OT_DENSE_WPE 4  // the same for the dense nodes' merge (the persistent 8-wave grid)
#endif

// One chunk of n_el <= 64 * NW * kOtItems events of a node (tin_n / rin_n:
// the node's tile-sorted offsets and rules): the M tiles' portions
// (portion(q, &src) -> count, thread q's tile; src node-relative), gathered,
// sorted in LDS by rel = offset - lo (`passes` 8-bit passes) and stored at
// tout_o / rout_o in (time, rule) order.  n_src: the node's events (M <=
// kOtMaxTiles tiles).  HX: rules past 2^20 (portion q's tile adds ph[q] <<
// 20; keys rel << 24 | rule, one pass: rel < 256).  Ends synchronised.
template <int NW, bool PACK, int IT, bool PIN, bool HX, class Portion>
__device__ __forceinline__ void ot_merge_chunk(const uint16_t* __restrict__ tin_n, const int32_t* __restrict__ rin_n,
                                               int M, int n_el, uint32_t lo, int passes, Portion&& portion,
                                               int64_t t0, int64_t* __restrict__ tout_o,
                                               int32_t* __restrict__ rout_o, OtRank<NW, 256>& s, uint32_t* pk,
                                               int32_t* rl, int32_t* ps, int32_t* psrc, int32_t* wsum,
                                               int64_t* __restrict__ err, uint32_t n_src, const int32_t* ph) {
  int32_t* own = reinterpret_cast<int32_t*>(pk);
  uint32_t key[IT];
  ot_portions<NW>(M, portion, ps, psrc, wsum);
  // each element's portion by search + walk, raw buffer loads
  ot_gather<true, 2, PACK, IT, true, PIN, HX>(tin_n, rin_n, ps, psrc, own, 0, n_el, key, rl, M, n_src, ph, lo);
  constexpr int IB = HX ? kOtRuleBits + kOtHiBits : (PACK ? kOtRuleBits : kOtIdxBits);
  ot_sort<NW, 256, false, IB, IT>(key, n_el, HX ? 0u : lo, 0, passes, pk, s);
  const int64_t tb = t0 + 1 + (HX ? int64_t(lo) : 0);
  constexpr uint32_t kRuleMask = HX ? (1u << (kOtRuleBits + kOtHiBits)) - 1u : kOtLowMask;
  bool bad = false;
  for (int p = threadIdx.x; p < n_el; p += 64 * NW) {
    const uint32_t v = pk[p];
    __builtin_nontemporal_store(tb + int64_t(v >> IB), tout_o + p);
    if (PACK) {
      __builtin_nontemporal_store(int32_t(v & kRuleMask), rout_o + p);
      const uint32_t u = ot_prev(pk, p, v);
      if (p > 0) bad |= u >= v;  // (time, rule) order of the chunk: the words ascend
    } else {
      __builtin_nontemporal_store(rl[v & kOtIdxMask], rout_o + p);
      const uint32_t u = ot_prev(pk, p, v);
      if (p > 0) bad |= ot_out_of_order(u, v, rl);  // (time, rule) order of the chunk
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull);
  ot_sync<NW>();
}

// Per node with e_lo <= events < e_hi: its slabs in runs that fit one chunk,
// each merged by ot_merge_chunk.  Two launches split the nodes by density:
// 4-wave blocks (4096-event chunks) for nodes averaging at most
// CG_OT_DENSE_PER_SLAB events per slab, 8-wave blocks (8192; a persistent
// grid taking nodes by ticket, on its own stream beside the 4-wave launch)
// for denser ones (same-box A/Bs, profiles/r04_ab_merge_shape.txt: 8-wave
// chunks for every node are 6-9 % faster on config 3's ~4.6 k events per
// slab and 11-13 % slower on pernode's ~1.6 k; the split at 4096 took
// config 3 from ~600 to 555 ms per step and left pernode unchanged; with the
// all-thread rank scan (no spills in the 8-wave merge) a split at 2048 is
// 1.6 % faster on pernode and equal on config 3, profiles/r04_ab_dense_2048.txt).  A slab of more than a chunk is queued: to k_ot_mid when it
// fits k_ot_mid's chunk (mid / mid_n), else to k_ot_big (big / big_n);
// entries (node << 8 | slab).
// HX: rule indices past 2^20 (tiles cut where rule >> 20 changes, ts_hi per
// tile): runs of at most 256 s, so a key holds rel << 24 | rule.
template <int NW, bool PACK, int IT = kOtItems, bool DYN = false, bool PIN = false, bool HX = false>  // DYN: nodes by ticket (persistent grid)
__global__ __launch_bounds__(64 * NW, PACK ? (DYN ? CG_OT_DENSE_WPE : CG_OT_MERGE_WPE) : 4) void k_ot_merge(const uint16_t* __restrict__ tin, const int32_t* __restrict__ rin,
                                                       const int64_t* __restrict__ tile_base,
                                                       const int64_t* __restrict__ node_off,
                                                       const int32_t* __restrict__ pre, int32_t N, int64_t t0,
                                                       const int64_t* __restrict__ slab_tab,
                                                       int64_t* __restrict__ tout, int32_t* __restrict__ rout,
                                                       int64_t* __restrict__ big, unsigned* __restrict__ big_n,
                                                       int64_t* __restrict__ mid, unsigned* __restrict__ mid_n,
                                                       int64_t* __restrict__ mid2, unsigned* __restrict__ mid2_n,
                                                       int64_t e_lo, int64_t e_hi, unsigned* __restrict__ ticket,
                                                       int64_t* __restrict__ err, int sb,
                                                       const int64_t* __restrict__ ts_start,
                                                       const int32_t* __restrict__ ts_hi) {
  constexpr int kThreads = 64 * NW, kChunk = kThreads * IT;
  constexpr int kMidChunk = 64 * kOtMidWaves * kOtItems, kMid2Chunk = 64 * kOtMid2Waves * kOtItems;
  __shared__ OtRank<NW, 256> s;
  __shared__ int32_t ph[HX ? kOtMaxTiles : 1];  // HX: rule >> 20 of tile q
  __shared__ uint32_t pk[kChunk + kChunk / 32];  // the owner list while gathering (padded), then the sorted words
  __shared__ int32_t rl[PACK ? 1 : kChunk];
  __shared__ int32_t ps[kOtMaxTiles + 1];
  __shared__ int32_t psrc[kOtMaxTiles];       // node-relative (M <= kOtMaxTiles: < 2^20)
  __shared__ int64_t slab_off[kOtSlabs + 1];  // node-relative first position of each slab
  __shared__ int32_t wsum[NW];
  __shared__ int32_t tk;
  auto next = [&]() -> int32_t {  // DYN: the next node by ticket, once every thread is done with the last
    if (!DYN) return N;
    ot_sync<NW>();
    if (threadIdx.x == 0) tk = int32_t(atomicAdd(ticket, 1u));
    ot_sync<NW>();
    return tk;
  };
  for (int32_t n = DYN ? next() : int32_t(blockIdx.x); n < N; n = next()) {
  const int64_t ta = tile_base[n], M = tile_base[n + 1] - ta, lo_n = node_off[n];
  if (M == 0) continue;
  const int64_t e_n = node_off[n + 1] - lo_n;
  if (e_n < e_lo || e_n >= e_hi) continue;  // the other merge launch's node
  if (M == 1) {  // one tile: already in order
    const uint32_t hi = HX ? uint32_t(ts_hi[ta]) << kOtRuleBits : 0u;
    for (int64_t p = threadIdx.x; p < e_n; p += kThreads) {
      const uint32_t w = uint32_t(rin[lo_n + p]);  // PIN: a packed word
      const int64_t off = PIN ? int64_t(w >> kOtRuleBits) : int64_t(tin[lo_n + p]);
      __builtin_nontemporal_store(t0 + 1 + off, tout + lo_n + p);
      __builtin_nontemporal_store(PIN ? int32_t(hi | (w & kOtLowMask)) : int32_t(w), rout + lo_n + p);
    }
    continue;
  }
  if (M > kOtMaxTiles) {  // every slab to k_ot_big
    for (int j = threadIdx.x; j < kOtSlabs; j += kThreads) big[atomicAdd(big_n, 1u)] = (int64_t(n) << 8) | j;
    continue;
  }
  for (int j = threadIdx.x; j <= kOtSlabs; j += kThreads) slab_off[j] = slab_tab[int64_t(n) * kOtPre + j];
  if (HX && threadIdx.x < M) ph[threadIdx.x] = ts_hi[ta + threadIdx.x];
  ot_sync<NW>();
  // the longest run of whole slabs [j0, j1) that fits one chunk (j1 == j0: a
  // slab of more than a chunk); HX: and spans at most 256 s
  auto run_end = [&](int j0) {
    int j1 = j0;
    while (j1 < kOtSlabs && (!HX || ((j1 + 1 - j0) << sb) <= 256) && slab_off[j1 + 1] - slab_off[j0] <= kChunk)
      j1++;
    return j1;
  };
  // thread q owns tile q (M <= kOtMaxTiles <= threads): its slab prefix at the
  // run's ends is held in registers, the next run's end loaded one run ahead
  static_assert(kOtMaxTiles <= kThreads, "one tile per thread");
  const int q_own = threadIdx.x;
  const int32_t* __restrict__ pq = pre + (ta + (q_own < M ? q_own : 0)) * kOtPre;
  const int32_t qs = int32_t(ts_start[ta + (q_own < M ? q_own : 0)] - lo_n);  // tile q's first event, node-relative
  int ja = 0, jb = run_end(0);
  int32_t pa = pq[0], pb = pq[jb];
  while (ja < kOtSlabs) {
    const int ja2 = jb == ja ? ja + 1 : jb;
    const int jb2 = ja2 < kOtSlabs ? run_end(ja2) : ja2;
    const int32_t pa2 = jb == ja ? pq[ja2 <= kOtSlabs ? ja2 : kOtSlabs] : pb;
    const int32_t pb2 = pq[jb2 <= kOtSlabs ? jb2 : kOtSlabs];  // in flight while this run is merged
    if (jb == ja) {  // one slab of more than a chunk
      if (threadIdx.x == 0) {
        const int64_t sz = slab_off[ja + 1] - slab_off[ja];
        if (sz <= kMidChunk) mid[atomicAdd(mid_n, 1u)] = (int64_t(n) << 8) | ja;
        else if (sz <= kMid2Chunk) mid2[atomicAdd(mid2_n, 1u)] = (int64_t(n) << 8) | ja;
        else big[atomicAdd(big_n, 1u)] = (int64_t(n) << 8) | ja;
      }
    } else if (slab_off[jb] > slab_off[ja]) {
      // per tile its sorted events of slabs [ja, jb): one contiguous range; by
      // rel = offset - the run's first second (< 64 * (jb - ja)): one 8-bit
      // pass for up to 4 slabs
      const int64_t o = lo_n + slab_off[ja];
      ot_merge_chunk<NW, PACK, IT, PIN, HX>(
          tin + lo_n, rin + lo_n, int(M), int(slab_off[jb] - slab_off[ja]), uint32_t(ja) << sb,
          ((jb - ja) << sb) > 256 ? 2 : 1,
          [&](int q, int32_t* src) {
            *src = qs + pa;  // q == q_own
            return pb - pa;
          },
          t0, tout + o, rout + o, s, pk, rl, ps, psrc, wsum, err, uint32_t(e_n), ph);
    }
    ja = ja2;
    jb = jb2;
    pa = pa2;
    pb = pb2;
  }
  }
}

// The slabs k_ot_merge queued for a bigger chunk (more than its own, at most
// 64 * kOtMidWaves * kOtItems events), one per workgroup turn: the same
// gather + one-pass LDS sort with NW waves (a slab of 64 s: one 8-bit pass).
template <int NW, bool PACK, int IT = kOtItems, bool PIN = false, bool HX = false>
__global__ __launch_bounds__(64 * NW, CG_OT_MID_WPE) void k_ot_mid(const uint16_t* __restrict__ tin, const int32_t* __restrict__ rin,
                                                    const int64_t* __restrict__ tile_base,
                                                    const int64_t* __restrict__ node_off,
                                                    const int32_t* __restrict__ pre, int64_t t0,
                                                    const int64_t* __restrict__ slab_tab,
                                                    int64_t* __restrict__ tout, int32_t* __restrict__ rout,
                                                    const int64_t* __restrict__ mid,
                                                    const unsigned* __restrict__ mid_n, int64_t* __restrict__ err,
                                                    int sb, const int64_t* __restrict__ ts_start,
                                                    const int32_t* __restrict__ ts_hi) {
  constexpr int kChunk = 64 * NW * IT;
  __shared__ OtRank<NW, 256> s;
  __shared__ int32_t ph[HX ? kOtMaxTiles : 1];
  __shared__ uint32_t pk[kChunk + kChunk / 32];
  __shared__ int32_t rl[PACK ? 1 : kChunk];
  __shared__ int32_t ps[kOtMaxTiles + 1];
  __shared__ int32_t psrc[kOtMaxTiles];
  __shared__ int32_t wsum[NW];
  static_assert(kOtMaxTiles <= 64 * NW, "one tile per thread");
  const unsigned nm = *mid_n;
  for (unsigned task = blockIdx.x; task < nm; task += gridDim.x) {
    const int64_t e = mid[task];
    const int32_t n = int32_t(e >> 8);
    const int j = int(e & 255);
    const int64_t ta = tile_base[n], M = tile_base[n + 1] - ta, lo_n = node_off[n];
    const int64_t* so = slab_tab + int64_t(n) * kOtPre;
    const int64_t a = so[j], n_el = so[j + 1] - a;
    if (n_el <= 0 || n_el > kChunk || M > kOtMaxTiles) {  // never queued so
      if (threadIdx.x == 0) atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull);
      continue;
    }
    if (HX && threadIdx.x < M) ph[threadIdx.x] = ts_hi[ta + threadIdx.x];
    ot_merge_chunk<NW, PACK, IT, PIN, HX>(
        tin + lo_n, rin + lo_n, int(M), int(n_el), uint32_t(j) << sb, 1,
        [&](int q, int32_t* src) {
          const int32_t* pt = pre + (ta + q) * kOtPre;
          *src = int32_t(ts_start[ta + q] - lo_n) + pt[j];
          return pt[j + 1] - pt[j];
        },
        t0, tout + lo_n + a, rout + lo_n + a, s, pk, rl, ps, psrc, wsum, err,
        uint32_t(node_off[n + 1] - lo_n), ph);
  }
}

// The slabs k_ot_merge queued, one per workgroup turn: the slab's
// histogram of its 16 seconds over all its portions first, then its chunks
// in order, each sorted in LDS and stored at its seconds' running bases.
template <bool PIN, bool HX = false>
__global__ __launch_bounds__(256) void k_ot_big(const uint16_t* __restrict__ tin, const int32_t* __restrict__ rin,
                                                 const int64_t* __restrict__ tile_base,
                                                 const int64_t* __restrict__ node_off,
                                                 const int32_t* __restrict__ pre, int64_t t0,
                                                 int64_t* __restrict__ tout, int32_t* __restrict__ rout,
                                                 const int64_t* __restrict__ big, const unsigned* __restrict__ big_n,
                                                 int64_t* __restrict__ err, int sb, const int64_t* __restrict__ ts_start,
                                                 const int32_t* __restrict__ ts_hi) {
  __shared__ OtRank<4, 64> s;
  __shared__ int32_t ph[HX ? kOtMaxTiles : 1];
  __shared__ uint32_t pk[kOtTile + kOtTile / 32];
  __shared__ int32_t rl[kOtTile];
  __shared__ int32_t ps[kOtMaxTiles + 1];
  __shared__ int32_t psrc[kOtMaxTiles];  // relative to the group's first tile
  __shared__ int64_t gbase[64];
  __shared__ int32_t hist[64];
  __shared__ int32_t wsum[4];
  __shared__ int64_t red[4];
  int32_t* own = reinterpret_cast<int32_t*>(pk);
  const int lane = threadIdx.x & 63, ebase = (threadIdx.x >> 6) * (64 * kOtItems);
  const uint32_t kSec = (1u << sb) - 1u;  // seconds of a slab
  const unsigned nb = *big_n;
  for (unsigned task = blockIdx.x; task < nb; task += gridDim.x) {
    const int32_t n = int32_t(big[task] >> 8);
    const int j = int(big[task] & 255);
    const int64_t ta = tile_base[n], M = tile_base[n + 1] - ta, lo_n = node_off[n];
    // portions of tiles [ga, ga + gm): per tile its events of slab j,
    // sources relative to tile ga's first event
    auto list = [&](int64_t ga, int64_t gm) {
      if (HX && threadIdx.x < gm) ph[threadIdx.x] = ts_hi[ta + ga + threadIdx.x];
      const int64_t g0 = ts_start[ta + ga];
      ot_portions<4>(
          int(gm),
          [&](int q, int32_t* src) {
            const int32_t* pt = pre + (ta + ga + q) * kOtPre;
            *src = int32_t(ts_start[ta + ga + q] - g0) + pt[j];
            return pt[j + 1] - pt[j];
          },
          ps, psrc, wsum);
      return int(gm);
    };
    // the slab's first position: events of earlier slabs over the node's tiles
    int64_t before = 0;
    for (int64_t t = ta + threadIdx.x; t < ta + M; t += 256) before += pre[t * kOtPre + j];
#pragma unroll
    for (int o = 32; o; o >>= 1) before += __shfl_xor(before, o, 64);
    if (lane == 0) red[threadIdx.x >> 6] = before;
    if (threadIdx.x < 64) hist[threadIdx.x] = 0;
    __syncthreads();
    const int64_t slab_lo = lo_n + red[0] + red[1] + red[2] + red[3];
    uint32_t key[kOtItems];
    for (int64_t ga = 0; ga < M; ga += kOtMaxTiles) {  // histogram of the slab's seconds
      const int Q = list(ga, M - ga < kOtMaxTiles ? M - ga : kOtMaxTiles);
      const int32_t n_grp = ps[Q];
      for (int32_t c0 = 0; c0 < n_grp; c0 += kOtTile) {
        const int n_el = n_grp - c0 < kOtTile ? int(n_grp - c0) : kOtTile;
        ot_owners<4>(ps, Q, c0, n_el, own, wsum);
        const int64_t g0 = ts_start[ta + ga];
        ot_gather<false, 0, false, kOtItems, false, PIN, HX>(tin + g0, rin + g0, ps, psrc, own, c0, n_el, key, rl, 0,
                                                             0, ph);
#pragma unroll
        for (int jj = 0; jj < kOtItems; jj++)
          if (ebase + jj * 64 + lane < n_el) atomicAdd(&hist[(key[jj] >> kOtIdxBits) & kSec], 1);
        __syncthreads();
      }
    }
    if (threadIdx.x < 64) {
      const int d = threadIdx.x;
      const int64_t c = hist[d];
      int64_t inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(inc, o, 64);
        if (d >= o) inc += y;
      }
      gbase[d] = slab_lo + inc - c;
    }
    __syncthreads();
    for (int64_t ga = 0; ga < M; ga += kOtMaxTiles) {  // chunks in order, each second at its running base
      const int Q = list(ga, M - ga < kOtMaxTiles ? M - ga : kOtMaxTiles);
      const int32_t n_grp = ps[Q];
      for (int32_t c0 = 0; c0 < n_grp; c0 += kOtTile) {
        const int n_el = n_grp - c0 < kOtTile ? int(n_grp - c0) : kOtTile;
        ot_owners<4>(ps, Q, c0, n_el, own, wsum);
        const int64_t g0 = ts_start[ta + ga];
        ot_gather<true, 0, false, kOtItems, false, PIN, HX>(tin + g0, rin + g0, ps, psrc, own, c0, n_el, key, rl, 0, 0,
                                                            ph);
        ot_sort<4, 64, false>(key, n_el, uint32_t(j) << sb, 0, 1, pk, s);
        bool bad = false;
        for (int p = threadIdx.x; p < n_el; p += 256) {
          const uint32_t v = pk[p];
          const uint32_t d = (v >> kOtIdxBits) & kSec;
          const int64_t dst = gbase[d] + (p - s.dbase[d]);
          tout[dst] = t0 + 1 + int64_t(v >> kOtIdxBits);
          rout[dst] = rl[v & kOtIdxMask];
          if (p > 0) bad |= ot_out_of_order(pk[p - 1], v, rl);
        }
        if (__ballot(bad) && lane == 0) atomicOr(reinterpret_cast<unsigned long long*>(err), 1ull);
        __syncthreads();
        if (threadIdx.x < 64) gbase[threadIdx.x] += s.dbase[threadIdx.x + 1] - s.dbase[threadIdx.x];
        __syncthreads();
      }
    }
  }
}

int gridn(int64_t n, int threads) { return int(std::max<int64_t>(1, (n + threads - 1) / threads)); }


}  // namespace

// Windows <= 4096 s, in three steps enqueued on st with no host sync (buffers
// sized from the output capacity cap, grids upper bounds trimmed on the
// device): order_setup (node-aligned tiles from the node offsets), the tiles
// (k_ot_tile over the writer's lists), order_tail (slab offsets, k_ot_merge, k_ot_big).
namespace {

int order_setup(cg_ctx* c, const int64_t* node_off, int32_t N, int64_t cap, hipStream_t st, int64_t* Tmax,
                const OtCut& cut) {
  *Tmax = cap / kOtTile + int64_t(N) * cut.H + 1;
  const int64_t toff_words = (cap + 3) / 4;  // 16-bit offsets in the int64 second buffer
  // ts_off: [k_ot_big queue N*kOtSlabs][big, mid, dense-node, mid2 counters: 2 words][slab_tab N*kOtPre]
  // [k_ot_mid queue N*kOtSlabs][its 16-wave form's queue N*kOtSlabs]
  const int64_t tab = 3 * int64_t(N) * kOtSlabs + 2 + int64_t(N) * kOtPre;
  // growing a buffer frees the old one: earlier windows' kernels finish first
  if (c->ts_cnt.cap < size_t(N) || c->ts_base.cap < size_t(N + 1) || c->ts_tile_node.cap < size_t(*Tmax) ||
      c->ts_hist.cap < size_t(*Tmax * kOtPre) || c->node_time2.cap < size_t(toff_words) ||
      c->node_rule2.cap < size_t(cap) || c->ts_off.cap < size_t(tab) || c->scan_tmp.cap < scan_temp_bytes(N) ||
      c->ts_start.cap < size_t(*Tmax + 1) || c->ts_hi.cap < size_t(*Tmax))
    HIPCHK(hipStreamSynchronize(st));
  int rc;
  if ((rc = c->ts_cnt.ensure(N)) || (rc = c->ts_base.ensure(int64_t(N) + 1)) || (rc = c->ts_tile_node.ensure(*Tmax)) ||
      (rc = c->ts_hist.ensure(*Tmax * kOtPre)) || (rc = c->node_time2.ensure(toff_words)) ||
      (rc = c->node_rule2.ensure(cap)) || (rc = c->ts_off.ensure(tab)) || (rc = c->ts_start.ensure(*Tmax + 1)) ||
      (rc = c->ts_hi.ensure(*Tmax)) || (rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(N)))))
    return rc;
  hipLaunchKernelGGL(k_ot_tile_count, dim3(gridn(N, 256)), dim3(256), 0, st, node_off, N, cap, cut, c->ts_cnt.p);
  launch_scan(c->ts_cnt.p, c->ts_base.p, N, c->scan_tmp.p, st);
  hipLaunchKernelGGL(k_ot_tiles, dim3(gridn(N, 256)), dim3(256), 0, st, c->ts_base.p, node_off, N, cut,
                     c->ts_tile_node.p, c->ts_start.p, c->ts_hi.p);
  return cg_hip_check(hipGetLastError(), "time-order tiles");
}

// Slab width 2^sb seconds for a window of H <= 4096 s: 64 s, or 32 s when the
// window fits 64 of them (H <= 2048: a dense node's 30-min window then puts
// half as many events in a slab, so they fit k_ot_mid's chunks instead of
// k_ot_big's two reads).  The tile pre rows keep 64 slabs either way.
int ot_slab_bits(int64_t H) { return H <= 2048 ? kOtSlabBits - 1 : kOtSlabBits; }

#ifndef CG_OT_DENSE_BPC
#define CG_OT_DENSE_BPC 2  // blocks per CU of the dense merge's persistent grid
#endif
#ifndef CG_OT_DENSE_PER_SLAB
#define CG_OT_DENSE_PER_SLAB 2048  // average events per 64-s slab above which a node takes the 8-wave merge
#endif
// pin: the tiles were stored as packed words offset << 20 | rule (in node_rule2)
// pack: the tiles hold packed words (rule indices < 2^20, or hx); hx: rule
// indices past 2^20 (tiles cut where rule >> 20 changes, ts_hi)
int order_tail(cg_ctx* c, const int64_t* node_off, int32_t N, int64_t t0, int64_t H, hipStream_t st, int64_t* err,
               bool pack, bool pin, bool hx, int sb) {
  const uint16_t* toff = reinterpret_cast<const uint16_t*>(c->node_time2.p);
  // [0] big, [1] mid, [2] the dense merge's node ticket, [3] mid2
  unsigned* big_n = reinterpret_cast<unsigned*>(c->ts_off.p + int64_t(N) * kOtSlabs);
  HIPCHK(hipMemsetAsync(big_n, 0, 16, st));
  int64_t* slab_tab = c->ts_off.p + int64_t(N) * kOtSlabs + 2;
  int64_t* mid = slab_tab + int64_t(N) * kOtPre;
  int64_t* mid2 = mid + int64_t(N) * kOtSlabs;
  const int cus = std::max(1, c->write_blocks / kWriteBlocksPerCU);
  // nodes split by density between a 4-wave and an 8-wave merge; the dense
  // nodes' merge runs on its own stream beside the sparse one (few dense
  // nodes after all the sparse ones would run as a tail at low occupancy)
  const int64_t dense_min = int64_t(CG_OT_DENSE_PER_SLAB) * std::max<int64_t>(1, (H + 63) / 64);
  hipLaunchKernelGGL(k_ot_slabs, dim3(unsigned(N)), dim3(64), 0, st, c->ts_base.p, c->ts_hist.p, N, slab_tab);
  if (!c->st_ot) {  // created together: the ctx holds all three or none
    hipStream_t so = nullptr;
    hipEvent_t ef = nullptr, ej = nullptr;
    if (hipStreamCreateWithFlags(&so, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&ef, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&ej, hipEventDisableTiming) != hipSuccess) {
      if (ef) (void)hipEventDestroy(ef);
      if (so) (void)hipStreamDestroy(so);
      return cg_fail(CG_EHIP, "time order: stream / event creation failed");
    }
    c->st_ot = so;
    c->ot_fork = ef;
    c->ot_join = ej;
  }
  HIPCHK(hipEventRecord(c->ot_fork, st));
  HIPCHK(hipStreamWaitEvent(c->st_ot, c->ot_fork, 0));
  // rule indices below 2^20: (offset, rule) packed in one word
  auto merges = [&](auto m4, auto m8, auto mid_k, auto mid2_k, int dense_waves = kOtDenseWaves) {
    // the dense merge: a persistent grid (2 blocks per CU) taking nodes by ticket
    hipLaunchKernelGGL(m8, dim3(unsigned(std::min<int64_t>(N, int64_t(cus) * CG_OT_DENSE_BPC))), dim3(64 * dense_waves), 0,
                       c->st_ot, toff, c->node_rule2.p, c->ts_base.p, node_off, c->ts_hist.p, N, t0, slab_tab,
                       c->node_time.p, c->node_rule.p, c->ts_off.p, big_n, mid, big_n + 1, mid2, big_n + 3,
                       dense_min, INT64_MAX, big_n + 2, err, sb, c->ts_start.p, c->ts_hi.p);
    hipLaunchKernelGGL(m4, dim3(unsigned(N)), dim3(64 * kOtMergeWaves), 0, st, toff, c->node_rule2.p, c->ts_base.p,
                       node_off, c->ts_hist.p, N, t0, slab_tab, c->node_time.p, c->node_rule.p, c->ts_off.p, big_n,
                       mid, big_n + 1, mid2, big_n + 3, int64_t(0), dense_min, nullptr, err, sb, c->ts_start.p,
                       c->ts_hi.p);
    // k_ot_mid's queue is filled by the 4-wave merge only (the 8-wave merge's
    // chunk holds any slab of <= 8192 events).  Its blocks find no room
    // beside the dense merge (whose persistent grid holds every CU's VGPRs),
    // so it is queued behind both merges on the dense merge's stream: it
    // starts when it can run, and an empty queue costs one short launch
    // instead of a launch that spans the dense merge.
    (void)hipEventRecord(c->ot_fork, st);  // the 4-wave merge's queue entries are in
    (void)hipStreamWaitEvent(c->st_ot, c->ot_fork, 0);
    hipLaunchKernelGGL(mid_k, dim3(unsigned(cus * 3)), dim3(64 * kOtMidWaves), 0, c->st_ot,
                       toff, c->node_rule2.p, c->ts_base.p, node_off, c->ts_hist.p, t0, slab_tab, c->node_time.p,
                       c->node_rule.p, mid, big_n + 1, err, sb, c->ts_start.p, c->ts_hi.p);
    (void)hipEventRecord(c->ot_join, c->st_ot);
    (void)hipStreamWaitEvent(st, c->ot_join, 0);
    hipLaunchKernelGGL(mid2_k, dim3(unsigned(cus)), dim3(64 * kOtMid2Waves), 0, st, toff, c->node_rule2.p,
                         c->ts_base.p, node_off, c->ts_hist.p, t0, slab_tab, c->node_time.p, c->node_rule.p, mid2,
                         big_n + 3, err, sb, c->ts_start.p, c->ts_hi.p);
  };
  // past 2^20 rules (config 4 per node: every node dense, 32-s slabs of ~9 k
  // events) the dense merge runs 16 waves, a 16384-event chunk, so those slabs
  // skip k_ot_mid<16>'s separate pass: 5 windows 195.1-203.3 vs 201.2-208.7 ms;
  // with 8 waves config 3 is equal and pernode 12 % faster
  // (profiles/r06_ab_dense_merge_waves.txt)
  if (hx)
    merges(k_ot_merge<kOtMergeWaves, true, kOtMergeItems, false, true, true>,
           k_ot_merge<kOtDenseWavesHx, true, kOtDenseItems, true, true, true>,
           k_ot_mid<kOtMidWaves, true, kOtItems, true, true>, k_ot_mid<kOtMid2Waves, true, kOtItems, true, true>,
           kOtDenseWavesHx);
  else if (pack && pin)
    merges(k_ot_merge<kOtMergeWaves, true, kOtMergeItems, false, true>,
           k_ot_merge<kOtDenseWaves, true, kOtDenseItems, true, true>, k_ot_mid<kOtMidWaves, true, kOtItems, true>,
           k_ot_mid<kOtMid2Waves, true, kOtItems, true>);
  else if (pack)
    merges(k_ot_merge<kOtMergeWaves, true, kOtMergeItems>, k_ot_merge<kOtDenseWaves, true, kOtDenseItems, true>,
           k_ot_mid<kOtMidWaves, true>, k_ot_mid<kOtMid2Waves, true>);
  else
    merges(k_ot_merge<kOtMergeWaves, false, kOtMergeItems>, k_ot_merge<kOtDenseWaves, false, kOtDenseItems, true>,
           k_ot_mid<kOtMidWaves, false>, k_ot_mid<kOtMid2Waves, false>);
  auto big = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(unsigned(std::max(1, c->write_blocks))), dim3(256), 0, st, toff, c->node_rule2.p,
                       c->ts_base.p, node_off, c->ts_hist.p, t0, c->node_time.p, c->node_rule.p, c->ts_off.p, big_n,
                       err, sb, c->ts_start.p, c->ts_hi.p);
  };
  hx ? big(k_ot_big<true, true>) : (pin ? big(k_ot_big<true>) : big(k_ot_big<false>));
  return cg_hip_check(hipGetLastError(), "time-order kernels");
}

}  // namespace

// The tile sort + merge of the per-node lists already in c->node_time /
// c->node_rule (node offsets node_off[N+1] on the device): the writer's
// packed words / 16-bit offsets, or (cg_node_result_order_by_time) int64
// times.  Packed words of rule indices past 2^20 (in_mode kInPacked) need the
// lists' band offsets (cut): their tiles are cut where rule >> 20 changes.
int order_merge_enqueue(cg_ctx* c, const int64_t* node_off, int32_t N, int64_t cap, int64_t t0, int64_t H,
                        hipStream_t st, int in_mode, int64_t* err, const TileCut& cut) {
  if (N == 0 || cap == 0) return CG_OK;
  const bool low = c->pn_R <= (int64_t(1) << kOtRuleBits);
  const bool hx = in_mode == kInPacked && !low;
  OtCut oc{nullptr, 1, 1, 1};
  if (hx) {
    if (!cut.seg_pos || cut.B <= 0 || (int64_t(1) << kOtRuleBits) % cut.B != 0 ||
        c->pn_R > (int64_t(1) << (kOtRuleBits + kOtHiBits)))
      return cg_fail(CG_EINVAL, "time order: packed lists past 2^20 rules need band offsets of bands dividing 2^20");
    oc = OtCut{cut.seg_pos, cut.K, int32_t((int64_t(1) << kOtRuleBits) / cut.B),
               int32_t((c->pn_R + (int64_t(1) << kOtRuleBits) - 1) >> kOtRuleBits)};
  }
  int64_t Tmax = 0;
  int rc = order_setup(c, node_off, N, cap, st, &Tmax, oc);
  if (rc) return rc;
  uint16_t* toff = reinterpret_cast<uint16_t*>(c->node_time2.p);
  // the tiles stored as packed words when every rule index is below 2^20, or
  // (hx) as the writer's words with the high bits per tile
  const bool pack = low || hx;
  const int sb = ot_slab_bits(H);
  auto tile = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(unsigned(Tmax)), dim3(256), 0, st, c->node_time.p, c->node_rule.p, c->ts_tile_node.p,
                       c->ts_base.p, node_off, t0, toff, c->node_rule2.p, c->ts_hist.p, c->ts_base.p + N, err, sb,
                       c->ts_start.p);
  };
  if (in_mode == kInPacked) {
    tile(k_ot_tile<2, true>);
  } else if (in_mode == kIn16) {
    low ? tile(k_ot_tile<1, true>) : tile(k_ot_tile<1, false>);
  } else {
    low ? tile(k_ot_tile<0, true>) : tile(k_ot_tile<0, false>);
  }
  return order_tail(c, node_off, N, t0, H, st, err, pack, pack, hx, sb);  // packed tiles: packed words in node_rule2
}

extern "C" int cg_node_result_order_by_time(cg_ctx* c) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_order_by_time: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  if (c->pn_time_ordered) {  // written in (time, rule) order already
    c->kt[12] = 0.f;
    return CG_OK;
  }
  if ((rc = order_by_time_locked(c))) {  // a failed pass may leave the lists half permuted
    c->pn_E = 0;
    c->pn_valid = false;
  }
  return rc;
}

bool pn_pack_ok(int64_t R) { return R <= (int64_t(1) << (kOtRuleBits + kOtHiBits)); }

bool order_lsd_only() {
  static const bool lsd_only = getenv("CG_ORDER_LSD") != nullptr;
  return lsd_only;
}

int order_by_time_locked(cg_ctx* c, int in_mode) {
  int rc = CG_OK;
  const int64_t En = c->pn_E;
  const int32_t N = int32_t(c->pn_N);
  if (En == 0 || N == 0) {
    c->pn_time_ordered = true;
    return CG_OK;
  }
  const int64_t H = c->pn_t1 - c->pn_t0;  // time offsets in [0, H - 1]
  int bits = 0;
  while (bits < 63 && (int64_t(1) << bits) < H) bits++;
  const int passes = std::max(1, (bits + kTsBits - 1) / kTsBits);
  hipStream_t st = c->st;

  // windows <= 4096 s: tile sort + merge (CG_ORDER_LSD=1: the LSD passes)
  if (bits <= 12 && !order_lsd_only()) {
    if ((rc = pn_ensure_res(c))) return rc;
    c->pn_res_host[2] = 0;
    (void)hipEventRecord(c->pev[0], st);
    TileCut cut;  // the writer's packed words past 2^20 rules: tiles cut at the band offsets of this result
    if (in_mode == kInPacked) cut = TileCut{c->seg_pos.p, c->pn_K, c->pn_B, c->pn_R};
    if ((rc = order_merge_enqueue(c, c->node_off.p, N, En, c->pn_t0, H, st, in_mode, c->pn_res_dev + 2, cut)))
      return rc;
    (void)hipEventRecord(c->pev[1], st);
    if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
    if (c->pn_res_host[2]) return cg_fail(CG_EHIP, kOrderCheckMsg);
    (void)hipEventElapsedTime(&c->kt[12], c->pev[0], c->pev[1]);
    c->pn_time_ordered = true;
    return CG_OK;
  }
  if ((rc = c->ts_cnt.ensure(N)) || (rc = c->ts_base.ensure(int64_t(N) + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(N))))) return rc;
  hipLaunchKernelGGL(k_ts_tile_count, dim3(gridn(N, 256)), dim3(256), 0, st, c->node_off.p, N, kTsTile, En,
                     c->ts_cnt.p);
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
  c->pn_time_ordered = true;
  return CG_OK;
}
