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

int gridn(int64_t n, int threads) { return int(std::max<int64_t>(1, (n + threads - 1) / threads)); }

}  // namespace

extern "C" int cg_node_result_order_by_time(cg_ctx* c) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_order_by_time: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  const int64_t En = c->pn_E;
  const int32_t N = int32_t(c->pn_N);
  if (En == 0 || N == 0) return CG_OK;
  const int64_t H = c->pn_t1 - c->pn_t0;  // time offsets in [0, H - 1]
  int bits = 0;
  while (bits < 63 && (int64_t(1) << bits) < H) bits++;
  const int passes = std::max(1, (bits + kTsBits - 1) / kTsBits);
  hipStream_t st = c->st;

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
