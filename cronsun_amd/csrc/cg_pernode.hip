// cg_pernode.hip -- rule -> node resolution (CSR join) and per-node fire
// lists on gfx950.
//
// Reference semantics (job.go:274-288, 591-630; group.go:111-119;
// web/job.go:222-257): a rule runs on node n when n is one of its NodeIDs or a
// member of one of its (existing) GroupIDs, the job is not paused, and --
// depending on the exclude mode -- n is not excluded.  Every cronsun node
// evaluates this for itself over all jobs (node/node.go:121-158); here one
// pass builds the whole rule -> node CSR, then per-node fire lists.
//
// Pipeline:
//   k_rule_nodes<false>  one wave per rule: node bitmap in LDS (ds_or), count
//   scan                 -> rule->node CSR offsets
//   k_rule_nodes<true>   same bitmap, ballot/prefix-sum compaction of set bits
//   k_rs_hist/scatter    stable LSD radix transpose to node -> rules (8 bits a pass)
//   k_node_bounds        per-node pair offsets (lower bound per node)
//   (cached per rule set and exclude mode up to here)
//   k_seg_bounds         (node, rule band) segment bounds (cached per band width)
//   k_seg_records -> scan  per segment: events, compact pair records -> offsets
//   k_node_write         per segment, in band-major order: each node's copy of
//                        its rules' fire times (whole 64-event blocks; pairs
//                        placed by a wave prefix sum, blocks spanning pairs
//                        resolved by an LDS start mask + popcount)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"
#include "cg_kernels.h"

using namespace cg;

namespace {

struct RulesDev {
  const int64_t* nid_off;
  const int32_t* nids;
  const int64_t* gid_off;
  const int32_t* gids;
  const int64_t* ex_off;
  const int32_t* ex;
  const int32_t* rule_job;
  const uint8_t* job_pause;
  const int64_t* group_off;
  const int32_t* group_nodes;
  const uint8_t* group_exists;
  const int32_t* next_same;  // next rule of the job with the same Cmd key, -1; null: none repeats
  const int32_t* prev_same;  // the previous one, -1 (with next_same)
  int32_t R, G, N, words;
};

// wave-local LDS hand-off (the rules of HIP's __syncwarp: release fence,
// wave barrier, acquire fence)
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void bm_set(uint32_t* bm, int32_t n, int32_t N) {
  if (n >= 0 && n < N) atomicOr(&bm[n >> 5], 1u << (n & 31));
}
__device__ __forceinline__ void bm_clear(uint32_t* bm, int32_t n, int32_t N) {
  if (n >= 0 && n < N) atomicAnd(&bm[n >> 5], ~(1u << (n & 31)));
}

// Rule q's node set under `mode` into the wave's bitmap bm (zeroed here):
// NodeIDs and existing groups' members (JobRule.included job.go:274-288,
// Group.Included group.go:111-119), minus the mode's excludes; empty for a
// paused job (job.go:593).
__device__ void rule_bitmap(const RulesDev& d, int mode, int64_t q, uint32_t* bm, int lane) {
  for (int w = lane; w < d.words; w += 64) bm[w] = 0;
  wave_sync_lds();
  const int32_t job = d.rule_job[q];
  if (d.job_pause[job]) return;
  for (int64_t k = d.nid_off[q] + lane; k < d.nid_off[q + 1]; k += 64) bm_set(bm, d.nids[k], d.N);
  for (int64_t k = d.gid_off[q]; k < d.gid_off[q + 1]; k++) {
    int32_t g = d.gids[k];
    if (g < 0 || g >= d.G || !d.group_exists[g]) continue;  // gs[gid] missing
    for (int64_t p = d.group_off[g] + lane; p < d.group_off[g + 1]; p += 64)
      bm_set(bm, d.group_nodes[p], d.N);
  }
  wave_sync_lds();
  if (mode == CG_EXCLUDE_RULE) {
    for (int64_t k = d.ex_off[q] + lane; k < d.ex_off[q + 1]; k += 64) bm_clear(bm, d.ex[k], d.N);
  } else if (mode == CG_EXCLUDE_CUMULATIVE) {
    int64_t r0 = q;
    while (r0 > 0 && d.rule_job[r0 - 1] == job) r0--;
    for (int64_t p = r0; p <= q; p++)
      for (int64_t k = d.ex_off[p] + lane; k < d.ex_off[p + 1]; k += 64) bm_clear(bm, d.ex[k], d.N);
  }
  wave_sync_lds();
}

// One wave per rule r: r's node set (rule_bitmap) minus the node sets of the
// later rules of r's job with the same Cmd key -- Job.Cmds' map keeps the
// last included rule per Job.ID+Rule.ID (job.go:604-609) -- then either the
// count (WRITE false) or the ballot/prefix compaction of the set bits into the
// rule-major pairs (WRITE true).  With repeated keys the wave of a key's last
// rule sweeps the key's rules from last to first, keeping the union of the
// later ones' sets in a second bitmap (sh): every rule's set is built once
// (a job with k rules of one key costs k bitmap builds, not k^2 / 2); the
// other rules' waves have nothing to do.
template <bool WRITE>
__global__ __launch_bounds__(256) void k_rule_nodes(RulesDev d, int mode, int wpb,
                                                     int32_t* __restrict__ rn_cnt,
                                                     const int64_t* __restrict__ rn_off,
                                                     int32_t* __restrict__ rn_nodes,
                                                     int32_t* __restrict__ pair_rule) {
  extern __shared__ uint32_t bm_all[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= wpb) return;
  const bool dup = d.next_same != nullptr;
  uint32_t* bm = bm_all + size_t(wave) * (dup ? 2 : 1) * d.words;
  uint32_t* sh = bm + d.words;  // dup: union of the later same-key rules' sets
  for (int64_t r = int64_t(blockIdx.x) * wpb + wave; r < d.R; r += int64_t(gridDim.x) * wpb) {
    if (dup) {
      if (d.next_same[r] >= 0) continue;  // the key's last rule sweeps it
      for (int w = lane; w < d.words; w += 64) sh[w] = 0;
    }
    int64_t q = r;
    do {
      rule_bitmap(d, mode, q, bm, lane);
      if (!WRITE) {
        int32_t c = 0;
        for (int w = lane; w < d.words; w += 64) c += __popc(dup ? bm[w] & ~sh[w] : bm[w]);
        for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
        if (lane == 0) rn_cnt[q] = c;
      } else {
        int64_t pos = rn_off[q];
        for (int base = 0; base < d.words; base += 64) {
          int w = base + lane;
          uint32_t bits = w < d.words ? (dup ? bm[w] & ~sh[w] : bm[w]) : 0u;
          int32_t c = __popc(bits);
          int32_t inc = c;
          for (int o = 1; o < 64; o <<= 1) {
            int32_t y = __shfl_up(inc, o, 64);
            if (lane >= o) inc += y;
          }
          int64_t p = pos + inc - c;
          while (bits) {
            int b = __builtin_ctz(bits);
            bits &= bits - 1;
            rn_nodes[p] = w * 32 + b;
            pair_rule[p] = int32_t(q);
            p++;
          }
          pos += __shfl(inc, 63, 64);
        }
      }
      if (!dup) break;
      q = d.prev_same[q];
      if (q >= 0)
        for (int w = lane; w < d.words; w += 64) sh[w] |= bm[w];
      wave_sync_lds();
    } while (q >= 0);
    wave_sync_lds();
  }
}

// nt_off[n] = first position of node n in the node-sorted pairs (n <= N):
// a lower bound per node, no atomics (a histogram of sorted keys would put
// every lane of a wave on the same counter)
__global__ void k_node_bounds(const uint32_t* __restrict__ keys, int64_t n, int32_t N,
                              int64_t* __restrict__ nt_off) {
  const int64_t v = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (v > N) return;
  int64_t lo = 0, hi = n;  // first index with keys[i] >= v
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (int64_t(keys[mid]) < v) lo = mid + 1;
    else hi = mid;
  }
  nt_off[v] = lo;
}

__global__ void k_node_counts(const int64_t* __restrict__ node_off, int32_t N, int64_t* __restrict__ out) {
  int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n < N) out[n] = node_off[n + 1] - node_off[n];
}

// ---- transpose: stable LSD radix sort of the rule-major (node, rule) pairs
// by node, 8 bits per pass.  Each pass keeps the order of equal digits, so
// rules stay ascending within every node (the order Job.Cmds is evaluated in
// when a node walks the jobs, job.go:591-614). ----
constexpr int kRsItems = 16;
constexpr int kRsTile = 256 * kRsItems;  // pairs per block
constexpr int kRsBuckets = 256;

__global__ __launch_bounds__(256) void k_rs_hist(const uint32_t* __restrict__ keys, int64_t n, int shift,
                                                  int32_t* __restrict__ hist, int64_t nb) {
  __shared__ uint32_t h[kRsBuckets];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = int64_t(blockIdx.x) * kRsTile;
  for (int j = 0; j < kRsItems; j++) {
    const int64_t i = base + j * 256 + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & (kRsBuckets - 1)], 1u);
  }
  __syncthreads();
  hist[int64_t(threadIdx.x) * nb + blockIdx.x] = int32_t(h[threadIdx.x]);  // digit-major
}

// One pass's stable scatter.  Input order inside a block: wave w owns pairs
// [tile + w*1024, +1024), item j the 64 pairs [j*64, j*64 + 64) of those.  A
// pair's rank among equal digits = earlier items of its wave (running counts
// in LDS) + earlier lanes of its item (8-ballot multisplit) + earlier waves
// (prefix per digit) + earlier blocks (the scanned digit-major histogram).
__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t* __restrict__ kin,
                                                     const int32_t* __restrict__ vin, int64_t n, int shift,
                                                     const int64_t* __restrict__ off, int64_t nb,
                                                     uint32_t* __restrict__ kout, int32_t* __restrict__ vout) {
  __shared__ int32_t run[4][kRsBuckets];
  __shared__ int64_t base_of[4][kRsBuckets];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * kRsBuckets; i += 256) (&run[0][0])[i] = 0;
  __syncthreads();
  const int64_t base = int64_t(blockIdx.x) * kRsTile + int64_t(w) * (64 * kRsItems);
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t key[kRsItems];
  int32_t val[kRsItems], rk[kRsItems];
#pragma unroll
  for (int j = 0; j < kRsItems; j++) {
    const int64_t i = base + j * 64 + lane;
    key[j] = i < n ? kin[i] : 0u;
    val[j] = i < n ? vin[i] : 0;
  }
#pragma unroll
  for (int j = 0; j < kRsItems; j++) {
    const bool valid = base + j * 64 + lane < n;
    const uint32_t d = (key[j] >> shift) & (kRsBuckets - 1);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
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
  {
    const int d = threadIdx.x;
    int64_t acc = off[int64_t(d) * nb + blockIdx.x];
    for (int ww = 0; ww < 4; ww++) {
      base_of[ww][d] = acc;
      acc += run[ww][d];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRsItems; j++) {
    if (base + j * 64 + lane >= n) continue;
    const int64_t pos = base_of[w][(key[j] >> shift) & (kRsBuckets - 1)] + rk[j];
    kout[pos] = key[j];
    vout[pos] = val[j];
  }
}

// ---- per-call segments: (node n, rule band k) = node n's pairs whose rule is
// in [k*B, (k+1)*B).  Bands keep a band's rule fire lists (and their
// offsets) L2-resident while every node's segment of the band is written. ----

// seg_pair[n*K + k] = first pair of node n with rule >= k*B; [N*K] = nnz
__global__ void k_seg_bounds(const int64_t* __restrict__ nt_off, const int32_t* __restrict__ nt_rule,
                             int32_t N, int32_t K, int32_t B, int64_t* __restrict__ seg_pair) {
  const int64_t t = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const int64_t NK = int64_t(N) * K;
  if (t > NK) return;
  if (t == NK) {
    seg_pair[t] = nt_off[N];
    return;
  }
  const int32_t n = int32_t(t / K), k = int32_t(t - int64_t(n) * K);
  int64_t lo = nt_off[n], hi = nt_off[n + 1];
  const int64_t x = int64_t(k) * B;
  while (lo < hi) {  // first pair with rule >= x
    const int64_t mid = (lo + hi) >> 1;
    if (int64_t(nt_rule[mid]) < x) lo = mid + 1;
    else hi = mid;
  }
  seg_pair[t] = lo;
}

// Per rule of the window's rule-major CSR, one 16-byte RuleInfo: its fire
// count, the band-relative index of its first fire, and whether its fires
// form an arithmetic progression {first fire - t0, stride} (stride 0: they do
// not, or it does not fit 32 bits).  In a 1-h window nearly every rule's
// fires are one (`0 */5 * * * *`, `@every`, `*/10 * * * * *`, any rule with
// <= 2 fires: 95 % of config 3's events), and the per-node writer computes
// those fires instead of gathering them.  k_seg_records then reads one
// 16-byte word per pair instead of three scattered ones.  One block per 256
// rules: lanes take the block's events in turn, find their rule by a binary
// search over the block's offsets in LDS and clear the rule's flag on a step
// that differs from its first one.
#ifndef CG_NODE_AP
#define CG_NODE_AP 1
#endif
constexpr int kApRules = 256;
inline int64_t rule_info_slots(int64_t R) { return std::max<int64_t>(R, 1); }
__global__ __launch_bounds__(256) void k_rule_info(const int64_t* __restrict__ rule_off,
                                                    const int64_t* __restrict__ times, int64_t R, int64_t t0,
                                                    int32_t B, int64_t cap, RuleInfo* __restrict__ info,
                                                    int64_t* __restrict__ err) {
  __shared__ int64_t off[kApRules + 1];
  __shared__ int64_t step[kApRules];
  __shared__ int32_t ok[kApRules];
  const int64_t r0 = int64_t(blockIdx.x) * kApRules;
  const int nr = int(R - r0 < kApRules ? R - r0 : kApRules);
  const int tid = threadIdx.x;
  if (rule_off[R] > cap) {  // a pipelined window past the fire-time capacity: no fires read, none written
    if (tid < nr) info[r0 + tid] = RuleInfo{0, 0, 0, 0};
    return;
  }
  const int64_t band_lo = rule_off[(r0 / B) * B];  // B is a multiple of kApRules
  // the writer's 32-bit band-relative indices and k_seg_records' int32
  // scans need a band to hold < 2^30 events (else the call fails)
  if (r0 % B == 0 && threadIdx.x == 0 && rule_off[r0 + B < R ? r0 + B : R] - band_lo > (int64_t(1) << 30))
    err[0] = 1;
  int64_t first = 0, cnt = 0;
  if (tid < nr) {
    const int64_t a = rule_off[r0 + tid];
    cnt = rule_off[r0 + tid + 1] - a;
    first = cnt > 0 ? times[a] : 0;
    off[tid] = a;
    step[tid] = cnt > 1 ? times[a + 1] - first : 1;
    ok[tid] = CG_NODE_AP;
  }
  if (tid == 0) off[nr] = rule_off[r0 + nr];
  __syncthreads();
  const int64_t e_end = off[nr];
  // kRiUnroll events per thread per round, their loads issued together: a
  // block whose rules fire thousands of times in the window (every-second
  // rules) walks a long span, and one dependent load pair per round made it
  // the kernel's latency tail
  constexpr int kRiUnroll = 4;
  for (int64_t e0 = off[0] + tid; e0 + 1 < e_end; e0 += int64_t(blockDim.x) * kRiUnroll) {
    int64_t ta[kRiUnroll], tb[kRiUnroll];
#pragma unroll
    for (int u = 0; u < kRiUnroll; u++) {
      const int64_t e = e0 + int64_t(u) * blockDim.x;
      const int64_t ec = e + 1 < e_end ? e : e_end - 2;  // clamped: every load in range
      ta[u] = times[ec];
      tb[u] = times[ec + 1];
    }
#pragma unroll
    for (int u = 0; u < kRiUnroll; u++) {
      const int64_t e = e0 + int64_t(u) * blockDim.x;
      if (e + 1 >= e_end) break;
      int lo = 0, hi = nr - 1;  // the last rule whose list starts at or before e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= e) lo = mid;
        else hi = mid - 1;
      }
      if (e + 1 < off[lo + 1] && tb[u] - ta[u] != step[lo]) ok[lo] = 0;
    }
  }
  __syncthreads();
  if (tid < nr) {
    const int64_t rel = first - t0, s = step[tid];
    const bool prog = cnt > 0 && ok[tid] && rel >= 0 && rel <= INT32_MAX && s > 0 && s <= INT32_MAX;
    // counts and band-relative indices are < 2^30 (k_seg_records checks the
    // band span and fails the call otherwise)
    info[r0 + tid] = RuleInfo{int32_t(cnt), int32_t(off[tid] - band_lo),
                              prog ? int32_t(rel) : 0, prog ? int32_t(s) : 0};
  }
}

// Inclusive scan of x within each 32-lane half of the wave, by DPP (no LDS
// round trips): row_shr 1/2/4/8 inside each 16-lane row, then row_bcast:15
// adds the last lane of rows 0 and 2 to rows 1 and 3.
__device__ __forceinline__ int32_t scan_halves(int32_t x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 into rows 1, 3
  return x;
}
// lane 31's value in the low half, lane 63's in the high half
__device__ __forceinline__ int32_t half_total(int32_t incl) {
  const int32_t lo = __builtin_amdgcn_readlane(incl, 31), hi = __builtin_amdgcn_readlane(incl, 63);
  return (threadIdx.x & 63) < 32 ? lo : hi;
}

#ifndef CG_SEG_PAIRS_PER_LANE
#define CG_SEG_PAIRS_PER_LANE 8
#endif
constexpr int kSegPairsPerLane = CG_SEG_PAIRS_PER_LANE;
#ifndef CG_SEG_NOINFO
#define CG_SEG_NOINFO 0  // diagnostic timing only: no rule-info gathers (wrong records)
#endif
#ifndef CG_SEG_WPE
#define CG_SEG_WPE 1  // min waves per SIMD of k_seg_records (caps its VGPRs; 1: no cap)
#endif

// Segment records, one wave per segment in band-major order (a band's
// offsets stay in L2): the segment's event count, and for each of its
// non-empty pairs (in order, compacted to the front of the segment's pair
// range) a record {rule, first event relative to the segment, x, stride}:
// for a progression rule (k_rule_info) x = first fire - t0 - position * stride,
// so its fire at segment position p is t0 + x + p * stride; otherwise stride
// is 0 and x = band-relative fire-list index minus the position.  The writer
// then reads plain records instead of chasing pair -> rule -> offsets per
// window.  Block 0 also resets the writer's tickets; err[0] is set if a
// segment or a band outgrows the writer's 32-bit positions.
__global__ __launch_bounds__(256, CG_SEG_WPE) void k_seg_records(const int64_t* __restrict__ seg_pair,
                                                      const int32_t* __restrict__ nt_rule,
                                                      const int64_t* __restrict__ rule_off,
                                                      const RuleInfo* __restrict__ info, int32_t N,
                                                      int32_t K, int32_t B, int64_t R,
                                                      int64_t* __restrict__ seg_cnt,
                                                      int32_t* __restrict__ seg_nrec,
                                                      PairRec* __restrict__ recs,
                                                      uint32_t* __restrict__ tickets,
                                                      int64_t* __restrict__ err, int32_t xg) {
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < kTicketGroups * kTicketStride; i += blockDim.x) tickets[i] = 0;
  // xg > 1: the blocks of one residue b % xg (the same XCD under the
  // round-robin dispatch, MI355X_MICROARCH.md; speed only) take the bands
  // k == b % xg (mod xg), so each XCD's L2 holds the rule infos of its own
  // one or two bands instead of every band the whole grid is working on
  const int32_t grp = int32_t(blockIdx.x % unsigned(xg));
  const int64_t nb_g = (int64_t(gridDim.x) - grp + xg - 1) / xg;
  const int64_t lb = blockIdx.x / unsigned(xg);
  const int64_t nbands = (int64_t(K) - grp + xg - 1) / xg;  // this group's bands
  const int64_t NKg = nbands * N;
  // Two segments per wave, one per half-wave (consecutive nodes of a band),
  // software-pipelined: the kernel is latency-bound (segment bounds -> pair
  // rules -> rule infos -> records), so each iteration issues the bounds two
  // segment pairs ahead, the first round of pair rules one ahead and its own
  // rule infos together, and waits once.
  constexpr int L = 32;  // lanes per segment
  constexpr int P = kSegPairsPerLane;
  const int lane = threadIdx.x & 63, hl = lane & (L - 1);
  // every half-wave walks its own run of `per` consecutive segments (in band
  // order): the blocks resident at any time cover a few consecutive bands, so
  // their rule infos stay in L2 even when the grid is many times the blocks
  // the CUs hold at once (a grid-stride walk spread the resident blocks over
  // ~20 bands: half the info gathers missed L2, 72 GB per config-4 window)
  const int64_t Hg = nb_g * (blockDim.x >> 6) * 2;
  const int64_t per = (NKg + Hg - 1) / Hg;
  const int64_t hid = (lb * int64_t(blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const uint32_t below = (1u << hl) - 1u;  // lanes of this half before this one
  struct Seg {
    int64_t s, p0, p1;
  };
  auto bounds = [&](int64_t u) -> Seg {
    const int64_t t = hid * per + u;
    Seg g{-1, 0, 0};
    if (u < per && t < NKg) {
      const int32_t i = int32_t(t / N), n = int32_t(t - int64_t(i) * N);
      const int32_t k = grp + xg * i;
      g.s = int64_t(n) * K + k;
      g.p0 = seg_pair[g.s];
      g.p1 = seg_pair[g.s + 1];
    }
    return g;
  };
  // pair u*L + hl of round pc: every load and record store instruction covers
  // consecutive pairs / records
  auto rules = [&](const Seg& g, int32_t pc, int32_t (&r)[P]) {
#pragma unroll
    for (int u = 0; u < P; u++) {
      const int64_t pp = g.p0 + pc + u * L + hl;
      r[u] = pp < g.p1 ? nt_rule[pp] : -1;
    }
  };
  Seg cur = bounds(0), nxt = bounds(1);
  int32_t r[P], rn[P];
  rules(cur, 0, r);
  for (int64_t u = 0; u < per; u++) {
    const Seg nn = bounds(u + 2);  // two ahead
    rules(nxt, 0, rn);                   // the next pair's first round
    int64_t run = 0;  // events of the segment so far
    int32_t nrec = 0;
    const int32_t len = int32_t(cur.p1 - cur.p0);
    const int32_t rounds_len = max(__builtin_amdgcn_readlane(len, 0), __builtin_amdgcn_readlane(len, 32));
    for (int32_t pc = 0; pc < rounds_len; pc += L * P) {
      if (pc > 0) rules(cur, pc, r);  // segments of more than L*P pairs
      RuleInfo g[P];
#pragma unroll
      for (int u = 0; u < P; u++)
        g[u] = r[u] >= 0 ? (CG_SEG_NOINFO ? RuleInfo{1, 0, 0, 1} : info[r[u]]) : RuleInfo{0, 0, 0, 0};
#pragma unroll
      for (int u = 0; u < P; u++) {
        // events before this pair: half-wave inclusive scan of the counts
        // (int32: a band holds < 2^30 events, k_rule_info checks)
        const int32_t incl = scan_halves(g[u].cnt);
        const int64_t d = run + (incl - g[u].cnt);
        const uint64_t ball = __ballot(g[u].cnt > 0);
        const uint32_t ne = uint32_t(lane < 32 ? ball : ball >> 32);  // this half's non-empty pairs
        if (g[u].cnt > 0) {
          const int64_t at = cur.p0 + nrec + __popc(ne & below);
          const int64_t x = int64_t(g[u].first) - d * g[u].st;
          const bool prog = g[u].st != 0 && x >= INT32_MIN && x <= INT32_MAX;
          recs[at] = PairRec{r[u], int32_t(d), int32_t(prog ? x : int64_t(g[u].off) - d), prog ? g[u].st : 0};
        }
        run += half_total(incl);
        nrec += __popc(ne);
      }
    }
    if (hl == 0 && cur.s >= 0) {
      seg_cnt[cur.s] = run;
      seg_nrec[cur.s] = nrec;
      if (run > (int64_t(1) << 30)) err[0] = 1;
    }
    cur = nxt;
    nxt = nn;
#pragma unroll
    for (int u = 0; u < P; u++) r[u] = rn[u];
  }
}

// node_off[n] = seg_pos[n*K] (n <= N); the total is also stored to res
__global__ void k_node_off_from_seg(const int64_t* __restrict__ seg_pos, int32_t N, int32_t K,
                                    int64_t* __restrict__ node_off, int64_t* __restrict__ res) {
  const int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n > N) return;
  node_off[n] = seg_pos[n * K];
  if (n == N) res[0] = seg_pos[n * K];
}

__device__ __forceinline__ int64_t rl64n(int64_t v, int i) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), i));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), i));
  return int64_t((uint64_t(hi) << 32) | lo);
}
__device__ __forceinline__ int64_t bperm64(int64_t v, int src) {
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(v)));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(uint64_t(v) >> 32)));
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}
__device__ __forceinline__ int64_t perm64(int64_t v, int dst) {  // ds_permute: push to lane dst
  const int lo = __builtin_amdgcn_ds_permute(dst << 2, int(uint32_t(v)));
  const int hi = __builtin_amdgcn_ds_permute(dst << 2, int(uint32_t(uint64_t(v) >> 32)));
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

// Per-node lists, one (node, band) segment per wave task, tasks taken by
// ticket in band-major order (every node's segment of band 0, then band 1, ...)
// so the band's rule-major fire lists are read from L2 by all of them.  A
// wave reads its segment's pair records (k_seg_records: rule, first position,
// x, stride) 64 at a time, lane i holding record i, the next chunk in flight.
// The output is filled in aligned 64-event blocks:
//   runs   a block one record owns entirely (no record starts inside it) is
//          stored straight from that record: a progression's fires are
//          t0 + x + p * stride, so a run of such blocks costs two stores and
//          an add per block (other records: one gather per block);
//   one()  a block where records start, and the chunk's first and last blocks
//          (shared with the neighbouring chunk, or at the segment's edges):
//          the records starting in it mark their first lane in an LDS row
//          (tagged, no clearing); lane l's record = (records starting before
//          the block: one ballot over the sorted starts) - 1 + popcount(marks
//          at lanes <= l); its x, stride and rule come from that record's lane
//          (ds_bpermute).  A block shared with the next chunk is carried in
//          registers; only blocks at segment edges are stored partially.
// Gathers are waited for where they are issued: a wave's loads and stores
// retire in issue order, so a wait after a join would drain its stores on
// every block.
// V (diagnostic build only): 1 = no gather (the index as the value),
// 2 = no stores, 8 = no rule-index stores.
#ifndef CG_NODE_STORE
#define CG_NODE_STORE 2
#endif
// Output stores: 0 plain, 1 sc1 (relaxed agent-scope atomic stores), 2 nt.
// Plain stores keep the written lines in the XCD's L2; nt (streaming) stores
// were the fastest on one box (pernode writer 2.36 ms vs 2.60 sc1, 2.71
// plain, profiles/r02_ab_node_store.json).
template <int V, class T>
__device__ __forceinline__ void out_store(T* p, T v) {
  if (V & 2) {
    asm volatile("" ::"v"(v));
    return;
  }
#if CG_NODE_STORE == 2
  __builtin_nontemporal_store(v, p);
#elif CG_NODE_STORE == 1
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}
// Writer task order: 0 band-major (every node's segment of band 0, then band
// 1, ...: a band's fire lists stay in L2 for the gathers), 1 node-major (the
// segments of one node in turn: the concurrent write fronts stay in a few
// nodes' lists).  Rule-ordered lists are written node-major (same-box A/B,
// profiles/r05_ab_writer_order.txt: config 3 150.4 -> 146.9 ms, pernode
// -3 %, config 4 per node -2 %) unless a node has many bands (node_major_for);
// the time-order writer's packed words band-major (node-major: config 3 in
// time order +1 %, pernode equal).
#ifndef CG_NODE_MAJOR
#define CG_NODE_MAJOR 1
#endif
#ifndef CG_NODE_MAJOR_ORDERED
#define CG_NODE_MAJOR_ORDERED 0
#endif
// ticket groups across the 8 XCDs, as k_write_cf's (same box,
// profiles/r06_ab_node_writer_groups.txt: config 3 174.9 -> 170.7 ms per
// step, node writer 152.1 -> 146.7; pernode equal)
// 8 ticket groups (same-box A/B, profiles/r06_ab_ticket_groups_pn.txt:
// pernode node writer 2.45 -> 2.29 ms with 8 instead of 32, config 3 -1.5 %)
#ifndef CG_NODE_GROUPS
#define CG_NODE_GROUPS 8
#endif
constexpr int kNodeGroups = CG_NODE_GROUPS < kTicketGroups ? CG_NODE_GROUPS : kTicketGroups;
#ifndef CG_NODE_GRP_XCD
#define CG_NODE_GRP_XCD 1
#endif
constexpr int kNodeMajorDefault = CG_NODE_MAJOR;
// rule-ordered lists with many bands per node go band-major: a node-major
// sweep of K bands spreads the gathers over every band's fire lists, while
// band-major keeps one band's in L2 (same-box A/B, profiles/r06_ab_writer_order_bands.txt:
// config 4 per node, K = 305, 5 windows 201.8-203.4 -> 195.8-197.3 ms; config 3
// and pernode, K = 31, stay node-major: 140.4 vs 152.6 ms, 3.14-3.18 vs 3.20)
#ifndef CG_NODE_BAND_MAJOR_K
#define CG_NODE_BAND_MAJOR_K 128
#endif
inline int node_major_for(int32_t K) { return K >= CG_NODE_BAND_MAJOR_K ? 0 : kNodeMajorDefault; }
constexpr int kNodeMajorOrdered = CG_NODE_MAJOR_ORDERED;  // the time-order writer (packed words / 16-bit offsets)

// One (node, band) segment's events from its records (k_seg_records), in
// output position order, 64-event blocks at a time: put(q, val, rv) for the
// lanes whose position q (relative to the 64-aligned abase) is in the
// segment -- the whole block, or the lanes inside the segment at its edges.
// The body of k_node_write (the bucket writer of commit 7beb946 shared it).
//   runs   a block one record owns entirely (no record starts inside it) is
//          stored straight from that record: a progression's fires are
//          t0 + x + p * stride, so a run of such blocks costs two stores and
//          an add per block (other records: one gather per block);
//   one()  a block where records start, and the chunk's first and last blocks
//          (shared with the neighbouring chunk, or at the segment's edges):
//          the records starting in it mark their first lane in an LDS row
//          (tagged, no clearing); lane l's record = (records starting before
//          the block: one ballot over the sorted starts) - 1 + popcount(marks
//          at lanes <= l); its x, stride and rule come from that record's lane
//          (ds_bpermute).  A block shared with the next chunk is carried in
//          registers; only blocks at segment edges are stored partially.
// Gathers are waited for where they are issued: a wave's loads and stores
// retire in issue order, so a wait after a join would drain its stores on
// every block.  V & 1 (diagnostic build only): no gather (the index as the value).
template <int V, class Put>
__device__ __forceinline__ void node_segment(int64_t p0, int32_t nrec, int32_t q_lo, int32_t q_hi,
                                             const int64_t* __restrict__ tb, const PairRec* __restrict__ recs,
                                             int64_t t0, uint32_t* marks, uint32_t& tag, uint64_t le, Put&& put) {
  const int lane = threadIdx.x & 63;
  int32_t pq = -1, prule = 0;  // a block carried into the next chunk
  int64_t ptime = 0;
  // records in chunks of 64 (lane i: record i), the next chunk in flight
  // (an unconditional load at a clamped index: a load under a branch is
  // waited for at the branch's end, so the prefetch would not stay in flight)
  PairRec nx;
  int32_t nx_end = q_hi;
  auto fetch = [&](int32_t w) {
    nx = recs[p0 + (w + lane < nrec ? w + lane : nrec - 1)];
    // the chunk ends where the next one's first record starts
    nx_end = w + 64 < nrec ? recs[p0 + w + 64].dst + q_lo : q_hi;
  };
  fetch(0);
  for (int32_t w = 0; w < nrec; w += 64) {
    // q of first event; x and stride of the record (k_seg_records)
    const int32_t rr = nx.rule, dst = nx.dst + q_lo, dlt = nx.x, sst = nx.st, we = nx_end;
    const int nc = nrec - w < 64 ? nrec - w : 64;
    const int32_t qw = __builtin_amdgcn_readlane(dst, 0);
    if (w + 64 < nrec) fetch(w + 64);
    const bool live = lane < nc;
    auto one = [&](int32_t b) {
      tag++;
      const bool mark = live && dst >= b && dst < b + 64;
      marks[mark ? dst - b : 64 + lane] = tag;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const int32_t q = b + lane;
      const uint64_t M = __ballot(marks[lane] == tag);
      const int before = __popcll(__ballot(live && dst < b));
      int own = before - 1 + __popcll(M & le);
      own = own < 0 ? 0 : (own >= nc ? nc - 1 : own);
      const int32_t dl = __builtin_amdgcn_ds_bpermute(own << 2, dlt);
      const int32_t sv = __builtin_amdgcn_ds_bpermute(own << 2, sst);
      int32_t rv = __builtin_amdgcn_ds_bpermute(own << 2, rr);
      const bool in = q >= qw && q < we;
      int64_t val = in && sv != 0 ? t0 + int64_t(dl) + int64_t(q - q_lo) * sv : 0;
      const int32_t gi = in && sv == 0 ? q + dl - q_lo : -1;
      if (__ballot(gi >= 0)) {  // waited for here, not after the branch
        if (gi >= 0) val = (V & 1) ? int64_t(gi) : tb[gi];
        asm volatile("" : "+v"(val));
      }
      if (b == pq) {  // lanes of the previous chunk
        val = q < qw ? ptime : val;
        rv = q < qw ? prule : rv;
      }
      if (b + 64 <= we || we == q_hi) {  // complete, or the segment's last block
        if ((b >= q_lo && b + 64 <= q_hi) || (q >= q_lo && q < q_hi)) {  // whole, or a segment edge
          put(q, val, rv);
        }
        pq = -1;
      } else {  // carried into the next chunk
        pq = b;
        ptime = val;
        prule = rv;
      }
    };
    const int32_t b0 = qw & ~63, bl = we & ~63;
    if (qw & 63) one(b0);
    for (int32_t b = (qw + 63) & ~63; b < bl;) {
      const int o = __popcll(__ballot(live && dst <= b)) - 1;  // owner of lane 0 (dst[0] = qw <= b)
      const int32_t e = o + 1 < nc ? __builtin_amdgcn_readlane(dst, o + 1) : we;
      if (e < b + 64) {  // a record starts inside
        one(b);
        b += 64;
        continue;
      }
      const int32_t bend = (e & ~63) < bl ? (e & ~63) : bl;  // blocks [b, bend) all o's
      const int32_t dl = __builtin_amdgcn_readlane(dlt, o), sv = __builtin_amdgcn_readlane(sst, o);
      const int32_t rv = __builtin_amdgcn_readlane(rr, o);
      if (sv != 0) {
        int64_t val = t0 + int64_t(dl) + int64_t(b + lane - q_lo) * sv;
        const int64_t step = int64_t(64) * sv;
        for (; b < bend; b += 64, val += step) {
          put(b + lane, val, rv);
        }
      } else {
        for (; b < bend; b += 64) {
          const int32_t gi = b + lane + dl - q_lo;
          int64_t val = (V & 1) ? int64_t(gi) : tb[gi];
          asm volatile("" : "+v"(val));
          put(b + lane, val, rv);
        }
      }
    }
    if ((we & 63) && (bl != b0 || !(qw & 63))) one(bl);
  }
}

// OUT (windows <= 4096 s whose lists the time-order tile sort reads next):
// kInTimes int64 times + int32 rules; kIn16 the times as 16-bit offsets
// t - t0 - 1 (2 B per event instead of 8); kInPacked one word per event,
// offset << 20 | rule, into out_rule (4 B per event instead of 2 + 4; rule
// indices < 2^20)
template <int V, int OUT = kInTimes>
__global__ __launch_bounds__(256) void k_node_write(
    const int64_t* __restrict__ seg_pair, const int64_t* __restrict__ seg_pos,
    const int32_t* __restrict__ seg_nrec, const PairRec* __restrict__ recs, int64_t t0,
    const int64_t* __restrict__ rule_off, const int64_t* __restrict__ times, int32_t N, int32_t K,
    int32_t B, int64_t cap, uint32_t* __restrict__ tickets, int64_t* __restrict__ out_time,
    int32_t* __restrict__ out_rule, int node_major) {
  // per wave one 128-slot mark row (slots 64..127: the writes of lanes that
  // mark nothing); tags only grow, so no clearing
  __shared__ uint32_t marks_all[4][128];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t* marks = marks_all[wave];
  marks[lane] = 0u;
  uint32_t tag = 0;
  const int64_t NK = int64_t(N) * K;
  if (seg_pos[NK] > cap) return;  // output too small: the host grows it and relaunches
  const uint64_t le = (2ull << lane) - 1ull;  // lanes <= this one
  const int ng = int(gridDim.x) < kNodeGroups ? int(gridDim.x) : kNodeGroups;
#if CG_NODE_GRP_XCD
  // every group across the 8 XCDs (cf. k_write_cf), when the grid gives
  // every group a block that way (a small grid: one group per block)
  const int grp = int(gridDim.x >= 8u * unsigned(ng) ? (blockIdx.x >> 3) % unsigned(ng) : blockIdx.x % unsigned(ng));
#else
  const int grp = int(blockIdx.x % unsigned(ng));
#endif
  auto take = [&]() -> int64_t {
    unsigned int t = 0;
    if (lane == 0) t = atomicAdd(tickets + grp * kTicketStride, 1u);
    return grp + int64_t(ng) * int64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(t))));
  };
  // a task's descriptor, loaded one task ahead by lanes 0..4
  auto desc = [&](int64_t t) -> int64_t {
    if (t >= NK) return 0;
    const int32_t k = node_major ? int32_t(t % K) : int32_t(t / N);
    const int32_t n = node_major ? int32_t(t / K) : int32_t(t - int64_t(k) * N);
    const int64_t s = int64_t(n) * K + k;
    switch (lane) {
      case 0: return seg_pair[s];
      case 1: return seg_nrec[s];
      case 2: return seg_pos[s];
      case 3: return seg_pos[s + 1];
      case 4: return rule_off[int64_t(k) * B];
      default: return 0;
    }
  };
  int64_t t = take();
  int64_t dsc = desc(t);
  while (t < NK) {
    const int64_t t_next = take();
    const int64_t dsc_next = desc(t_next);
    const int64_t p0 = rl64n(dsc, 0), o0 = rl64n(dsc, 2), o1 = rl64n(dsc, 3), band_lo = rl64n(dsc, 4);
    const int32_t nrec = int32_t(rl64n(dsc, 1));
    t = t_next;
    dsc = dsc_next;
    if (o0 == o1) continue;
    // segment-local 32-bit positions: q = output index - abase (abase 64-aligned)
    const int64_t abase = o0 & ~int64_t(63);
    const int32_t q_lo = int32_t(o0 - abase), q_hi = q_lo + int32_t(o1 - o0);
    const int64_t* __restrict__ tb = times + band_lo;
    int64_t* __restrict__ ot = out_time + abase;
    uint16_t* __restrict__ o16 = reinterpret_cast<uint16_t*>(out_time) + abase;
    int32_t* __restrict__ orl = out_rule + abase;
    auto put = [&](int32_t q, int64_t val, int32_t rv) {
      if constexpr (OUT == kInPacked) {
        out_store<V>(orl + q, int32_t((uint32_t(val - t0 - 1) << 20) | (uint32_t(rv) & 0xFFFFFu)));  // rule >> 20: per tile
        return;
      }
      if constexpr (OUT == kIn16) out_store<V>(o16 + q, uint16_t(val - t0 - 1));
      else out_store<V>(ot + q, val);
      if (!(V & 8)) out_store<V>(orl + q, rv);
    };
    node_segment<V>(p0, nrec, q_lo, q_hi, tb, recs, t0, marks, tag, le, put);
  }
}

// One rank's per-node slice placed into the gathered per-node CSR
// (cg_node_csr_place): node n's events [src_off[n], src_off[n+1]) go to
// dst_start[n] onwards, rules shifted to global indices.  Event i of src_off's
// numbering is src[i - src_shift] (a gather chunk staged from position
// src_shift of the peer's CSR).  One block per node (grid-stride over nodes),
// four loads in flight per thread.
__global__ __launch_bounds__(256) void k_node_place(const int64_t* __restrict__ src_off, int32_t N, int64_t src_shift,
                                                     const int64_t* __restrict__ src_time,
                                                     const int32_t* __restrict__ src_rule, int32_t rule_add,
                                                     const int64_t* __restrict__ dst_start,
                                                     int64_t* __restrict__ dst_time, int32_t* __restrict__ dst_rule) {
  for (int64_t n = blockIdx.x; n < N; n += gridDim.x) {
    const int64_t a = src_off[n] - src_shift, b = src_off[n + 1] - src_shift, d = dst_start[n] - a;
    int64_t i = a + threadIdx.x;
    for (; i + 768 < b; i += 1024) {
      int64_t t[4];
      int32_t r[4];
#pragma unroll
      for (int u = 0; u < 4; u++) {
        t[u] = src_time[i + 256 * u];
        r[u] = src_rule[i + 256 * u];
      }
#pragma unroll
      for (int u = 0; u < 4; u++) {
        dst_time[i + 256 * u + d] = t[u];
        dst_rule[i + 256 * u + d] = r[u] + rule_add;
      }
    }
    for (; i < b; i += 256) {
      dst_time[i + d] = src_time[i];
      dst_rule[i + d] = src_rule[i] + rule_add;
    }
  }
}

// n contiguous events copied to dst, rules shifted (a part of one node's slice
// in the chunked gather, cg_comm.cpp)
__global__ __launch_bounds__(256) void k_span_place(int64_t n, const int64_t* __restrict__ src_time,
                                                     const int32_t* __restrict__ src_rule, int32_t rule_add,
                                                     int64_t* __restrict__ dst_time, int32_t* __restrict__ dst_rule) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    dst_time[i] = src_time[i];
    dst_rule[i] = src_rule[i] + rule_add;
  }
}

// Time-ordered gather (cg_node_csr_merge_ranks, cg_comm_gather_node_csr on
// time-ordered results).  A node's gathered list holds the ranks' slices in
// rank (= job-ID) order, each already in (time, rule) order, and every rule of
// rank g precedes every rule of rank g+1.  So an event's place in the node's
// byTime list (cron.go:64-79,220; ties by rule) is its index in its own run
// plus, for every other run q, the events of q before it: those with time <= t
// when q < g (smaller rules), time < t when q > g.  One block per tile of
// kMrTile events of one run: the tile's first and last times bound each other
// run's searches to a window (found once per block), then every event
// binary-searches the windows.  Reads a copy of the node group (src, index =
// position - src_base), writes the merged lists in place.
constexpr int kMrTile = 1024;

template <bool LE>
__device__ __forceinline__ int64_t mr_bound(const int64_t* __restrict__ t, int64_t lo, int64_t hi, int64_t v) {
  // the first index in [lo, hi) whose time is > v (LE) or >= v
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t x = t[mid];
    if (LE ? x <= v : x < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_merge_ranks(const int64_t* __restrict__ rb, const int64_t* __restrict__ tp,
                                                      int64_t n_runs, int32_t W, int64_t tile0,
                                                      const int64_t* __restrict__ src_t,
                                                      const int32_t* __restrict__ src_r, int64_t src_base,
                                                      int64_t* __restrict__ dst_t, int32_t* __restrict__ dst_r) {
  __shared__ int64_t s_lo[kMergeMaxRanks], s_hi[kMergeMaxRanks];
  __shared__ int64_t s_run;
  const int64_t b = tile0 + blockIdx.x;
  if (threadIdx.x == 0) {
    // the run holding tile b: the last r with tp[r] <= b (runs without tiles
    // share their successor's prefix)
    int64_t lo = 0, hi = n_runs;
    while (hi - lo > 1) {
      const int64_t mid = (lo + hi) >> 1;
      if (tp[mid] <= b)
        lo = mid;
      else
        hi = mid;
    }
    s_run = lo;
  }
  __syncthreads();
  const int64_t r = s_run;
  const int64_t n = r / W;
  const int g = int(r - n * W);
  const int64_t* nb = rb + n * (W + 1);
  const int64_t a = nb[g] - src_base, len = nb[g + 1] - nb[g];
  const int64_t i0 = (b - tp[r]) * kMrTile;
  const int64_t i1 = i0 + kMrTile < len ? i0 + kMrTile : len;
  const int64_t tmin = src_t[a + i0], tmax = src_t[a + i1 - 1];
  for (int q = threadIdx.x; q < W; q += blockDim.x) {
    if (q == g) continue;
    const int64_t qa = nb[q] - src_base, qb = nb[q + 1] - src_base;
    if (q < g) {
      s_lo[q] = mr_bound<true>(src_t, qa, qb, tmin);
      s_hi[q] = mr_bound<true>(src_t, s_lo[q], qb, tmax);
    } else {
      s_lo[q] = mr_bound<false>(src_t, qa, qb, tmin);
      s_hi[q] = mr_bound<false>(src_t, s_lo[q], qb, tmax);
    }
  }
  __syncthreads();
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int64_t tv = src_t[a + i];
    const int32_t rv = src_r[a + i];
    int64_t pos = nb[0] + i;
    for (int q = 0; q < W; q++) {
      if (q == g) continue;
      const int64_t k = q < g ? mr_bound<true>(src_t, s_lo[q], s_hi[q], tv) : mr_bound<false>(src_t, s_lo[q], s_hi[q], tv);
      pos += k - (nb[q] - src_base);
    }
    dst_t[pos] = tv;
    dst_r[pos] = rv;
  }
}

// Order-sensitive checksums of k nodes' lists (cg_node_checksum_enqueue): for
// node nodes[i], out[2i] = sum_j mix(j, time[j]) and out[2i+1] = sum_j
// mix(j, rule[j]) over its list (j node-relative), the cg_checksum_device mix.
// One block per node; nothing is read when the lists' total exceeds cap.
__device__ __forceinline__ uint64_t ck_mix(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}
__global__ __launch_bounds__(256) void k_node_checksums(const int64_t* __restrict__ node_off, int32_t N, int64_t cap,
                                                         const int64_t* __restrict__ time,
                                                         const int32_t* __restrict__ rule,
                                                         const int32_t* __restrict__ nodes,
                                                         unsigned long long* __restrict__ out) {
  __shared__ uint64_t s[2][4];
  const int32_t n = nodes[blockIdx.x];
  uint64_t at = 0, ar = 0;
  if (n >= 0 && n < N && node_off[N] <= cap) {
    const int64_t a = node_off[n], b = node_off[n + 1];
    for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
      const uint64_t h = ck_mix(uint64_t(i - a) * 0x9E3779B97F4A7C15ull);
      at += ck_mix(uint64_t(time[i]) ^ h);
      ar += ck_mix(uint64_t(int64_t(rule[i])) ^ h);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    at += __shfl_xor(at, o, 64);
    ar += __shfl_xor(ar, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s[0][threadIdx.x >> 6] = at;
    s[1][threadIdx.x >> 6] = ar;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = s[0][0] + s[0][1] + s[0][2] + s[0][3];
    out[2 * blockIdx.x + 1] = s[1][0] + s[1][1] + s[1][2] + s[1][3];
  }
}

// persistent k_node_write grid: as many 4-wave blocks per CU as its register
// and LDS use let run at once (no block of the grid waits for a slot)
#ifndef CG_NODE_BPC
#define CG_NODE_BPC 0  // 0: as many as the occupancy allows (up to 8)
#endif
int node_write_blocks_per_cu() {
  if (CG_NODE_BPC > 0) return CG_NODE_BPC + 2;  // the pipelined windows leave two slots free
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_node_write<0>, 256, 0) != hipSuccess || n < 1) n = 4;
  return std::min(n, 8);
}

int gridn(int64_t n, int threads, int cap) {
  int64_t b = (n + threads - 1) / threads;
  if (b < 1) b = 1;
  return int(std::min<int64_t>(b, cap));
}

template <class T>
int upload(DBuf<T>& b, const T* h, size_t n, hipStream_t st) {
  int rc = b.ensure(std::max<size_t>(n, 1));
  if (rc) return rc;
  if (n) return cg_hip_check(hipMemcpyAsync(b.p, h, n * sizeof(T), hipMemcpyHostToDevice, st),
                             "hipMemcpyAsync(rules)");
  return CG_OK;
}

int validate_rules(const cg_rules_in* in) {
  if (in->n_rules < 0 || in->n_nodes < 0 || in->n_groups < 0 || in->n_jobs < 0)
    return cg_fail(CG_EINVAL, "negative sizes");
  if (in->n_rules && (!in->nid_off || !in->gid_off || !in->ex_off || !in->rule_job))
    return cg_fail(CG_EINVAL, "rules arrays missing");
  if (in->n_groups && (!in->group_off || !in->group_exists))
    return cg_fail(CG_EINVAL, "group arrays missing");
  if (in->n_jobs && !in->job_pause) return cg_fail(CG_EINVAL, "job_pause missing");
  std::vector<uint8_t> seen(size_t(std::max(in->n_jobs, 1)), 0);
  for (int32_t r = 0; r < in->n_rules; r++) {
    int32_t j = in->rule_job[r];
    if (j < 0 || j >= in->n_jobs) return cg_fail(CG_EINVAL, "rule_job out of range");
    if (r == 0 || j != in->rule_job[r - 1]) {
      if (seen[j]) return cg_fail(CG_EINVAL, "a job's rules must be contiguous");
      seen[j] = 1;
    }
  }
  auto check_list = [&](const int64_t* off, const int32_t* v, int64_t cnt, int32_t lim,
                        const char* what) -> int {
    if (off[0] != 0) return cg_fail(CG_EINVAL, std::string(what) + ": offsets must start at 0");
    for (int64_t i = 0; i < cnt; i++)
      if (off[i + 1] < off[i]) return cg_fail(CG_EINVAL, std::string(what) + ": offsets decrease");
    for (int64_t k = 0; k < off[cnt]; k++)
      if (v[k] < 0 || v[k] >= lim) return cg_fail(CG_EINVAL, std::string(what) + ": index out of range");
    return CG_OK;
  };
  int rc;
  if (in->n_rules) {
    if ((rc = check_list(in->nid_off, in->nids, in->n_rules, in->n_nodes, "nids"))) return rc;
    if ((rc = check_list(in->gid_off, in->gids, in->n_rules, in->n_groups, "gids"))) return rc;
    if ((rc = check_list(in->ex_off, in->ex, in->n_rules, INT32_MAX, "exclude_nids"))) return rc;
  }
  if (in->n_groups && (rc = check_list(in->group_off, in->group_nodes, in->n_groups, in->n_nodes, "groups")))
    return rc;
  return CG_OK;
}

// validates a host rule set and copies it into a device store
int upload_rules(const cg_rules_in* in, RulesStore* st, hipStream_t s) {
  int rc = validate_rules(in);
  if (rc) return rc;
  const int32_t R = in->n_rules, G = in->n_groups;
  const int64_t n_nid = R ? in->nid_off[R] : 0, n_gid = R ? in->gid_off[R] : 0,
                n_ex = R ? in->ex_off[R] : 0, n_gn = G ? in->group_off[G] : 0;
  if ((rc = upload(st->nid_off, in->nid_off, R ? R + 1 : 0, s))) return rc;
  if ((rc = upload(st->nids, in->nids, n_nid, s))) return rc;
  if ((rc = upload(st->gid_off, in->gid_off, R ? R + 1 : 0, s))) return rc;
  if ((rc = upload(st->gids, in->gids, n_gid, s))) return rc;
  if ((rc = upload(st->ex_off, in->ex_off, R ? R + 1 : 0, s))) return rc;
  if ((rc = upload(st->ex, in->ex, n_ex, s))) return rc;
  if ((rc = upload(st->rule_job, in->rule_job, R, s))) return rc;
  if ((rc = upload(st->job_pause, in->job_pause, in->n_jobs, s))) return rc;
  if ((rc = upload(st->group_off, in->group_off, G ? G + 1 : 0, s))) return rc;
  if ((rc = upload(st->group_nodes, in->group_nodes, n_gn, s))) return rc;
  if ((rc = upload(st->group_exists, in->group_exists, G, s))) return rc;
  // Cmd keys: next_same[r] = the next rule of r's job with r's key (Job.Cmds'
  // later-rule-wins map, job.go:604-609), uploaded only when a key repeats
  std::vector<int32_t> next_same, prev_same;
  st->has_dup = false;
  if (in->rule_key && R) {
    next_same.assign(size_t(R), -1);
    prev_same.assign(size_t(R), -1);
    std::unordered_map<int32_t, int32_t> last;  // key -> the job's latest rule seen (walking back)
    for (int32_t r = R - 1; r >= 0; r--) {
      if (r == R - 1 || in->rule_job[r] != in->rule_job[r + 1]) last.clear();
      auto it = last.find(in->rule_key[r]);
      if (it != last.end()) {
        next_same[size_t(r)] = it->second;
        prev_same[size_t(it->second)] = r;
        it->second = r;
        st->has_dup = true;
      } else {
        last.emplace(in->rule_key[r], r);
      }
    }
  }
  if (st->has_dup && ((rc = upload(st->next_same, next_same.data(), size_t(R), s)) ||
                      (rc = upload(st->prev_same, prev_same.data(), size_t(R), s))))
    return rc;
  st->n_nodes = in->n_nodes;
  st->n_groups = G;
  st->n_rules = R;
  st->n_jobs = in->n_jobs;
  static std::atomic<uint64_t> next_serial{1};
  st->serial = next_serial.fetch_add(1);
  return cg_hip_check(hipStreamSynchronize(s), "upload rules");  // host arrays may go away
}

// builds the rule->node CSR on the device; leaves rn_off/rn_nodes/pair_rule in ctx
int rule_nodes_locked(cg_ctx* c, const RulesStore& st, int mode, int64_t* nnz_out) {
  if (mode < 0 || mode > 2) return cg_fail(CG_EINVAL, "bad exclude mode");
  const int32_t R = st.n_rules, G = st.n_groups, N = st.n_nodes;
  const int32_t words = (N + 31) / 32;
  if (size_t(words) * 4 * (st.has_dup ? 2 : 1) > 64 * 1024)
    return cg_fail(CG_ERANGE, st.has_dup ? "more than 262144 nodes with repeated Cmd keys"
                                         : "more than 524288 nodes");
  hipStream_t s = c->st;
  int rc;
  if ((rc = c->rn_cnt.ensure(std::max(R, 1)))) return rc;
  if ((rc = c->rn_off.ensure(R + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(R))))) return rc;
  RulesDev d{st.nid_off.p, st.nids.p, st.gid_off.p, st.gids.p, st.ex_off.p, st.ex.p,
             st.rule_job.p, st.job_pause.p, st.group_off.p, st.group_nodes.p,
             st.group_exists.p, st.has_dup ? st.next_same.p : nullptr,
             st.has_dup ? st.prev_same.p : nullptr, R, G, N, std::max(words, 1)};
  const size_t per = st.has_dup ? 2 : 1;  // a second bitmap per wave for repeated Cmd keys
  int wpb = int(std::min<size_t>(4, std::max<size_t>(1, (64 * 1024) / (per * size_t(d.words) * 4))));
  size_t lds = size_t(wpb) * per * d.words * 4;
  int grid = gridn(R, wpb, 256 * 16);
  if (R > 0)
    hipLaunchKernelGGL(k_rule_nodes<false>, dim3(grid), dim3(64 * wpb), lds, s, d, mode, wpb,
                       c->rn_cnt.p, nullptr, nullptr, nullptr);
  launch_scan(c->rn_cnt.p, c->rn_off.p, R, c->scan_tmp.p, s);
  int64_t nnz = 0;
  if ((rc = cg_hip_check(hipMemcpyAsync(&nnz, c->rn_off.p + R, 8, hipMemcpyDeviceToHost, s), "nnz")))
    return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(s), "sync"))) return rc;
  if ((rc = c->rn_nodes.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_rule.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if (R > 0 && nnz > 0)
    hipLaunchKernelGGL(k_rule_nodes<true>, dim3(grid), dim3(64 * wpb), lds, s, d, mode, wpb,
                       nullptr, c->rn_off.p, c->rn_nodes.p, c->pair_rule.p);
  if ((rc = cg_hip_check(hipGetLastError(), "k_rule_nodes"))) return rc;
  *nnz_out = nnz;
  return CG_OK;
}

// Stable transpose of the rule-major pairs (rn_nodes, pair_rule) into node
// order: nt_rule (rules ascending within a node) and nt_off[N+1].
int transpose_locked(cg_ctx* c, int64_t nnz, int32_t N) {
  hipStream_t st = c->st;
  int rc;
  if ((rc = c->nt_rule.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_node.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->nt_off.ensure(N + 1))) return rc;
  uint32_t* kin = reinterpret_cast<uint32_t*>(c->rn_nodes.p);
  int32_t* vin = c->pair_rule.p;
  uint32_t* kout = reinterpret_cast<uint32_t*>(c->pair_node.p);
  int32_t* vout = c->nt_rule.p;
  if (nnz > 0) {
    const int64_t nb = (nnz + kRsTile - 1) / kRsTile;
    if ((rc = c->rs_hist.ensure(kRsBuckets * nb))) return rc;
    if ((rc = c->rs_off.ensure(kRsBuckets * nb + 1))) return rc;
    if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(kRsBuckets * nb))))) return rc;
    int passes = 0;
    for (int shift = 0; shift == 0 || (int64_t(1) << shift) < int64_t(N); shift += 8) {
      hipLaunchKernelGGL(k_rs_hist, dim3(unsigned(nb)), dim3(256), 0, st, kin, nnz, shift, c->rs_hist.p, nb);
      launch_scan(c->rs_hist.p, c->rs_off.p, kRsBuckets * nb, c->scan_tmp.p, st);
      hipLaunchKernelGGL(k_rs_scatter, dim3(unsigned(nb)), dim3(256), 0, st, kin, vin, nnz, shift,
                         c->rs_off.p, nb, kout, vout);
      std::swap(kin, kout);
      std::swap(vin, vout);
      passes++;
    }
    // the sorted pairs are in (kin, vin): keep them in (pair_node, nt_rule)
    if (passes % 2 == 0) {
      std::swap(c->rn_nodes, c->pair_node);
      std::swap(c->pair_rule, c->nt_rule);
    }
  }
  hipLaunchKernelGGL(k_node_bounds, dim3(gridn(int64_t(N) + 1, 256, 1 << 30)), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t*>(c->pair_node.p), nnz, N, c->nt_off.p);
  return cg_hip_check(hipGetLastError(), "transpose");
}

// Rules per band: the band's rule-major fire lists (E_band * 8 B) should sit
// in one XCD's 4 MiB L2 beside the write stream; a power of two, so the
// cached segment bounds stay valid across windows of similar volume.
#ifndef CG_BAND_MIN_RULES
#define CG_BAND_MIN_RULES 32768  // rules per band at least (profiles/r06_ab_band_floor.txt: config 3 146-151 -> 144 ms)
#endif
#ifndef CG_BAND_BYTES
#define CG_BAND_BYTES (1536 * 1024)
#endif
// largest fire-list span of a band of B rules (rule-major offsets): *out = max_k
// off[min((k+1)B, R)] - off[kB] (atomicMax; *out zeroed by the caller)
__global__ void k_band_max(const int64_t* __restrict__ off, int64_t R, int32_t B, unsigned long long* out) {
  const int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  const int64_t a = k * B;
  if (a >= R) return;
  const int64_t b = a + B < R ? a + B : R;
  atomicMax(out, (unsigned long long)(off[b] - off[a]));
}

#ifndef CG_SEG_XCD
#define CG_SEG_XCD 8  // k_seg_records' XCD band groups (1: every block on the bands in order)
#endif
// band groups of k_seg_records: one per XCD when there are enough bands to
// balance them (else every XCD's blocks walk the bands in order)
int32_t seg_xcd_groups(int32_t K) { return CG_SEG_XCD > 1 && K >= 4 * CG_SEG_XCD ? CG_SEG_XCD : 1; }

// (at most 2^20 rules: the time-order pass cuts its tiles at multiples of
// 2^20 in rule index, found at band boundaries)
int32_t band_rules(int64_t R, int64_t E) {
  const double per_rule = double(std::max<int64_t>(E, 1)) * 8.0 / double(std::max<int64_t>(R, 1));
  int64_t B = int64_t(double(CG_BAND_BYTES) / per_rule);
  int64_t p = CG_BAND_MIN_RULES;
  while (p < B && p < R && p < (int64_t(1) << 20)) p <<= 1;
  return int32_t(std::max<int64_t>(p, 1024));
}

int per_node_locked(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                    const RulesStore& in, int mode, int64_t* n_events, int64_t* nnz_out) {
  if (int64_t(s->n) != in.n_rules)
    return cg_fail(CG_EINVAL, "specs count != rules n_rules");
  int64_t E = 0;
  int rc = expand_device_locked(c, s, z, t0, t1, &E);
  if (rc) return rc;
  int64_t nnz = 0;
  const int32_t N = in.n_nodes;
  const int64_t R = in.n_rules;
  hipStream_t st = c->st;
  const bool cached = in.serial != 0 && in.serial == c->pn_cache_serial && mode == c->pn_cache_mode;
  c->pn_E = 0;  // no readable result until this call succeeds
  c->pn_valid = false;
  c->pn_time_ordered = false;
  c->pn_R = R;
  (void)hipEventRecord(c->pev[0], st);
  if (cached) {
    nnz = c->pn_nnz;
  } else {
    c->pn_cache_serial = 0;  // the transpose buffers are about to change
    c->pn_K = 0;
    if ((rc = rule_nodes_locked(c, in, mode, &nnz))) return rc;
  }
  (void)hipEventRecord(c->pev[1], st);
  if (!cached && (rc = transpose_locked(c, nnz, N))) return rc;
  // segments (node, rule band): bounds cached per band width.  The writer's
  // band-relative indices are 32-bit: when the window holds more than 2^30
  // fires, bands whose fire lists pass 2^30 are halved (down to kApRules
  // rules; e.g. 1024 every-second rules over 13 days)
  int32_t B = band_rules(R, E);
  if (E > (int64_t(1) << 30) && R > 0) {
    if ((rc = c->cksum.ensure(1))) return rc;
    for (;;) {
      HIPCHK(hipMemsetAsync(c->cksum.p, 0, 8, st));
      hipLaunchKernelGGL(k_band_max, dim3(gridn((R + B - 1) / B, 256, 1 << 30)), dim3(256), 0, st, c->offsets.p, R,
                         B, c->cksum.p);
      unsigned long long mx = 0;
      HIPCHK(hipMemcpyAsync(&mx, c->cksum.p, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (mx <= (1ull << 30) || B <= kApRules) break;
      B /= 2;
    }
  }
  const int32_t K = int32_t(std::max<int64_t>(1, (R + B - 1) / B));
  const int64_t NK = int64_t(N) * K;
  if ((rc = c->seg_pair.ensure(NK + 1)) || (rc = c->seg_cnt.ensure(std::max<int64_t>(NK, 1))) ||
      (rc = c->seg_pos.ensure(NK + 1)) || (rc = c->node_off.ensure(N + 1)) ||
      (rc = c->pn_tickets.ensure(kTicketGroups * kTicketStride)))
    return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(NK))))) return rc;
  if (!(cached && c->pn_B == B && c->pn_K == K)) {
    hipLaunchKernelGGL(k_seg_bounds, dim3(gridn(NK + 1, 256, 1 << 30)), dim3(256), 0, st, c->nt_off.p,
                       c->nt_rule.p, N, K, B, c->seg_pair.p);
    c->pn_B = B;
    c->pn_K = K;
  }
  if ((rc = pn_ensure_res(c))) return rc;
  if ((rc = c->seg_nrec.ensure(std::max<int64_t>(NK, 1))) ||
      (rc = c->recs.ensure(std::max<int64_t>(nnz, 1))) ||
      (rc = c->rule_info.ensure(rule_info_slots(R))))
    return rc;
  c->pn_res_host[1] = 0;  // error flag (nothing of this ctx is in flight here)
  if (R > 0)
    hipLaunchKernelGGL(k_rule_info, dim3(unsigned((R + kApRules - 1) / kApRules)), dim3(256), 0, st,
                       c->offsets.p, c->times.p, R, t0, B, int64_t(c->times.cap), c->rule_info.p, c->pn_res_dev + 1);
  if (NK > 0)
    hipLaunchKernelGGL(k_seg_records, dim3(gridn(NK, 4, 256 * 64)), dim3(256), 0, st, c->seg_pair.p,
                       c->nt_rule.p, c->offsets.p, c->rule_info.p, N, K, B, R, c->seg_cnt.p, c->seg_nrec.p,
                       c->recs.p, c->pn_tickets.p,
                       c->pn_res_dev + 1, seg_xcd_groups(K));
  launch_scan64(c->seg_cnt.p, c->seg_pos.p, NK, c->scan_tmp.p, st);
  hipLaunchKernelGGL(k_node_off_from_seg, dim3(gridn(int64_t(N) + 1, 256, 1 << 30)), dim3(256), 0, st,
                     c->seg_pos.p, N, K, c->node_off.p, c->pn_res_dev);
  (void)hipEventRecord(c->pev[2], st);
  // the writer reads the total on the device and does nothing if it exceeds
  // the output capacity (first call or a larger result: grow, relaunch)
#ifdef CG_DIAG
  static const int variant = [] {  // diagnostic: 1 no gather, 2 no stores, 3 neither, 8 no rule stores
    const char* e = getenv("CG_NODE_VARIANT");
    return e ? atoi(e) : 0;
  }();
  static const int per_cu = [] {  // persistent grid: blocks of 4 waves per CU
    const char* e = getenv("CG_NODE_BLOCKS_PER_CU");
    return e ? std::max(1, atoi(e)) : node_write_blocks_per_cu();
  }();
  static const int node_major = [] {  // writer task order (see k_node_write)
    const char* e = getenv("CG_NODE_ORDER");
    return e ? atoi(e) : kNodeMajorDefault;
  }();
#else
  constexpr int variant = 0;
  const int node_major = node_major_for(K);
  static const int per_cu = node_write_blocks_per_cu();
#endif
  const int nw_blocks = c->write_blocks / kWriteBlocksPerCU * per_cu;
  // (time, rule) order of a window <= 4096 s (the predicate of
  // order_by_time_locked's tile sort: bits <= 12, not LSD): the writer emits
  // 16-bit offsets t - t0 - 1 (or packed words) for the tile sort
  const bool off16 = c->node_order == CG_NODE_ORDER_TIME && t1 - t0 <= 4096 && variant == 0 && !order_lsd_only();
  // packed words (offset << 20 | rule) when every rule index fits 20 bits
  const int in_mode = !off16 ? kInTimes : (pn_pack_ok(R) ? kInPacked : kIn16);
  c->pn_res_host[2] = 0;
  int64_t En = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    const int64_t cap = int64_t(std::min(c->node_time.cap, c->node_rule.cap));
    if (NK > 0 && cap > 0 && off16) {
      if (in_mode == kInPacked)
        hipLaunchKernelGGL((k_node_write<0, kInPacked>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))),
                           dim3(256), 0, st, c->seg_pair.p, c->seg_pos.p, c->seg_nrec.p, c->recs.p, t0, c->offsets.p,
                           c->times.p, N, K, B, cap, c->pn_tickets.p, c->node_time.p, c->node_rule.p, kNodeMajorOrdered);
      else
        hipLaunchKernelGGL((k_node_write<0, kIn16>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))),
                           dim3(256), 0, st, c->seg_pair.p, c->seg_pos.p, c->seg_nrec.p, c->recs.p, t0, c->offsets.p,
                           c->times.p, N, K, B, cap, c->pn_tickets.p, c->node_time.p, c->node_rule.p, kNodeMajorOrdered);
    } else if (NK > 0 && cap > 0) {
#define CG_NW(V)                                                                                    \
  hipLaunchKernelGGL((k_node_write<V, kInTimes>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))), dim3(256), \
                     0, st, c->seg_pair.p, c->seg_pos.p, c->seg_nrec.p, c->recs.p, t0, c->offsets.p,      \
                     c->times.p, N, K, B, cap, c->pn_tickets.p, c->node_time.p,     \
                     c->node_rule.p, node_major)
      switch (variant) {
        case 1: CG_NW(1); break;
        case 2: CG_NW(2); break;
        case 3: CG_NW(3); break;
        case 8: CG_NW(8); break;
        default: CG_NW(0); break;
      }
#undef CG_NW
    }
    (void)hipEventRecord(c->pev[3], st);
    if ((rc = cg_hip_check(hipGetLastError(), "per-node kernels"))) return rc;
    if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
    En = c->pn_res_host[0];
    if (c->pn_res_host[1] != 0)
      return cg_fail(CG_ERANGE, "per-node output: " + std::to_string(B) + " consecutive rules fire more than 2^30 "
                                "times in this window (the writer's 32-bit band indices; narrow the time window)");
    if (En <= cap) break;
    // grow the output, reset the tickets the first launch consumed, rerun
    if ((rc = c->node_time.ensure(En)) || (rc = c->node_rule.ensure(En))) return rc;
    HIPCHK(hipMemsetAsync(c->pn_tickets.p, 0, kTicketGroups * kTicketStride * 4, st));
    (void)hipEventRecord(c->pev[2], st);
  }
  (void)hipEventElapsedTime(&c->kt[6], c->pev[0], c->pev[1]);
  (void)hipEventElapsedTime(&c->kt[7], c->pev[1], c->pev[2]);
  (void)hipEventElapsedTime(&c->kt[8], c->pev[2], c->pev[3]);
  c->pn_E = En;
  c->pn_valid = true;
  c->pn_nnz = nnz;
  c->pn_N = N;
  c->pn_t0 = t0;
  c->pn_t1 = t1;
  c->pn_cache_serial = in.serial;
  c->pn_cache_mode = mode;
  *n_events = En;
  *nnz_out = nnz;
  // (time, rule) order: the tile sort + merge (or, past 4096 s, the LSD
  // passes) after the writer; if it fails nothing is readable (the lists may
  // hold the writer's 16-bit offsets)
  if (c->node_order == CG_NODE_ORDER_TIME) {
    if ((rc = order_by_time_locked(c, in_mode))) {
      c->pn_E = 0;
      c->pn_valid = false;
      *n_events = 0;
    }
    return rc;
  }
  c->kt[12] = 0.f;
  return CG_OK;
}

}  // namespace

// ---- pipelined per-node windows -------------------------------------------
// A node scheduler's tick loop (node/node.go:121-158 filtering every job,
// node/cron/cron.go:210-275 firing them) asks for consecutive windows of every
// node's list.  The synchronous entry point runs a window's expansion, records
// and writer in series with two host syncs; here window k+1's rule-major
// expansion, rule infos, segment records and node offsets run on the second
// stream (into set (k+1) % 3) while window k's k_node_write streams on the
// first.  The rule->node join, its transpose, the band width and the segment
// bounds come from an earlier synchronous call on the same rule set and mode.

namespace {

void pn_check_set(cg_ctx* c, PnAsyncSet& a) {
  if (!a.pending) return;
  a.pending = false;
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a.nw0, a.nw1) == hipSuccess) {
    c->nw_ms_sum += ms;
    c->nw_n++;
  }
  const int64_t E = a.rm.res_host[0], En = a.res_host[0];
  c->pa_en_sum += En;
  if (c->pa_rc) return;  // keep the first error
  const unsigned long long stuck = static_cast<unsigned long long>(a.rm.res_host[1]);
  if (stuck != ~0ULL) {
    c->pa_rc = CG_ERANGE;
    c->pa_msg = "rule " + std::to_string(stuck) +
                ": the reference Next loop never terminates inside this horizon "
                "(Next does not return, or returns a time <= its input and cycles)";
  } else if (E > a.rm_cap) {
    c->pa_rc = CG_ECAPACITY;
    c->pa_msg = "per-node async window (" + std::to_string(a.t0) + ", " + std::to_string(a.t1) + "]: " +
                std::to_string(E) + " rule-major events exceed the capacity " + std::to_string(a.rm_cap) +
                " (run a synchronous per-node call on a window this large first)";
  } else if (a.res_host[2] != 0) {
    c->pa_rc = CG_EHIP;
    c->pa_msg = kOrderCheckMsg;
  } else if (a.res_host[1] != 0) {
    c->pa_rc = CG_ERANGE;
    c->pa_msg = "per-node output: a (node, rule band) segment or a band's fire lists exceed 2^30 events";
  } else if (En > a.node_cap) {
    c->pa_rc = CG_ECAPACITY;
    c->pa_msg = "per-node async window (" + std::to_string(a.t0) + ", " + std::to_string(a.t1) + "]: " +
                std::to_string(En) + " node events exceed the output capacity " + std::to_string(a.node_cap) +
                " (run a synchronous per-node call on a window this large first)";
  }
}

int pn_ensure_async(cg_ctx* c) {
  int rc = ensure_async(c);  // the second stream
  if (rc) return rc;
  for (PnAsyncSet& a : c->pns) {
    if (a.written) continue;
    HIPCHK(hipEventCreateWithFlags(&a.side_done, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&a.written, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&a.nw0, hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&a.nw1, hipEventDisableSystemFence));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&a.res_host), 32, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.res_dev), a.res_host, 0));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&a.rm.res_host), 16, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.rm.res_dev), a.rm.res_host, 0));
    a.res_host[0] = a.res_host[1] = a.res_host[2] = 0;
    a.rm.res_host[0] = 0;
    a.rm.res_host[1] = -1;
  }
  return CG_OK;
}

}  // namespace

int pn_ensure_res(cg_ctx* c) {
  if (c->pn_res_host) return CG_OK;
  HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->pn_res_host), 32, hipHostMallocMapped | hipHostMallocCoherent));
  HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->pn_res_dev), c->pn_res_host, 0));
  c->pn_res_host[0] = c->pn_res_host[1] = c->pn_res_host[2] = 0;
  return CG_OK;
}

bool pn_async_pending(const cg_ctx* c) {
  for (const PnAsyncSet& a : c->pns)
    if (a.pending) return true;
  return false;
}

int pn_async_drain(cg_ctx* c) {
  if (!pn_async_pending(c)) return CG_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  for (PnAsyncSet& a : c->pns) pn_check_set(c, a);
  return CG_OK;
}

extern "C" {

int cg_expand_per_node_rules_device_async(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                                          const cg_rules* rules, int mode) {
  if (!c || !s || !z || !rules) return cg_fail(CG_EINVAL, "cg_expand_per_node_rules_device_async: null");
  if (rules->ctx != c) return cg_fail(CG_EINVAL, "rule set uploaded on another context");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  const RulesStore& in = rules->st;
  if (int64_t(s->n) != in.n_rules) return cg_fail(CG_EINVAL, "specs count != rules n_rules");
  if (!(in.serial != 0 && in.serial == c->pn_cache_serial && mode == c->pn_cache_mode && c->pn_K > 0))
    return cg_fail(CG_EINVAL, "cg_expand_per_node_rules_device_async: run cg_expand_per_node_rules_device once "
                              "on this rule set and exclude mode first (rule->node join, bands, capacity)");
  if (t1 - t0 > CG_MAX_HORIZON || t0 < -(int64_t(1) << 45) || t1 > (int64_t(1) << 45))
    return cg_fail(CG_ERANGE, "horizon must satisfy t1 - t0 <= CG_MAX_HORIZON (40 years)");
  if (async_pending(c))  // their only readable result would be lost below
    return cg_fail(CG_EINVAL, "pipelined rule-major calls pending (call cg_expand_wait first)");
  const int64_t rm_cap = int64_t(c->times.cap);
  const int64_t node_cap = int64_t(std::min(c->node_time.cap, c->node_rule.cap));
  if (rm_cap == 0 || node_cap == 0) return cg_fail(CG_ECAPACITY, "no output capacity yet (run a synchronous call)");
  int rc = pn_ensure_async(c);
  if (rc) return rc;
  // the rule-major result and the time-order records no longer describe a result
  c->as_last = -1;
  c->last_R = 0;
  c->last_E = 0;
  const int k = c->pa_next;
  PnAsyncSet& a = c->pns[k];
  // the set was last used kPnSets calls ago: its writer must be done
  HIPCHK(hipEventSynchronize(a.written));
  pn_check_set(c, a);
  const int32_t N = in.n_nodes, K = c->pn_K, B = c->pn_B;
  const int64_t R = in.n_rules, NK = int64_t(N) * K, nnz = c->pn_nnz;
  hipStream_t sc = c->st_cs, st = c->st;
  const bool timed = c->node_order == CG_NODE_ORDER_TIME;
  c->pn_R = R;
  if (timed && t1 - t0 > 4096)
    return cg_fail(CG_EINVAL, "pipelined per-node windows in time order: windows of at most 4096 s");
  bool empty = false;
  if ((rc = async_count_scan(c, a.rm, s, z, t0, t1, rm_cap, &empty))) return rc;
  if ((rc = a.times.ensure(std::max<int64_t>(rm_cap, 1))) || (rc = a.rule_info.ensure(rule_info_slots(R))) ||
      (rc = a.seg_cnt.ensure(std::max<int64_t>(NK, 1))) || (rc = a.seg_pos.ensure(NK + 1)) ||
      (rc = a.seg_nrec.ensure(std::max<int64_t>(NK, 1))) || (rc = a.recs.ensure(std::max<int64_t>(nnz, 1))) ||
      (rc = a.tickets.ensure(kTicketGroups * kTicketStride)) || (rc = a.node_off.ensure(int64_t(N) + 1)) ||
      (rc = a.seg_tmp.ensure(scan_temp_bytes(std::max<int64_t>(NK, 1)))))
    return rc;
  a.res_host[0] = 0;
  a.res_host[1] = 0;
  a.res_host[2] = 0;
  if (empty) {  // no rules: every list empty
    a.rm.res_host[0] = 0;
    a.rm.res_host[1] = -1;
    HIPCHK(hipMemsetAsync(a.seg_pos.p, 0, (NK + 1) * 8, sc));
    HIPCHK(hipMemsetAsync(a.rule_info.p, 0, rule_info_slots(R) * sizeof(RuleInfo), sc));
  } else {
    const PlanArgs& pa = a.rm.pa;
    const int64_t nruns = R * int64_t(pa.G);
    // the whole persistent grid: beside the previous window's per-node writer
    // only its free block slots run, and a smaller grid left this
    // latency-bound writer with fewer waves (same-box A/B,
    // profiles/r03_ab_pn_side.json: a quarter grid 3.21, a half 3.13, the
    // whole 3.12 ms per pernode step)
    launch_write_cf(s->d, pa, a.rm.run_anchor.p, a.rm.run_count.p, a.rm.run_dmask.p, a.rm.run_off.p, nruns,
                    a.rm.block_run.p, rm_cap, a.times.p, c->write_blocks, sc);
    if ((a.rm.plan.flags & (kPlanT0Walk | kPlanWalkSegs)) != 0)
      launch_write_walk(s->d, R, pa, a.rm.run_anchor.p, a.rm.run_count.p, a.rm.run_dmask.p, a.rm.run_off.p, rm_cap,
                        a.times.p, sc);
    if (R > 0)
      hipLaunchKernelGGL(k_rule_info, dim3(unsigned((R + kApRules - 1) / kApRules)), dim3(256), 0, sc,
                         a.rm.offsets.p, a.times.p, R, t0, B, rm_cap, a.rule_info.p, a.res_dev + 1);
  }
  if (NK > 0) {
    if (!empty)
      hipLaunchKernelGGL(k_seg_records, dim3(gridn(NK, 4, 256 * 64)), dim3(256), 0, sc, c->seg_pair.p, c->nt_rule.p,
                         a.rm.offsets.p, a.rule_info.p, N, K, B, R, a.seg_cnt.p, a.seg_nrec.p, a.recs.p,
                         a.tickets.p, a.res_dev + 1, seg_xcd_groups(K));
    else
      HIPCHK(hipMemsetAsync(a.seg_cnt.p, 0, NK * 8, sc));
    launch_scan64(a.seg_cnt.p, a.seg_pos.p, NK, a.seg_tmp.p, sc);
  }
  hipLaunchKernelGGL(k_node_off_from_seg, dim3(gridn(int64_t(N) + 1, 256, 1 << 30)), dim3(256), 0, sc, a.seg_pos.p,
                     N, K, a.node_off.p, a.res_dev);
  HIPCHK(hipEventRecord(a.side_done, sc));
  // the writer after the previous window's writer, once this window's records are built
  HIPCHK(hipStreamWaitEvent(st, a.side_done, 0));
  (void)hipEventRecord(a.nw0, st);
  if (NK > 0 && !empty) {
    // two block slots per CU fewer than the synchronous path's persistent
    // grid: the next window's count, records and offsets (second stream) get
    // wave slots beside this writer instead of waiting for it to retire
    static const int per_cu = std::max(1, node_write_blocks_per_cu() - 2);
    const int nw_blocks = c->write_blocks / kWriteBlocksPerCU * per_cu;
    if (timed) {  // packed words (or 16-bit offsets), then the tile sort + merge on the same stream
      const int in_mode = pn_pack_ok(R) ? kInPacked : kIn16;
      if (in_mode == kInPacked)
        hipLaunchKernelGGL((k_node_write<0, kInPacked>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))),
                           dim3(256), 0, st, c->seg_pair.p, a.seg_pos.p, a.seg_nrec.p, a.recs.p, t0, a.rm.offsets.p,
                           a.times.p, N, K, B, node_cap, a.tickets.p, c->node_time.p, c->node_rule.p,
                           kNodeMajorOrdered);
      else
        hipLaunchKernelGGL((k_node_write<0, kIn16>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))),
                           dim3(256), 0, st, c->seg_pair.p, a.seg_pos.p, a.seg_nrec.p, a.recs.p, t0, a.rm.offsets.p,
                           a.times.p, N, K, B, node_cap, a.tickets.p, c->node_time.p, c->node_rule.p,
                           kNodeMajorOrdered);
      if ((rc = order_merge_enqueue(c, a.node_off.p, N, node_cap, t0, t1 - t0, st, in_mode, a.res_dev + 2,
                                    TileCut{a.seg_pos.p, K, B, R})))
        return rc;
    } else {
      hipLaunchKernelGGL((k_node_write<0, kInTimes>), dim3(unsigned(std::min<int64_t>(NK / 4 + 1, nw_blocks))), dim3(256),
                         0, st, c->seg_pair.p, a.seg_pos.p, a.seg_nrec.p, a.recs.p, t0, a.rm.offsets.p, a.times.p, N,
                         K, B, node_cap, a.tickets.p, c->node_time.p, c->node_rule.p, node_major_for(K));
    }
  }
  (void)hipEventRecord(a.nw1, st);
  HIPCHK(hipEventRecord(a.written, st));
  HIPCHK(hipGetLastError());
  a.pending = true;
  a.timed = timed;
  a.t0 = t0;
  a.t1 = t1;
  a.rm_cap = rm_cap;
  a.node_cap = node_cap;
  a.N = N;
  c->pa_next = (k + 1) % cg_ctx::kPnSets;
  c->pa_last = k;
  c->pn_E = 0;  // nothing readable until cg_expand_per_node_wait
  c->pn_valid = false;
  return CG_OK;
}

int cg_expand_per_node_wait(cg_ctx* c, int64_t* n_events, int64_t* n_events_all) {
  if (!c) return cg_fail(CG_EINVAL, "cg_expand_per_node_wait: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = pn_async_drain(c);
  if (rc) return rc;
  if (c->nw_n > 0) c->kt[8] = float(c->nw_ms_sum / c->nw_n);  // mean per-node writer time of the calls checked
  c->nw_ms_sum = 0;
  c->nw_n = 0;
  const int rc_async = c->pa_rc;
  const std::string msg = c->pa_msg;
  c->pa_rc = 0;
  c->pa_msg.clear();
  int64_t En = 0;
  if (c->pa_last >= 0) {
    PnAsyncSet& a = c->pns[c->pa_last];
    En = a.res_host[0];
    if (!rc_async) {  // the last window becomes the readable per-node result
      if ((rc = c->node_off.ensure(int64_t(a.N) + 1))) return rc;
      HIPCHK(hipMemcpyAsync(c->node_off.p, a.node_off.p, (int64_t(a.N) + 1) * 8, hipMemcpyDeviceToDevice, c->st));
      HIPCHK(hipStreamSynchronize(c->st));
      c->pn_E = En;
      c->pn_valid = true;
      c->pn_time_ordered = a.timed;
      c->pn_N = a.N;
      c->pn_t0 = a.t0;
      c->pn_t1 = a.t1;
    }
    c->pa_last = -1;
  }
  if (n_events) *n_events = rc_async ? 0 : En;
  if (n_events_all) *n_events_all = c->pa_en_sum;
  c->pa_en_sum = 0;
  if (rc_async) return cg_fail(rc_async, msg);
  return CG_OK;
}

}  // extern "C"

extern "C" {

int cg_rule_nodes(cg_ctx* c, const cg_rules_in* in, int mode, int64_t* rn_off, int32_t* rn_nodes,
                  int64_t cap, int64_t* nnz) {
  if (!c || !in || !nnz) return cg_fail(CG_EINVAL, "cg_rule_nodes: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if ((rc = upload_rules(in, &c->rules, c->st))) return rc;
  if ((rc = rule_nodes_locked(c, c->rules, mode, nnz))) return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(c->st), "sync"))) return rc;
  if (rn_off &&
      (rc = cg_hip_check(hipMemcpy(rn_off, c->rn_off.p, size_t(in->n_rules + 1) * 8, hipMemcpyDeviceToHost),
                         "copy rn_off")))
    return rc;
  if (rn_nodes) {
    if (cap < *nnz) return cg_fail(CG_ECAPACITY, "rn_nodes buffer too small; see nnz");
    if (*nnz && (rc = cg_hip_check(hipMemcpy(rn_nodes, c->rn_nodes.p, size_t(*nnz) * 4, hipMemcpyDeviceToHost),
                                   "copy rn_nodes")))
      return rc;
  }
  return CG_OK;
}

int cg_expand_per_node_device(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                              const cg_rules_in* rules, int mode, int64_t* n_events, int64_t* nnz) {
  if (!c || !s || !z || !rules || !n_events || !nnz)
    return cg_fail(CG_EINVAL, "cg_expand_per_node_device: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if ((rc = upload_rules(rules, &c->rules, c->st))) return rc;
  return per_node_locked(c, s, z, t0, t1, c->rules, mode, n_events, nnz);
}

int cg_rules_upload(cg_ctx* c, const cg_rules_in* in, cg_rules** out) {
  if (!c || !in || !out) return cg_fail(CG_EINVAL, "cg_rules_upload: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  cg_rules* r = new cg_rules();
  r->ctx = c;
  if ((rc = upload_rules(in, &r->st, c->st))) {
    r->st.release();
    delete r;
    return rc;
  }
  *out = r;
  return CG_OK;
}

void cg_rules_free(cg_rules* r) {
  if (!r) return;
  (void)hipSetDevice(r->ctx->device);
  r->st.release();
  delete r;
}

int cg_expand_per_node_rules_device(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0,
                                    int64_t t1, const cg_rules* rules, int mode, int64_t* n_events,
                                    int64_t* nnz) {
  if (!c || !s || !z || !rules || !n_events || !nnz)
    return cg_fail(CG_EINVAL, "cg_expand_per_node_rules_device: null");
  if (rules->ctx != c) return cg_fail(CG_EINVAL, "rule set uploaded on another context");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  return per_node_locked(c, s, z, t0, t1, rules->st, mode, n_events, nnz);
}

int cg_expand_per_node(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                       const cg_rules_in* rules, int mode, cg_node_csr* out) {
  if (!c || !s || !z || !rules || !out) return cg_fail(CG_EINVAL, "cg_expand_per_node: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  int64_t En = 0, nnz = 0;
  if ((rc = upload_rules(rules, &c->rules, c->st))) return rc;
  if ((rc = per_node_locked(c, s, z, t0, t1, c->rules, mode, &En, &nnz))) return rc;
  out->n_events = En;
  out->nnz = nnz;
  if (out->node_off &&
      (rc = cg_hip_check(hipMemcpy(out->node_off, c->node_off.p, size_t(rules->n_nodes + 1) * 8,
                                   hipMemcpyDeviceToHost), "copy node_off")))
    return rc;
  if (out->time || out->rule) {
    if (out->cap < En) return cg_fail(CG_ECAPACITY, "per-node buffers too small; see n_events");
    if (En && out->time &&
        (rc = cg_hip_check(hipMemcpy(out->time, c->node_time.p, size_t(En) * 8, hipMemcpyDeviceToHost),
                           "copy time")))
      return rc;
    if (En && out->rule &&
        (rc = cg_hip_check(hipMemcpy(out->rule, c->node_rule.p, size_t(En) * 4, hipMemcpyDeviceToHost),
                           "copy rule")))
      return rc;
  }
  return CG_OK;
}

int cg_node_result_device(cg_ctx* c, const int64_t** d_node_off, const int64_t** d_time,
                          const int32_t** d_rule, int64_t* n_events) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_device: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  if (d_node_off) *d_node_off = c->node_off.p;
  if (d_time) *d_time = c->node_time.p;
  if (d_rule) *d_rule = c->node_rule.p;
  if (n_events) *n_events = c->pn_E;
  return CG_OK;
}

int cg_node_result_copy(cg_ctx* c, int64_t* node_off, int64_t* time, int32_t* rule, int64_t cap) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_copy: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (node_off && (rc = cg_hip_check(hipMemcpy(node_off, c->node_off.p, size_t(c->pn_N + 1) * 8,
                                               hipMemcpyDeviceToHost), "copy node_off")))
    return rc;
  if (time || rule) {
    if (cap < c->pn_E) return cg_fail(CG_ECAPACITY, "per-node buffers too small; see n_events");
    if (c->pn_E && time &&
        (rc = cg_hip_check(hipMemcpy(time, c->node_time.p, size_t(c->pn_E) * 8, hipMemcpyDeviceToHost),
                           "copy time")))
      return rc;
    if (c->pn_E && rule &&
        (rc = cg_hip_check(hipMemcpy(rule, c->node_rule.p, size_t(c->pn_E) * 4, hipMemcpyDeviceToHost),
                           "copy rule")))
      return rc;
  }
  return CG_OK;
}

int cg_node_result_copy_range(cg_ctx* c, int64_t first, int64_t count, int64_t* time, int32_t* rule) {
  if (!c || (count && !time && !rule)) return cg_fail(CG_EINVAL, "cg_node_result_copy_range: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (first < 0 || count < 0 || first + count > c->pn_E)
    return cg_fail(CG_EINVAL, "range outside the last per-node result");
  if (count && time &&
      (rc = cg_hip_check(hipMemcpy(time, c->node_time.p + first, size_t(count) * 8, hipMemcpyDeviceToHost),
                         "copy time")))
    return rc;
  if (count && rule &&
      (rc = cg_hip_check(hipMemcpy(rule, c->node_rule.p + first, size_t(count) * 4, hipMemcpyDeviceToHost),
                         "copy rule")))
    return rc;
  return CG_OK;
}

int cg_node_csr_place(cg_ctx* c, int32_t n_nodes, const int64_t* d_src_node_off, const int64_t* d_src_time,
                      const int32_t* d_src_rule, int32_t rule_add, const int64_t* d_dst_start, int64_t* d_dst_time,
                      int32_t* d_dst_rule) {
  if (!c || n_nodes < 0 || (n_nodes > 0 && (!d_src_node_off || !d_dst_start)))
    return cg_fail(CG_EINVAL, "cg_node_csr_place: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (n_nodes > 0)
    hipLaunchKernelGGL(k_node_place, dim3(unsigned(std::min<int64_t>(n_nodes, int64_t(c->write_blocks) * 2))),
                       dim3(256), 0, c->st, d_src_node_off, n_nodes, int64_t(0), d_src_time, d_src_rule, rule_add, d_dst_start,
                       d_dst_time, d_dst_rule);
  if ((rc = cg_hip_check(hipGetLastError(), "k_node_place"))) return rc;
  return cg_hip_check(hipStreamSynchronize(c->st), "sync");
}

}  // extern "C"

// placement launchers for the RCCL gather (cg_comm.cpp); enqueued on st
int launch_node_place(cg_ctx* c, hipStream_t st, int32_t N, const int64_t* src_off, int64_t src_shift,
                      const int64_t* src_time, const int32_t* src_rule, int32_t rule_add, const int64_t* dst_start,
                      int64_t* dst_time, int32_t* dst_rule) {
  if (N > 0)
    hipLaunchKernelGGL(k_node_place, dim3(unsigned(std::min<int64_t>(N, int64_t(c->write_blocks) * 2))), dim3(256),
                       0, st, src_off, N, src_shift, src_time, src_rule, rule_add, dst_start, dst_time, dst_rule);
  return cg_hip_check(hipGetLastError(), "k_node_place");
}

int launch_span_place(cg_ctx* c, hipStream_t st, int64_t n, const int64_t* src_time, const int32_t* src_rule,
                      int32_t rule_add, int64_t* dst_time, int32_t* dst_rule) {
  if (n > 0)
    hipLaunchKernelGGL(k_span_place, dim3(unsigned(gridn(n, 256, c->write_blocks * 4))), dim3(256), 0, st, n,
                       src_time, src_rule, rule_add, dst_time, dst_rule);
  return cg_hip_check(hipGetLastError(), "k_span_place");
}

int launch_node_counts(cg_ctx* c, hipStream_t st, int64_t* d_counts) {
  if (c->pn_N > 0)
    hipLaunchKernelGGL(k_node_counts, dim3(gridn(c->pn_N, 256, 1 << 30)), dim3(256), 0, st, c->node_off.p,
                       int32_t(c->pn_N), d_counts);
  return cg_hip_check(hipGetLastError(), "k_node_counts");
}

int merge_ranks_locked(cg_ctx* c, hipStream_t st, int32_t N, int32_t W, const int64_t* h_rb, int64_t* d_time,
                       int32_t* d_rule, int64_t scratch_ev, DBuf<int64_t>& scr_t, DBuf<int32_t>& scr_r) {
  if (W <= 1 || N <= 0) return CG_OK;
  if (W > kMergeMaxRanks) return cg_fail(CG_EINVAL, "time-ordered gather: more than 64 ranks");
  const int64_t NW = int64_t(N) * W;
  // tiles per run; a node with fewer than two non-empty runs is already merged
  std::vector<int64_t> tp(size_t(NW + 1), 0);
  int64_t big = 0;  // the largest node that needs a merge
  for (int64_t n = 0; n < N; n++) {
    const int64_t* nb = h_rb + n * (W + 1);
    int nonempty = 0;
    for (int q = 0; q < W; q++) {
      if (nb[q + 1] < nb[q]) return cg_fail(CG_EINVAL, "time-ordered gather: run bounds not ascending");
      nonempty += nb[q + 1] > nb[q];
    }
    if (n > 0 && nb[0] < h_rb[(n - 1) * (W + 1) + W])
      return cg_fail(CG_EINVAL, "time-ordered gather: node lists overlap");
    for (int q = 0; q < W; q++)
      tp[size_t(n * W + q + 1)] = tp[size_t(n * W + q)] + (nonempty >= 2 ? (nb[q + 1] - nb[q] + kMrTile - 1) / kMrTile : 0);
    if (nonempty >= 2) big = std::max(big, nb[W] - nb[0]);
  }
  if (tp[size_t(NW)] == 0) return CG_OK;
  // the scratch never exceeds the events of the lists being merged (a small
  // CSR with the default 2-GiB budget needs only its own size), nor falls
  // below the largest merging node
  scratch_ev = std::max(std::min(scratch_ev, h_rb[NW + N - 1] - h_rb[0]), big);
  int rc;
  if ((rc = c->mr_rb.ensure(size_t(N) * (W + 1))) || (rc = c->mr_tp.ensure(size_t(NW + 1))) ||
      (rc = scr_t.ensure(size_t(scratch_ev))) || (rc = scr_r.ensure(size_t(scratch_ev))))
    return rc;
  HIPCHK(hipMemcpyAsync(c->mr_rb.p, h_rb, size_t(N) * (W + 1) * 8, hipMemcpyHostToDevice, st));
  HIPCHK(hipMemcpyAsync(c->mr_tp.p, tp.data(), tp.size() * 8, hipMemcpyHostToDevice, st));
  // node groups of at most scratch_ev events; every group: a copy of its
  // lists, then the tiles of its runs merge from the copy into place
  int64_t n0 = 0;
  while (n0 < N) {
    const int64_t base = h_rb[n0 * (W + 1)];
    int64_t n1 = n0 + 1;
    while (n1 < N && h_rb[n1 * (W + 1) + W] - base <= scratch_ev) n1++;
    const int64_t t0 = tp[size_t(n0 * W)], t1 = tp[size_t(n1 * W)];
    if (t1 > t0) {
      const int64_t ev = h_rb[(n1 - 1) * (W + 1) + W] - base;
      HIPCHK(hipMemcpyAsync(scr_t.p, d_time + base, size_t(ev) * 8, hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(scr_r.p, d_rule + base, size_t(ev) * 4, hipMemcpyDeviceToDevice, st));
      for (int64_t tb = t0; tb < t1; tb += int64_t(1) << 30) {
        const int64_t nt = std::min<int64_t>(t1 - tb, int64_t(1) << 30);
        hipLaunchKernelGGL(k_merge_ranks, dim3(unsigned(nt)), dim3(256), 0, st, c->mr_rb.p, c->mr_tp.p, NW, W, tb,
                           scr_t.p, scr_r.p, base, d_time, d_rule);
      }
      HIPCHK(hipGetLastError());
    }
    n0 = n1;
  }
  // the host arrays above are read by the queued copies: drain before they go
  return cg_hip_check(hipStreamSynchronize(st), "time-ordered gather merge");
}

extern "C" {

int cg_node_csr_merge_ranks(cg_ctx* c, int32_t n_nodes, int32_t world, const int64_t* run_bounds, int64_t* d_time,
                            int32_t* d_rule, int64_t budget_bytes) {
  if (!c || n_nodes < 0 || world < 1 || budget_bytes < 12 || (n_nodes > 0 && world > 1 && (!run_bounds || !d_time || !d_rule)))
    return cg_fail(CG_EINVAL, "cg_node_csr_merge_ranks: bad argument");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  return merge_ranks_locked(c, c->st, n_nodes, world, run_bounds, d_time, d_rule, budget_bytes / 12, c->mr_t,
                            c->mr_r);
}

int cg_node_checksum_enqueue(cg_ctx* c, const int32_t* d_nodes, int32_t k, uint64_t* d_out) {
  if (!c || k < 0 || (k > 0 && (!d_nodes || !d_out))) return cg_fail(CG_EINVAL, "cg_node_checksum_enqueue: bad argument");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  // the lists of the last enqueued window (pipelined) or of the last result
  const int64_t* off = nullptr;
  int32_t N = 0;
  if (pn_async_pending(c) && c->pa_last >= 0) {
    off = c->pns[c->pa_last].node_off.p;
    N = c->pns[c->pa_last].N;
  } else {
    if (c->pn_E == 0 && c->pn_N == 0) return cg_fail(CG_EINVAL, "cg_node_checksum_enqueue: no per-node result");
    off = c->node_off.p;
    N = int32_t(c->pn_N);
  }
  const int64_t cap = int64_t(std::min(c->node_time.cap, c->node_rule.cap));
  if (k > 0)
    hipLaunchKernelGGL(k_node_checksums, dim3(unsigned(k)), dim3(256), 0, c->st, off, N, cap, c->node_time.p,
                       c->node_rule.p, d_nodes, reinterpret_cast<unsigned long long*>(d_out));
  return cg_hip_check(hipGetLastError(), "k_node_checksums");
}

int cg_node_counts_to_device(cg_ctx* c, int64_t* d_counts) {
  if (!c || !d_counts) return cg_fail(CG_EINVAL, "cg_node_counts_to_device: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (pn_async_pending(c))
    return cg_fail(CG_EINVAL, "pipelined per-node windows pending (call cg_expand_per_node_wait first)");
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  if (c->pn_N > 0)
    hipLaunchKernelGGL(k_node_counts, dim3(gridn(c->pn_N, 256, 1 << 30)), dim3(256), 0, c->st,
                       c->node_off.p, int32_t(c->pn_N), d_counts);
  if ((rc = cg_hip_check(hipGetLastError(), "k_node_counts"))) return rc;
  return cg_hip_check(hipStreamSynchronize(c->st), "sync");
}

}  // extern "C"
