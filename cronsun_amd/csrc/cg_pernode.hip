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
//   radix sort (node)    stable transpose to node -> rules (rocPRIM)
//   k_node_bounds        per-node pair offsets (lower bound per node)
//   pair event counts -> scan -> per-node offsets
//   k_node_write         output-parallel copy of each rule's fire times into
//                        every node list that contains the rule (whole
//                        64-event blocks, pairs found by shuffle search)
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
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

template <bool WRITE>
__global__ __launch_bounds__(256) void k_rule_nodes(RulesDev d, int mode, int wpb,
                                                     int32_t* __restrict__ rn_cnt,
                                                     const int64_t* __restrict__ rn_off,
                                                     int32_t* __restrict__ rn_nodes,
                                                     int32_t* __restrict__ pair_rule) {
  extern __shared__ uint32_t bm_all[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= wpb) return;
  uint32_t* bm = bm_all + size_t(wave) * d.words;
  for (int64_t r = int64_t(blockIdx.x) * wpb + wave; r < d.R; r += int64_t(gridDim.x) * wpb) {
    for (int w = lane; w < d.words; w += 64) bm[w] = 0;
    wave_sync_lds();
    const int32_t job = d.rule_job[r];
    if (!d.job_pause[job]) {  // job.go:593
      for (int64_t k = d.nid_off[r] + lane; k < d.nid_off[r + 1]; k += 64) bm_set(bm, d.nids[k], d.N);
      for (int64_t k = d.gid_off[r]; k < d.gid_off[r + 1]; k++) {
        int32_t g = d.gids[k];
        if (g < 0 || g >= d.G || !d.group_exists[g]) continue;  // gs[gid] missing
        for (int64_t q = d.group_off[g] + lane; q < d.group_off[g + 1]; q += 64)
          bm_set(bm, d.group_nodes[q], d.N);
      }
      wave_sync_lds();
      if (mode == CG_EXCLUDE_RULE) {
        for (int64_t k = d.ex_off[r] + lane; k < d.ex_off[r + 1]; k += 64) bm_clear(bm, d.ex[k], d.N);
      } else if (mode == CG_EXCLUDE_CUMULATIVE) {
        int64_t r0 = r;
        while (r0 > 0 && d.rule_job[r0 - 1] == job) r0--;
        for (int64_t q = r0; q <= r; q++)
          for (int64_t k = d.ex_off[q] + lane; k < d.ex_off[q + 1]; k += 64)
            bm_clear(bm, d.ex[k], d.N);
      }
      wave_sync_lds();
    }
    if (!WRITE) {
      int32_t c = 0;
      for (int w = lane; w < d.words; w += 64) c += __popc(bm[w]);
      for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
      if (lane == 0) rn_cnt[r] = c;
    } else {
      int64_t pos = rn_off[r];
      for (int base = 0; base < d.words; base += 64) {
        int w = base + lane;
        uint32_t bits = w < d.words ? bm[w] : 0u;
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
          pair_rule[p] = int32_t(r);
          p++;
        }
        pos += __shfl(inc, 63, 64);
      }
    }
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

// per (node, rule) pair: its event count and its rule's fire-list start
__global__ void k_pair_events(const int32_t* __restrict__ nt_rule, int64_t nnz,
                              const int64_t* __restrict__ rule_off, int32_t* __restrict__ ev,
                              int64_t* __restrict__ src) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < nnz;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int32_t r = nt_rule[i];
    const int64_t a = rule_off[r];
    ev[i] = int32_t(rule_off[r + 1] - a);
    src[i] = a;
  }
}

__global__ void k_node_offsets(const int64_t* __restrict__ nt_off, const int64_t* __restrict__ pair_pos,
                               int32_t N, int64_t* __restrict__ node_off) {
  int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n <= N) node_off[n] = pair_pos[nt_off[n]];
}

__global__ void k_node_counts(const int64_t* __restrict__ node_off, int32_t N, int64_t* __restrict__ out) {
  int64_t n = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (n < N) out[n] = node_off[n + 1] - node_off[n];
}

__device__ __forceinline__ int64_t search_le(const int64_t* __restrict__ off, int64_t lo, int64_t hi,
                                             int64_t x) {
  while (lo < hi) {
    int64_t mid = (lo + hi + 1) >> 1;
    if (off[mid] <= x) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// first pair touched by each kNodeTask-event output task
__global__ void k_pair_block_map(const int64_t* __restrict__ pair_pos, int64_t nnz, int64_t ntasks,
                                 int64_t* __restrict__ task_pair) {
  int64_t b = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (b > ntasks) return;
  task_pair[b] = b == ntasks ? nnz - 1 : search_le(pair_pos, 0, nnz - 1, b * int64_t(kNodeTask));
}

__device__ __forceinline__ int64_t rl64n(int64_t v, int i) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), i));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), i));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// Per-node lists: node event e copies fire k of the rule of its (node, rule)
// pair.  Waves take kNodeTask-event output tasks; a wave keeps 64 consecutive
// pairs in registers (lane i: pair jw + i, its output start, end, rule and
// the rule's fire-list start) and fills its task in aligned 64-event blocks:
// lane l finds the pair of event b + l by a 6-step shuffle search, gathers the
// fire time (rule lists are re-read once per node of the rule: L2/MALL hits)
// and the block is stored whole (8-B times, 4-B rule indices).  (Two blocks
// per round with independent searches measured slower: 7 waves per SIMD.)
// (A wave-uniform walk over the pairs instead of the search measured 1.5x
// slower: ~10 fires per pair make the per-pair readlane chain the bottleneck.)
template <int V>
__global__ __launch_bounds__(256) void k_node_write(
    const int64_t* __restrict__ pair_pos, const int32_t* __restrict__ nt_rule,
    const int64_t* __restrict__ task_pair, const int64_t* __restrict__ pair_src,
    const int64_t* __restrict__ times, int64_t En, int64_t nnz, int64_t* __restrict__ out_time,
    int32_t* __restrict__ out_rule) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t ntasks = (En + kNodeTask - 1) / kNodeTask;
  const int64_t nwaves = int64_t(gridDim.x) * (blockDim.x >> 6);
  for (int64_t t = int64_t(blockIdx.x) * (blockDim.x >> 6) + wave; t < ntasks; t += nwaves) {
    const int64_t B0 = t * kNodeTask;
    const int64_t B1 = En - B0 < kNodeTask ? En : B0 + kNodeTask;
    const int64_t jend = task_pair[t + 1] + 1;  // pairs this task can touch
    int64_t jw = task_pair[t];
    // lane i: pair jw + i as (output start - B0) clamped to int32, and the
    // fire-list shift delta = rule list start - output start (event e of the
    // pair reads times[e + delta]): 3 shuffles per event instead of 5, and
    // 32-bit search steps
    int32_t dst = INT32_MAX;
    int64_t delta = 0, dend = INT64_MAX;
    int32_t rr = 0;
    // the next window's raw loads are issued one window ahead
    int64_t n_d = INT64_MAX, n_dend = INT64_MAX, n_src = 0;
    int32_t n_r = 0;
    auto fetch = [&](int64_t base) {
      const int64_t p = base + lane;
      if (p < jend) {
        n_d = pair_pos[p];
        n_dend = pair_pos[p + 1];
        n_r = nt_rule[p];
        n_src = pair_src[p];
      } else {
        n_d = INT64_MAX;
      }
    };
    auto load = [&]() {  // window jw from the prefetched loads, then prefetch jw + 64
      if (n_d != INT64_MAX) {
        dend = n_dend;
        rr = n_r;
        delta = n_src - n_d;
        dst = int32_t(n_d - B0 < int64_t(INT32_MAX)
                          ? (n_d - B0 > INT32_MIN ? n_d - B0 : INT32_MIN + 1)
                          : INT32_MAX - 1);
      } else {
        dst = INT32_MAX;
        dend = INT64_MAX;
        rr = 0;
        delta = 0;
      }
      fetch(jw + 64);
    };
    fetch(jw);
    load();
    // jc: window lane of the pair that holds event b (wave-uniform), -1 when
    // unknown.  A full block inside that one pair (long fire lists: second-
    // granularity and frequent @every rules carry most node events) needs no
    // search: one uniform shift, a coalesced 512-B read and the stores.
    int jc = -1;
    for (int64_t b = B0; b < B1; b += 64) {
      const int64_t e = b + lane;
      int64_t val = 0;
      int32_t rv = 0;
      if (jc >= 0 && b + 64 <= B1 && rl64n(dend, jc) >= b + 64) {
        const int64_t d = rl64n(delta, jc);
        val = (V & 1) ? e + d : times[e + d];
        rv = __builtin_amdgcn_readlane(rr, jc);
      } else {
        bool done = e >= B1;
        int j = 0;
        for (;;) {
          const int L = 63 - __builtin_clzll(__ballot(dst != INT32_MAX));
          const int64_t wend = rl64n(dend, L);
          j = 0;
#pragma unroll
          for (int st = 32; st > 0; st >>= 1) {
            const int32_t v = __shfl(dst, (j + st) & 63, 64);
            if (j + st < 64 && int64_t(v) <= e - B0) j += st;
          }
          const int64_t jdelta = __shfl(delta, j, 64);
          const int32_t jr = __shfl(rr, j, 64);
          if (!done && e < wend) {
            val = (V & 1) ? e + jdelta : times[e + jdelta];
            rv = jr;
            done = true;
          }
          if (__ballot(!done) == 0) break;
          jw += 64;  // some lane's event lies past the window's last pair
          load();
        }
        // the pair of the block's last event, in the final window (a full
        // block's lane 63 is found in the last window visited)
        jc = b + 64 <= B1 ? __builtin_amdgcn_readlane(j, 63) : -1;
      }
      if (V & 2) {
        asm volatile("" ::"v"(val), "v"(rv));
      } else if (e < B1) {
        out_time[e] = val;
        out_rule[e] = rv;
      }
    }
  }
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
  if (size_t(words) * 4 > 64 * 1024) return cg_fail(CG_ERANGE, "more than 524288 nodes");
  hipStream_t s = c->st;
  int rc;
  if ((rc = c->rn_cnt.ensure(std::max(R, 1)))) return rc;
  if ((rc = c->rn_off.ensure(R + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(R))))) return rc;
  RulesDev d{st.nid_off.p, st.nids.p, st.gid_off.p, st.gids.p, st.ex_off.p, st.ex.p,
             st.rule_job.p, st.job_pause.p, st.group_off.p, st.group_nodes.p,
             st.group_exists.p, R, G, N, std::max(words, 1)};
  int wpb = int(std::min<size_t>(4, std::max<size_t>(1, (64 * 1024) / (size_t(d.words) * 4))));
  size_t lds = size_t(wpb) * d.words * 4;
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

int per_node_locked(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                    const RulesStore& in, int mode, int64_t* n_events, int64_t* nnz_out) {
  if (int64_t(s->n) != in.n_rules)
    return cg_fail(CG_EINVAL, "specs count != rules n_rules");
  int64_t E = 0;
  int rc = expand_device_locked(c, s, z, t0, t1, &E);
  if (rc) return rc;
  int64_t nnz = 0;
  const int32_t N = in.n_nodes;
  hipStream_t st = c->st;
  const bool cached = in.serial != 0 && in.serial == c->pn_cache_serial && mode == c->pn_cache_mode;
  (void)hipEventRecord(c->pev[0], c->st);
  if (cached) {
    nnz = c->pn_nnz;
  } else {
    c->pn_cache_serial = 0;  // the transpose buffers are about to change
    if ((rc = rule_nodes_locked(c, in, mode, &nnz))) return rc;
  }
  (void)hipEventRecord(c->pev[1], c->st);
  if ((rc = c->nt_off.ensure(N + 1))) return rc;
  if ((rc = c->nt_rule.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_node.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->node_off.ensure(N + 1))) return rc;
  // transpose: stable radix sort of (node, rule) pairs by node
  if (nnz > 0 && !cached) {
    unsigned end_bit = 1;
    while ((1u << end_bit) < unsigned(std::max(N, 2))) end_bit++;
    size_t tmp_bytes = 0;
    (void)rocprim::radix_sort_pairs(nullptr, tmp_bytes, reinterpret_cast<uint32_t*>(c->rn_nodes.p),
                              reinterpret_cast<uint32_t*>(c->pair_node.p), c->pair_rule.p,
                              c->nt_rule.p, size_t(nnz), 0, end_bit, st);
    if ((rc = c->pn_tmp.ensure(tmp_bytes + 16))) return rc;
    if ((rc = cg_hip_check(
             rocprim::radix_sort_pairs(c->pn_tmp.p, tmp_bytes,
                                       reinterpret_cast<uint32_t*>(c->rn_nodes.p),
                                       reinterpret_cast<uint32_t*>(c->pair_node.p), c->pair_rule.p,
                                       c->nt_rule.p, size_t(nnz), 0, end_bit, st),
             "radix_sort_pairs")))
      return rc;
  }
  if (!cached)
    hipLaunchKernelGGL(k_node_bounds, dim3(gridn(int64_t(N) + 1, 256, 1 << 30)), dim3(256), 0, st,
                       reinterpret_cast<const uint32_t*>(c->pair_node.p), nnz, N, c->nt_off.p);
  if ((rc = c->scan_tmp.ensure(std::max(scan_temp_bytes(N), scan_temp_bytes(nnz))))) return rc;
  // per-pair event counts -> positions
  if ((rc = c->rn_cnt.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_pos.ensure(nnz + 1))) return rc;
  if ((rc = c->pair_src.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if (nnz > 0)
    hipLaunchKernelGGL(k_pair_events, dim3(gridn(nnz, 256, 4096)), dim3(256), 0, st, c->nt_rule.p,
                       nnz, c->offsets.p, c->rn_cnt.p, c->pair_src.p);
  launch_scan(c->rn_cnt.p, c->pair_pos.p, nnz, c->scan_tmp.p, st);
  hipLaunchKernelGGL(k_node_offsets, dim3(gridn(N + 1, 256, 1 << 30)), dim3(256), 0, st,
                     c->nt_off.p, c->pair_pos.p, N, c->node_off.p);
  int64_t En = 0;
  if ((rc = cg_hip_check(hipMemcpyAsync(&En, c->pair_pos.p + nnz, 8, hipMemcpyDeviceToHost, st), "En")))
    return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  if ((rc = c->node_time.ensure(std::max<int64_t>(En, 1)))) return rc;
  if ((rc = c->node_rule.ensure(std::max<int64_t>(En, 1)))) return rc;
  const int64_t ntasks = (En + kNodeTask - 1) / kNodeTask;
  if ((rc = c->block_run.ensure(ntasks + 1))) return rc;
  (void)hipEventRecord(c->pev[2], st);
  if (En > 0) {
    hipLaunchKernelGGL(k_pair_block_map, dim3(gridn(ntasks + 1, 256, 1 << 30)), dim3(256), 0, st,
                       c->pair_pos.p, nnz, ntasks, c->block_run.p);
#ifdef CG_DIAG
    static const int variant = [] {  // diagnostic: 1 no gather, 2 no stores, 3 neither
      const char* e = getenv("CG_NODE_VARIANT");
      return e ? atoi(e) : 0;
    }();
    static const int per_cu = [] {  // persistent grid: blocks of 4 waves per CU
      const char* e = getenv("CG_NODE_BLOCKS_PER_CU");
      return e ? std::max(1, atoi(e)) : 8;
    }();
#else
    constexpr int variant = 0, per_cu = 8;
#endif
    const int nw_blocks = c->write_blocks / kWriteBlocksPerCU * per_cu;
#define CG_NW(V)                                                                              \
  hipLaunchKernelGGL(k_node_write<V>, dim3(gridn(ntasks, 4, nw_blocks)), dim3(256), 0, st,      \
                     c->pair_pos.p, c->nt_rule.p, c->block_run.p, c->pair_src.p, c->times.p, En, \
                     nnz, c->node_time.p, c->node_rule.p)
    switch (variant) {
      case 1: CG_NW(1); break;
      case 2: CG_NW(2); break;
      case 3: CG_NW(3); break;
      default: CG_NW(0); break;
    }
#undef CG_NW
  }
  (void)hipEventRecord(c->pev[3], st);
  if ((rc = cg_hip_check(hipGetLastError(), "per-node kernels"))) return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  (void)hipEventElapsedTime(&c->kt[6], c->pev[0], c->pev[1]);
  (void)hipEventElapsedTime(&c->kt[7], c->pev[1], c->pev[2]);
  (void)hipEventElapsedTime(&c->kt[8], c->pev[2], c->pev[3]);
  c->pn_E = En;
  c->pn_nnz = nnz;
  c->pn_N = N;
  c->pn_cache_serial = in.serial;
  c->pn_cache_mode = mode;
  *n_events = En;
  *nnz_out = nnz;
  return CG_OK;
}

}  // namespace

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
  if (d_node_off) *d_node_off = c->node_off.p;
  if (d_time) *d_time = c->node_time.p;
  if (d_rule) *d_rule = c->node_rule.p;
  if (n_events) *n_events = c->pn_E;
  return CG_OK;
}

int cg_node_result_copy(cg_ctx* c, int64_t* node_off, int64_t* time, int32_t* rule, int64_t cap) {
  if (!c) return cg_fail(CG_EINVAL, "cg_node_result_copy: null");
  std::lock_guard<std::mutex> g(c->mu);
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

int cg_node_counts_to_device(cg_ctx* c, int64_t* d_counts) {
  if (!c || !d_counts) return cg_fail(CG_EINVAL, "cg_node_counts_to_device: null");
  std::lock_guard<std::mutex> g(c->mu);
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
