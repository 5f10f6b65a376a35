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
//   pair event counts -> scan -> per-node offsets
//   k_node_write         output-parallel copy of each rule's fire times into
//                        every node list that contains the rule
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
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

__global__ void k_histogram(const int32_t* __restrict__ keys, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    atomicAdd(&cnt[keys[i]], 1);
}

__global__ void k_pair_events(const int32_t* __restrict__ nt_rule, int64_t nnz,
                              const int64_t* __restrict__ rule_off, int32_t* __restrict__ ev) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < nnz;
       i += int64_t(gridDim.x) * blockDim.x) {
    int32_t r = nt_rule[i];
    ev[i] = int32_t(rule_off[r + 1] - rule_off[r]);
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

__global__ void k_pair_block_map(const int64_t* __restrict__ pair_pos, int64_t nnz, int64_t nblocks,
                                 int64_t* __restrict__ block_pair) {
  int64_t b = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
  if (b > nblocks) return;
  block_pair[b] = b == nblocks ? nnz - 1 : search_le(pair_pos, 0, nnz - 1, b * int64_t(kWriteChunk));
}

constexpr int kStride = kWritePerThread + 1;

__global__ __launch_bounds__(kWriteThreads) void k_node_write(
    const int64_t* __restrict__ pair_pos, const int32_t* __restrict__ nt_rule,
    const int64_t* __restrict__ block_pair, const int64_t* __restrict__ rule_off,
    const int64_t* __restrict__ times, int64_t En, int64_t* __restrict__ out_time,
    int32_t* __restrict__ out_rule) {
  __shared__ int64_t st_t[kWriteThreads * kStride];
  __shared__ int32_t st_r[kWriteThreads * kStride];
  const int64_t B0 = int64_t(blockIdx.x) * kWriteChunk;
  int64_t i = B0 + int64_t(threadIdx.x) * kWritePerThread;
  if (i < En) {
    int64_t p = search_le(pair_pos, block_pair[blockIdx.x], block_pair[blockIdx.x + 1], i);
    int64_t k = i - pair_pos[p];
    int64_t n = pair_pos[p + 1] - pair_pos[p];
    int32_t r = nt_rule[p];
    const int64_t* src = times + rule_off[r];
    for (int q = 0; q < kWritePerThread && i < En; q++, i++, k++) {
      while (k >= n) {
        p++;
        k = 0;
        n = pair_pos[p + 1] - pair_pos[p];
        r = nt_rule[p];
        src = times + rule_off[r];
      }
      st_t[threadIdx.x * kStride + q] = src[k];
      st_r[threadIdx.x * kStride + q] = r;
    }
  }
  __syncthreads();
  const int64_t lim = En - B0;
  for (int e = threadIdx.x; e < kWriteChunk; e += kWriteThreads) {
    if (e >= lim) break;
    int t = e / kWritePerThread, q = e % kWritePerThread;
    out_time[B0 + e] = st_t[t * kStride + q];
    out_rule[B0 + e] = st_r[t * kStride + q];
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

// builds the rule->node CSR on the device; leaves rn_off/rn_nodes/pair_rule in ctx
int rule_nodes_locked(cg_ctx* c, const cg_rules_in* in, int mode, int64_t* nnz_out) {
  int rc = validate_rules(in);
  if (rc) return rc;
  if (mode < 0 || mode > 2) return cg_fail(CG_EINVAL, "bad exclude mode");
  const int32_t R = in->n_rules, G = in->n_groups, N = in->n_nodes;
  const int32_t words = (N + 31) / 32;
  if (size_t(words) * 4 > 64 * 1024) return cg_fail(CG_ERANGE, "more than 524288 nodes");
  hipStream_t st = c->st;
  const int64_t n_nid = R ? in->nid_off[R] : 0, n_gid = R ? in->gid_off[R] : 0,
                n_ex = R ? in->ex_off[R] : 0, n_gn = G ? in->group_off[G] : 0;
  if ((rc = upload(c->d_nid_off, in->nid_off, R ? R + 1 : 0, st))) return rc;
  if ((rc = upload(c->d_nids, in->nids, n_nid, st))) return rc;
  if ((rc = upload(c->d_gid_off, in->gid_off, R ? R + 1 : 0, st))) return rc;
  if ((rc = upload(c->d_gids, in->gids, n_gid, st))) return rc;
  if ((rc = upload(c->d_ex_off, in->ex_off, R ? R + 1 : 0, st))) return rc;
  if ((rc = upload(c->d_ex, in->ex, n_ex, st))) return rc;
  if ((rc = upload(c->d_rule_job, in->rule_job, R, st))) return rc;
  if ((rc = upload(c->d_job_pause, in->job_pause, in->n_jobs, st))) return rc;
  if ((rc = upload(c->d_group_off, in->group_off, G ? G + 1 : 0, st))) return rc;
  if ((rc = upload(c->d_group_nodes, in->group_nodes, n_gn, st))) return rc;
  if ((rc = upload(c->d_group_exists, in->group_exists, G, st))) return rc;
  if ((rc = c->rn_cnt.ensure(std::max(R, 1)))) return rc;
  if ((rc = c->rn_off.ensure(R + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(std::max(c->scan_tmp.cap, scan_temp_bytes(R))))) return rc;
  RulesDev d{c->d_nid_off.p, c->d_nids.p, c->d_gid_off.p, c->d_gids.p, c->d_ex_off.p, c->d_ex.p,
             c->d_rule_job.p, c->d_job_pause.p, c->d_group_off.p, c->d_group_nodes.p,
             c->d_group_exists.p, R, G, N, std::max(words, 1)};
  int wpb = int(std::min<size_t>(4, std::max<size_t>(1, (64 * 1024) / (size_t(d.words) * 4))));
  size_t lds = size_t(wpb) * d.words * 4;
  int grid = gridn(R, wpb, 256 * 16);
  if (R > 0)
    hipLaunchKernelGGL(k_rule_nodes<false>, dim3(grid), dim3(64 * wpb), lds, st, d, mode, wpb,
                       c->rn_cnt.p, nullptr, nullptr, nullptr);
  launch_scan(c->rn_cnt.p, c->rn_off.p, R, c->scan_tmp.p, st);
  int64_t nnz = 0;
  if ((rc = cg_hip_check(hipMemcpyAsync(&nnz, c->rn_off.p + R, 8, hipMemcpyDeviceToHost, st), "nnz")))
    return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  if ((rc = c->rn_nodes.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_rule.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if (R > 0 && nnz > 0)
    hipLaunchKernelGGL(k_rule_nodes<true>, dim3(grid), dim3(64 * wpb), lds, st, d, mode, wpb,
                       nullptr, c->rn_off.p, c->rn_nodes.p, c->pair_rule.p);
  if ((rc = cg_hip_check(hipGetLastError(), "k_rule_nodes"))) return rc;
  *nnz_out = nnz;
  return CG_OK;
}

int per_node_locked(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                    const cg_rules_in* in, int mode, int64_t* n_events, int64_t* nnz_out) {
  if (int64_t(s->n) != in->n_rules)
    return cg_fail(CG_EINVAL, "specs count != rules n_rules");
  int64_t E = 0;
  int rc = expand_device_locked(c, s, z, t0, t1, &E);
  if (rc) return rc;
  int64_t nnz = 0;
  if ((rc = rule_nodes_locked(c, in, mode, &nnz))) return rc;
  const int32_t N = in->n_nodes;
  hipStream_t st = c->st;
  if ((rc = c->node_cnt32.ensure(std::max(N, 1)))) return rc;
  if ((rc = c->nt_off.ensure(N + 1))) return rc;
  if ((rc = c->nt_rule.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_node.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->node_off.ensure(N + 1))) return rc;
  // transpose: stable radix sort of (node, rule) pairs by node
  if (nnz > 0) {
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
  if ((rc = cg_hip_check(hipMemsetAsync(c->node_cnt32.p, 0, size_t(std::max(N, 1)) * 4, st), "memset")))
    return rc;
  if (nnz > 0)
    hipLaunchKernelGGL(k_histogram, dim3(gridn(nnz, 256, 4096)), dim3(256), 0, st, c->pair_node.p,
                       nnz, c->node_cnt32.p);
  if ((rc = c->scan_tmp.ensure(std::max(scan_temp_bytes(N), scan_temp_bytes(nnz))))) return rc;
  launch_scan(c->node_cnt32.p, c->nt_off.p, N, c->scan_tmp.p, st);
  // per-pair event counts -> positions
  if ((rc = c->rn_cnt.ensure(std::max<int64_t>(nnz, 1)))) return rc;
  if ((rc = c->pair_pos.ensure(nnz + 1))) return rc;
  if (nnz > 0)
    hipLaunchKernelGGL(k_pair_events, dim3(gridn(nnz, 256, 4096)), dim3(256), 0, st, c->nt_rule.p,
                       nnz, c->offsets.p, c->rn_cnt.p);
  launch_scan(c->rn_cnt.p, c->pair_pos.p, nnz, c->scan_tmp.p, st);
  hipLaunchKernelGGL(k_node_offsets, dim3(gridn(N + 1, 256, 1 << 30)), dim3(256), 0, st,
                     c->nt_off.p, c->pair_pos.p, N, c->node_off.p);
  int64_t En = 0;
  if ((rc = cg_hip_check(hipMemcpyAsync(&En, c->pair_pos.p + nnz, 8, hipMemcpyDeviceToHost, st), "En")))
    return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  if ((rc = c->node_time.ensure(std::max<int64_t>(En, 1)))) return rc;
  if ((rc = c->node_rule.ensure(std::max<int64_t>(En, 1)))) return rc;
  const int64_t nblocks = (En + kWriteChunk - 1) / kWriteChunk;
  if ((rc = c->block_run.ensure(nblocks + 1))) return rc;
  if (En > 0) {
    hipLaunchKernelGGL(k_pair_block_map, dim3(gridn(nblocks + 1, 256, 1 << 30)), dim3(256), 0, st,
                       c->pair_pos.p, nnz, nblocks, c->block_run.p);
    hipLaunchKernelGGL(k_node_write, dim3(nblocks), dim3(kWriteThreads), 0, st, c->pair_pos.p,
                       c->nt_rule.p, c->block_run.p, c->offsets.p, c->times.p, En, c->node_time.p,
                       c->node_rule.p);
  }
  if ((rc = cg_hip_check(hipGetLastError(), "per-node kernels"))) return rc;
  if ((rc = cg_hip_check(hipStreamSynchronize(st), "sync"))) return rc;
  c->pn_E = En;
  c->pn_nnz = nnz;
  c->pn_N = N;
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
  if ((rc = rule_nodes_locked(c, in, mode, nnz))) return rc;
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
  return per_node_locked(c, s, z, t0, t1, rules, mode, n_events, nnz);
}

int cg_expand_per_node(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                       const cg_rules_in* rules, int mode, cg_node_csr* out) {
  if (!c || !s || !z || !rules || !out) return cg_fail(CG_EINVAL, "cg_expand_per_node: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int rc = cg_hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  int64_t En = 0, nnz = 0;
  if ((rc = per_node_locked(c, s, z, t0, t1, rules, mode, &En, &nnz))) return rc;
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
