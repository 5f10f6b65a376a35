// cg_comm.cpp -- the multi-GPU exchanges of include/cronsun_gpu.h over RCCL
// (xGMI between the MI355X of one node): the all-gather of per-node event
// counts / offsets and the chunked gather of the per-node CSR (north_star;
// SURVEY.md §8e).  Rules shard by job-ID range with no data-path collective:
// the reference's nodes each filter every job (node/node.go:121-141), here a
// rank evaluates one range of jobs for every node, and node n's global list
// is the ranks' slices in rank (= job-ID) order.
//
// RCCL is loaded at run time: the RCCL already in the process (torch's) or
// the one beside the HIP runtime this library links (its runpath), else
// /opt/rocm/lib -- so the library has no link-time dependency on RCCL and a
// process that also runs torch.distributed over RCCL holds one copy.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string err;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    // torch's copy is "librccl.so" (no soname; libtorch_hip needs that name)
    void* h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);  // this library's runpath: beside its HIP runtime
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("RCCL not loadable: ") + (e ? e : "librccl.so.1 not found");
      return;
    }
    bool all = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      if (!f) all = false;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    if (!all) {
      r.err = "RCCL library lacks an expected symbol";
      return;
    }
    r.ok = true;
  });
  return r;
}

int nccl_check(ncclResult_t e, const char* what) {
  if (e == ncclSuccess) return CG_OK;
  return cg_fail(CG_EHIP, std::string(what) + ": " + rccl().GetErrorString(e));
}

#define NCCLCHK(x, what)                  \
  do {                                    \
    int _rc = nccl_check((x), what);      \
    if (_rc != CG_OK) return _rc;         \
  } while (0)

}  // namespace

struct cg_comm {
  cg_ctx* ctx = nullptr;
  ncclComm_t nc = nullptr;
  int world = 0, rank = 0;
  DBuf<int64_t> scratch;       // small all-gathers
  DBuf<int64_t> cnt;           // [world * N] per-node counts
  DBuf<int64_t> off_all;       // [world * (N+1)] every rank's node offsets
  DBuf<int64_t> starts;        // [world * N] destinations of every rank's slices
  DBuf<int64_t> stage_t;       // root: one chunk of peer times
  DBuf<int32_t> stage_r;       // root: and rules
};

namespace {

// c->mu held.  all[g*n + i] = rank g's mine[i], through device scratch.
int allgather_locked(cg_comm* m, const int64_t* mine, size_t n, int64_t* all) {
  cg_ctx* c = m->ctx;
  const size_t tot = n * size_t(m->world);
  int rc = m->scratch.ensure(std::max<size_t>(tot, 1));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(m->scratch.p + size_t(m->rank) * n, mine, n * 8, hipMemcpyHostToDevice, c->st));
  NCCLCHK(rccl().AllGather(m->scratch.p + size_t(m->rank) * n, m->scratch.p, n, ncclInt64, m->nc, c->st),
          "ncclAllGather");
  HIPCHK(hipMemcpyAsync(all, m->scratch.p, tot * 8, hipMemcpyDeviceToHost, c->st));
  return cg_hip_check(hipStreamSynchronize(c->st), "allgather sync");
}

// every rank's per-node counts of its last per-node result -> m->cnt (device)
// and host_cnt [world * N]; c->mu held; every rank has N nodes (checked)
int node_counts_locked(cg_comm* m, int64_t N, std::vector<int64_t>& host_cnt) {
  cg_ctx* c = m->ctx;
  int rc;
  if ((rc = m->cnt.ensure(std::max<int64_t>(N * m->world, 1)))) return rc;
  if (N > 0) {
    if ((rc = launch_node_counts(c, c->st, m->cnt.p + int64_t(m->rank) * N))) return rc;
    NCCLCHK(rccl().AllGather(m->cnt.p + int64_t(m->rank) * N, m->cnt.p, size_t(N), ncclInt64, m->nc, c->st),
            "ncclAllGather(node counts)");
  }
  host_cnt.assign(size_t(N * m->world), 0);
  if (N > 0) HIPCHK(hipMemcpyAsync(host_cnt.data(), m->cnt.p, size_t(N * m->world) * 8, hipMemcpyDeviceToHost, c->st));
  return cg_hip_check(hipStreamSynchronize(c->st), "node counts sync");
}

// The chunks of the gather, the same on every rank: whole node ranges
// [n0, n1) whose peer events (every rank but root) fit cap_ev, and a node
// with more than cap_ev peer events in k parts (part j of peer g: its events
// [c*j/k, c*(j+1)/k) of that node, so a part holds at most
// P/k + world - 1 <= cap_ev events).  (cronsun_amd/shard.py restates it.)
struct Chunk {
  int64_t n0, n1, j, k;
};
std::vector<Chunk> gather_plan(const std::vector<int64_t>& cnt, int world, int64_t N, int root, int64_t cap_ev) {
  std::vector<Chunk> out;
  std::vector<int64_t> P(size_t(N), 0);
  for (int g = 0; g < world; g++)
    if (g != root)
      for (int64_t n = 0; n < N; n++) P[size_t(n)] += cnt[size_t(g * N + n)];
  int64_t n = 0;
  while (n < N) {
    if (P[size_t(n)] > cap_ev) {
      const int64_t per = cap_ev - (world - 1);
      const int64_t k = (P[size_t(n)] + per - 1) / per;
      for (int64_t j = 0; j < k; j++) out.push_back({n, n + 1, j, k});
      n++;
      continue;
    }
    const int64_t n0 = n;
    int64_t acc = 0;
    while (n < N && P[size_t(n)] <= cap_ev && acc + P[size_t(n)] <= cap_ev) acc += P[size_t(n++)];
    if (acc > 0) out.push_back({n0, n, 0, 1});
  }
  return out;
}

}  // namespace

extern "C" {

int cg_comm_unique_id(uint8_t id[CG_COMM_ID_BYTES]) {
  if (!id) return cg_fail(CG_EINVAL, "cg_comm_unique_id: null");
  const Rccl& r = rccl();
  if (!r.ok) return cg_fail(CG_ENODEV, r.err);
  static_assert(sizeof(ncclUniqueId) == CG_COMM_ID_BYTES, "unique id size");
  ncclUniqueId u;
  NCCLCHK(r.GetUniqueId(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, CG_COMM_ID_BYTES);
  return CG_OK;
}

int cg_comm_init(cg_ctx* c, int world, int rank, const uint8_t id[CG_COMM_ID_BYTES], cg_comm** out) {
  if (!c || !id || !out || world < 1 || rank < 0 || rank >= world) return cg_fail(CG_EINVAL, "cg_comm_init: bad argument");
  const Rccl& r = rccl();
  if (!r.ok) return cg_fail(CG_ENODEV, r.err);
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, CG_COMM_ID_BYTES);
  ncclComm_t nc = nullptr;
  NCCLCHK(r.CommInitRank(&nc, world, u, rank), "ncclCommInitRank");
  cg_comm* m = new cg_comm();
  m->ctx = c;
  m->nc = nc;
  m->world = world;
  m->rank = rank;
  *out = m;
  return CG_OK;
}

void cg_comm_free(cg_comm* m) {
  if (!m) return;
  {
    std::lock_guard<std::mutex> g(m->ctx->mu);
    (void)hipSetDevice(m->ctx->device);
    (void)hipStreamSynchronize(m->ctx->st);
    if (m->nc) (void)rccl().CommDestroy(m->nc);
    m->scratch.release();
    m->cnt.release();
    m->off_all.release();
    m->starts.release();
    m->stage_t.release();
    m->stage_r.release();
  }
  delete m;
}

int cg_comm_allgather_i64(cg_comm* m, const int64_t* mine, size_t n, int64_t* all) {
  if (!m || (n && (!mine || !all))) return cg_fail(CG_EINVAL, "cg_comm_allgather_i64: null");
  cg_ctx* c = m->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return CG_OK;
  return allgather_locked(m, mine, n, all);
}

int cg_comm_node_offsets(cg_comm* m, int64_t* node_start, int64_t* node_base) {
  if (!m) return cg_fail(CG_EINVAL, "cg_comm_node_offsets: null");
  cg_ctx* c = m->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  // every rank's node count and whether it has a readable result
  const int64_t mine[2] = {c->pn_N, pn_async_pending(c) ? 1 : 0};
  std::vector<int64_t> meta(size_t(2 * m->world));
  int rc = allgather_locked(m, mine, 2, meta.data());
  if (rc) return rc;
  for (int q = 0; q < m->world; q++) {
    if (meta[size_t(2 * q)] != c->pn_N) return cg_fail(CG_EINVAL, "cg_comm_node_offsets: ranks differ in node count");
    if (meta[size_t(2 * q + 1)])
      return cg_fail(CG_EINVAL, "cg_comm_node_offsets: a rank has pipelined per-node windows pending");
  }
  const int64_t N = c->pn_N;
  std::vector<int64_t> cnt;
  if ((rc = node_counts_locked(m, N, cnt))) return rc;
  int64_t base = 0;
  for (int64_t n = 0; n < N; n++) {
    int64_t before = 0, tot = 0;
    for (int q = 0; q < m->world; q++) {
      const int64_t v = cnt[size_t(q * N + n)];
      if (q < m->rank) before += v;
      tot += v;
    }
    if (node_base) node_base[n] = base;
    if (node_start) node_start[n] = base + before;
    base += tot;
  }
  if (node_base) node_base[N] = base;
  return CG_OK;
}

int cg_comm_gather_node_csr(cg_comm* m, int root, int64_t rule_base, int64_t budget_bytes, int64_t* d_node_off,
                            int64_t* d_time, int32_t* d_rule, int64_t cap, int64_t* n_events) {
  constexpr int kMeta = 6;  // node count, events, ok, rule_base, cap, budget
  if (!m || root < 0 || root >= m->world) return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: bad argument");
  cg_ctx* c = m->ctx;
  const int W = m->world, me = m->rank;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  // every rank's preconditions travel with one all-gather, so every rank
  // returns the same status instead of leaving its peers blocked in a transfer
  const bool local_ok = !pn_async_pending(c) && !c->pn_time_ordered && rule_base >= 0 && rule_base <= INT32_MAX &&
                        (me != root || ((d_node_off && d_time && d_rule) || c->pn_N == 0)) && budget_bytes > 0;
  const int64_t mine[kMeta] = {c->pn_N, c->pn_E, local_ok ? 1 : 0, rule_base, cap, budget_bytes};
  std::vector<int64_t> meta(size_t(kMeta * W));
  int rc = allgather_locked(m, mine, kMeta, meta.data());
  if (rc) return rc;
  const int64_t N = c->pn_N;
  int64_t total = 0;
  for (int q = 0; q < W; q++) {
    const int64_t* mq = &meta[size_t(kMeta * q)];
    if (mq[0] != N) return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: ranks differ in node count");
    if (!mq[2])
      return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: rank " + std::to_string(q) +
                                    " has no gatherable result (pending windows, a time-ordered result, a bad "
                                    "rule_base or budget, or null output buffers on root)");
    total += mq[1];
  }
  if (n_events) *n_events = total;
  const int64_t root_cap = meta[size_t(kMeta * root + 4)];
  if (total > root_cap)
    return cg_fail(CG_ECAPACITY, "cg_comm_gather_node_csr: " + std::to_string(total) +
                                     " node events exceed root's capacity " + std::to_string(root_cap));
  // every rank plans the chunks with the same budget: the smallest passed
  int64_t budget = INT64_MAX;
  for (int q = 0; q < W; q++) budget = std::min(budget, meta[size_t(kMeta * q + 5)]);
  const int64_t cap_ev = budget / 12;
  if (W > 1 && cap_ev < 2 * int64_t(W))
    return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: budget below 24 bytes per rank");
  std::vector<int64_t> cnt;
  if ((rc = node_counts_locked(m, N, cnt))) return rc;
  // every rank's node offsets, and the destinations of every rank's slices
  std::vector<int64_t> off(size_t(W * (N + 1))), st(size_t(W * N)), base(size_t(N + 1));
  for (int q = 0; q < W; q++) {
    int64_t a = 0;
    for (int64_t n = 0; n < N; n++) {
      off[size_t(q * (N + 1) + n)] = a;
      a += cnt[size_t(q * N + n)];
    }
    off[size_t(q * (N + 1) + N)] = a;
  }
  int64_t b = 0;
  for (int64_t n = 0; n < N; n++) {
    base[size_t(n)] = b;
    for (int q = 0; q < W; q++) {
      st[size_t(q * N + n)] = b;
      b += cnt[size_t(q * N + n)];
    }
  }
  base[size_t(N)] = b;
  const std::vector<Chunk> plan = gather_plan(cnt, W, N, root, cap_ev);
  hipStream_t s = c->st;
  if (me == root) {
    if (N > 0) {
      if ((rc = m->off_all.ensure(size_t(W * (N + 1)))) || (rc = m->starts.ensure(size_t(W * N)))) return rc;
      HIPCHK(hipMemcpyAsync(m->off_all.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(m->starts.p, st.data(), st.size() * 8, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(d_node_off, base.data(), base.size() * 8, hipMemcpyHostToDevice, s));
    }
    int64_t stage = 1;
    for (const Chunk& ch : plan) {
      int64_t ev = 0;
      for (int q = 0; q < W; q++) {
        if (q == root) continue;
        const int64_t cq = cnt[size_t(q * N + ch.n0)];
        ev += ch.k == 1 ? off[size_t(q * (N + 1) + ch.n1)] - off[size_t(q * (N + 1) + ch.n0)]
                        : cq * (ch.j + 1) / ch.k - cq * ch.j / ch.k;
      }
      stage = std::max(stage, ev);
    }
    if (!plan.empty() && ((rc = m->stage_t.ensure(size_t(stage))) || (rc = m->stage_r.ensure(size_t(stage)))))
      return rc;
    // root's own slice, straight from its result
    if (N > 0 && (rc = launch_node_place(c, s, int32_t(N), c->node_off.p, c->node_time.p, c->node_rule.p,
                                         int32_t(rule_base), m->starts.p + int64_t(root) * N, d_time, d_rule)))
      return rc;
  }
  for (const Chunk& ch : plan) {
    // peer q's piece: its events [lo, hi) of its own CSR
    auto piece = [&](int q, int64_t* lo, int64_t* hi) {
      const int64_t a = off[size_t(q * (N + 1) + ch.n0)];
      if (ch.k == 1) {
        *lo = a;
        *hi = off[size_t(q * (N + 1) + ch.n1)];
      } else {
        const int64_t cq = cnt[size_t(q * N + ch.n0)];
        *lo = a + cq * ch.j / ch.k;
        *hi = a + cq * (ch.j + 1) / ch.k;
      }
    };
    NCCLCHK(rccl().GroupStart(), "ncclGroupStart");
    if (me == root) {
      int64_t o = 0;
      for (int q = 0; q < W; q++) {
        if (q == root) continue;
        int64_t lo, hi;
        piece(q, &lo, &hi);
        if (hi > lo) {
          NCCLCHK(rccl().Recv(m->stage_t.p + o, size_t(hi - lo), ncclInt64, q, m->nc, s), "ncclRecv");
          NCCLCHK(rccl().Recv(m->stage_r.p + o, size_t(hi - lo), ncclInt32, q, m->nc, s), "ncclRecv");
        }
        o += hi - lo;
      }
    } else {
      int64_t lo, hi;
      piece(me, &lo, &hi);
      if (hi > lo) {
        NCCLCHK(rccl().Send(c->node_time.p + lo, size_t(hi - lo), ncclInt64, root, m->nc, s), "ncclSend");
        NCCLCHK(rccl().Send(c->node_rule.p + lo, size_t(hi - lo), ncclInt32, root, m->nc, s), "ncclSend");
      }
    }
    NCCLCHK(rccl().GroupEnd(), "ncclGroupEnd");
    if (me != root) continue;
    // place the chunk (same stream: after the receives, before the next chunk's)
    int64_t o = 0;
    for (int q = 0; q < W; q++) {
      if (q == root) continue;
      int64_t lo, hi;
      piece(q, &lo, &hi);
      const int32_t add = int32_t(meta[size_t(kMeta * q + 3)]);
      if (hi > lo) {
        if (ch.k == 1) {
          // src indexed by the peer's own positions: shift the stage base by lo
          rc = launch_node_place(c, s, int32_t(ch.n1 - ch.n0), m->off_all.p + int64_t(q) * (N + 1) + ch.n0,
                                 m->stage_t.p + o - lo, m->stage_r.p + o - lo, add,
                                 m->starts.p + int64_t(q) * N + ch.n0, d_time, d_rule);
        } else {
          const int64_t dst = st[size_t(q * N + ch.n0)] + (lo - off[size_t(q * (N + 1) + ch.n0)]);
          rc = launch_span_place(c, s, hi - lo, m->stage_t.p + o, m->stage_r.p + o, add, d_time + dst, d_rule + dst);
        }
        if (rc) return rc;
      }
      o += hi - lo;
    }
  }
  return cg_hip_check(hipStreamSynchronize(s), "gather sync");
}

}  // extern "C"
