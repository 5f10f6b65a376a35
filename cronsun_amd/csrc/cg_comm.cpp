// cg_comm.cpp -- the multi-GPU exchanges of include/cronsun_gpu.h over RCCL
// (xGMI between the MI355X of one node): the all-gather of per-node event
// counts / offsets and the chunked gather of the per-node CSR (north_star;
// SURVEY.md §8e).  Rules shard by job-ID range with no data-path collective:
// the reference's nodes each filter every job (node/node.go:121-141), here a
// rank evaluates one range of jobs for every node, and node n's global list
// is the ranks' slices in rank (= job-ID) order -- or, for time-ordered
// results, those slices merged by (time, rule) (the byTime order of the node's
// Cron, node/cron/cron.go:64-79,220).
//
// RCCL is loaded at run time, one copy per process: the RCCL already mapped
// (e.g. torch's), else the librccl.so beside the HIP runtime this library
// runs on (with PyTorch-ROCm: torch's own copy, so a torch imported later maps
// the same file), else /opt/rocm/lib -- always by full path and RTLD_LOCAL, so
// the name "librccl.so" never resolves a later DT_NEEDED to our copy and our
// symbols never interpose on another copy's users.  A second, different RCCL
// mapped afterwards makes every cg_comm call fail (cg_last_error names both)
// instead of mixing the two.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <link.h>
#include <rccl/rccl.h>
#include <sys/stat.h>

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
  std::string err, path;
  dev_t dev = 0;
  ino_t ino = 0;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclAllGather) AllGather = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
};

bool is_rccl_name(const char* path) {
  const char* b = strrchr(path, '/');
  b = b ? b + 1 : path;
  return strncmp(b, "librccl.so", 10) == 0;
}

// every RCCL file mapped in this process (distinct files)
struct Mapped {
  std::vector<std::string> paths;
  std::vector<std::pair<dev_t, ino_t>> ids;
};
Mapped mapped_rccl() {
  Mapped m;
  dl_iterate_phdr(
      [](dl_phdr_info* info, size_t, void* arg) -> int {
        Mapped& mm = *static_cast<Mapped*>(arg);
        if (!info->dlpi_name || !*info->dlpi_name || !is_rccl_name(info->dlpi_name)) return 0;
        struct stat sb;
        if (stat(info->dlpi_name, &sb) != 0) return 0;
        for (auto& id : mm.ids)
          if (id.first == sb.st_dev && id.second == sb.st_ino) return 0;
        mm.ids.push_back({sb.st_dev, sb.st_ino});
        mm.paths.push_back(info->dlpi_name);
        return 0;
      },
      &m);
  return m;
}

// the directory of the HIP runtime this library runs on
std::string hip_runtime_dir() {
  Dl_info di;
  if (!dladdr(reinterpret_cast<void*>(static_cast<hipError_t (*)(void**, size_t)>(&hipMalloc)), &di) || !di.dli_fname) return "";
  std::string p = di.dli_fname;
  const size_t s = p.rfind('/');
  return s == std::string::npos ? "" : p.substr(0, s);
}

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    const Mapped m = mapped_rccl();
    if (!m.paths.empty()) {  // already in the process (torch.distributed's)
      h = dlopen(m.paths[0].c_str(), RTLD_NOW | RTLD_NOLOAD);
      if (h) r.path = m.paths[0];
    }
    std::vector<std::string> cand;
    const std::string hd = hip_runtime_dir();
    if (!hd.empty()) cand.push_back(hd + "/librccl.so");
    cand.push_back("/opt/rocm/lib/librccl.so.1");
    for (size_t i = 0; !h && i < cand.size(); i++) {
      struct stat sb;
      if (stat(cand[i].c_str(), &sb) != 0) continue;
      h = dlopen(cand[i].c_str(), RTLD_NOW | RTLD_LOCAL);
      if (h) r.path = cand[i];
    }
    if (!h) {
      const char* e = dlerror();
      r.err = std::string("RCCL not loadable: ") + (e ? e : "no librccl.so beside the HIP runtime or in /opt/rocm/lib");
      return;
    }
    struct stat sb;
    if (stat(r.path.c_str(), &sb) == 0) {
      r.dev = sb.st_dev;
      r.ino = sb.st_ino;
    }
    bool all = true;
    auto sym = [&](auto& f, const char* name) {
      f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(h, name));
      if (!f) all = false;
    };
    sym(r.GetUniqueId, "ncclGetUniqueId");
    sym(r.CommInitRank, "ncclCommInitRank");
    sym(r.CommDestroy, "ncclCommDestroy");
    sym(r.CommAbort, "ncclCommAbort");
    sym(r.AllGather, "ncclAllGather");
    sym(r.Send, "ncclSend");
    sym(r.Recv, "ncclRecv");
    sym(r.GroupStart, "ncclGroupStart");
    sym(r.GroupEnd, "ncclGroupEnd");
    sym(r.GetErrorString, "ncclGetErrorString");
    if (!all) {
      r.err = "RCCL library " + r.path + " lacks an expected symbol";
      return;
    }
    r.ok = true;
  });
  return r;
}

// RCCL usable, and no other RCCL file mapped beside ours (a second copy --
// e.g. a torch imported after the first cg_comm call that found its RCCL
// elsewhere -- would mix two libraries' state in one process)
int rccl_ready() {
  const Rccl& r = rccl();
  if (!r.ok) return cg_fail(CG_ENODEV, r.err);
  const Mapped m = mapped_rccl();
  for (size_t i = 0; i < m.ids.size(); i++)
    if (m.ids[i].first != r.dev || m.ids[i].second != r.ino)
      return cg_fail(CG_EINVAL, "two RCCL libraries in this process: " + r.path + " (used by cg_comm) and " +
                                    m.paths[i] + " (mapped later); load the host's RCCL before the first cg_comm call");
  return CG_OK;
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
  ncclComm_t nc = nullptr;  // null after an abort
  int world = 0, rank = 0;
  DBuf<int64_t> scratch;       // small all-gathers
  DBuf<int64_t> cnt;           // [world * N] per-node counts
  DBuf<int64_t> off_all;       // [world * (N+1)] every rank's node offsets
  DBuf<int64_t> starts;        // [world * N] destinations of every rank's slices
  DBuf<int64_t> stage_t;       // root: one chunk of peer times (and the merge's scratch)
  DBuf<int32_t> stage_r;       // root: and rules
};

namespace {

int comm_usable(cg_comm* m) {
  int rc = rccl_ready();
  if (rc) return rc;
  if (!m->nc) return cg_fail(CG_EHIP, "cg_comm: the communicator was aborted by an earlier failed transfer");
  return CG_OK;
}

// A transfer failed after every rank agreed to run it: peers may be blocked in
// the matching send/receive, so the communicator is aborted (their RCCL calls
// then fail instead of waiting forever) and refuses every later call.
void abort_comm(cg_comm* m) {
  if (m->nc) (void)rccl().CommAbort(m->nc);
  m->nc = nullptr;
}

// c->mu held.  all[g*n + i] = rank g's mine[i], through device scratch.
int allgather_locked(cg_comm* m, const int64_t* mine, size_t n, int64_t* all) {
  cg_ctx* c = m->ctx;
  const size_t tot = n * size_t(m->world);
  int rc = m->scratch.ensure(std::max<size_t>(tot, 1));
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(m->scratch.p + size_t(m->rank) * n, mine, n * 8, hipMemcpyHostToDevice, c->st));
  rc = nccl_check(rccl().AllGather(m->scratch.p + size_t(m->rank) * n, m->scratch.p, n, ncclInt64, m->nc, c->st),
                  "ncclAllGather");
  if (rc) {
    abort_comm(m);
    return rc;
  }
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
    rc = nccl_check(rccl().AllGather(m->cnt.p + int64_t(m->rank) * N, m->cnt.p, size_t(N), ncclInt64, m->nc, c->st),
                    "ncclAllGather(node counts)");
    if (rc) {
      abort_comm(m);
      return rc;
    }
  }
  host_cnt.assign(size_t(N * m->world), 0);
  if (N > 0) HIPCHK(hipMemcpyAsync(host_cnt.data(), m->cnt.p, size_t(N * m->world) * 8, hipMemcpyDeviceToHost, c->st));
  return cg_hip_check(hipStreamSynchronize(c->st), "node counts sync");
}

// The chunks of the gather, the same on every rank: whole node ranges
// [n0, n1) whose peer events (every rank but root) fit cap_ev, and a node
// with more than cap_ev peer events in k parts (part j of peer g: its events
// [c*j/k, c*(j+1)/k) of that node, so a part holds at most
// P/k + world - 1 <= cap_ev events).  (cronsun_amd/shard.py restates it;
// cg_comm_gather_plan exposes this one.)
struct Chunk {
  int64_t n0, n1, j, k;
};
std::vector<Chunk> gather_plan(const int64_t* cnt, int world, int64_t N, int root, int64_t cap_ev) {
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
  int rc = rccl_ready();
  if (rc) return rc;
  static_assert(sizeof(ncclUniqueId) == CG_COMM_ID_BYTES, "unique id size");
  ncclUniqueId u;
  NCCLCHK(rccl().GetUniqueId(&u), "ncclGetUniqueId");
  std::memcpy(id, &u, CG_COMM_ID_BYTES);
  return CG_OK;
}

int cg_comm_init(cg_ctx* c, int world, int rank, const uint8_t id[CG_COMM_ID_BYTES], cg_comm** out) {
  if (!c || !id || !out || world < 1 || rank < 0 || rank >= world) return cg_fail(CG_EINVAL, "cg_comm_init: bad argument");
  int rc = rccl_ready();
  if (rc) return rc;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, CG_COMM_ID_BYTES);
  ncclComm_t nc = nullptr;
  NCCLCHK(rccl().CommInitRank(&nc, world, u, rank), "ncclCommInitRank");
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
  int rc = comm_usable(m);
  if (rc) return rc;
  cg_ctx* c = m->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  if (n == 0) return CG_OK;
  return allgather_locked(m, mine, n, all);
}

int cg_comm_node_offsets(cg_comm* m, int64_t* node_start, int64_t* node_base) {
  if (!m) return cg_fail(CG_EINVAL, "cg_comm_node_offsets: null");
  int rc = comm_usable(m);
  if (rc) return rc;
  cg_ctx* c = m->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  // every rank's node count and whether it has a readable result
  const bool ok = c->pn_valid && !pn_async_pending(c);
  const int64_t mine[2] = {c->pn_N, ok ? 1 : 0};
  std::vector<int64_t> meta(size_t(2 * m->world));
  if ((rc = allgather_locked(m, mine, 2, meta.data()))) return rc;
  for (int q = 0; q < m->world; q++) {
    if (!meta[size_t(2 * q + 1)])
      return cg_fail(CG_EINVAL, "cg_comm_node_offsets: rank " + std::to_string(q) +
                                    " has no readable per-node result (none yet, a failed call, or pipelined "
                                    "windows pending)");
    if (meta[size_t(2 * q)] != c->pn_N) return cg_fail(CG_EINVAL, "cg_comm_node_offsets: ranks differ in node count");
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

int cg_comm_gather_plan(const int64_t* counts, int32_t world, int32_t n_nodes, int32_t root, int64_t budget_bytes,
                        int64_t* chunks, int64_t cap, int64_t* n_chunks) {
  if (!counts || world < 1 || n_nodes < 0 || root < 0 || root >= world || (cap > 0 && !chunks) || !n_chunks)
    return cg_fail(CG_EINVAL, "cg_comm_gather_plan: bad argument");
  const int64_t cap_ev = budget_bytes / 12;
  if (world > 1 && cap_ev < 2 * int64_t(world)) return cg_fail(CG_EINVAL, "cg_comm_gather_plan: budget below 24 bytes per rank");
  const std::vector<Chunk> plan = gather_plan(counts, world, n_nodes, root, cap_ev);
  *n_chunks = int64_t(plan.size());
  if (int64_t(plan.size()) > cap)
    return cg_fail(CG_ECAPACITY, "cg_comm_gather_plan: " + std::to_string(plan.size()) + " chunks");
  for (size_t i = 0; i < plan.size(); i++) {
    chunks[4 * i] = plan[i].n0;
    chunks[4 * i + 1] = plan[i].n1;
    chunks[4 * i + 2] = plan[i].j;
    chunks[4 * i + 3] = plan[i].k;
  }
  return CG_OK;
}

int cg_comm_gather_node_csr(cg_comm* m, int root, int64_t rule_base, int64_t budget_bytes, int64_t* d_node_off,
                            int64_t* d_time, int32_t* d_rule, int64_t cap, int64_t* n_events) {
  constexpr int kMeta = 7;  // node count, events, ok, rule_base, cap, budget, time-ordered
  if (!m || root < 0 || root >= m->world) return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: bad argument");
  int rc = comm_usable(m);
  if (rc) return rc;
  cg_ctx* c = m->ctx;
  const int W = m->world, me = m->rank;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  // Agreement 1: every rank's preconditions travel with one all-gather, so
  // every rank returns the same status instead of leaving its peers blocked
  // in a transfer
  const bool local_ok = c->pn_valid && !pn_async_pending(c) && rule_base >= 0 && rule_base <= INT32_MAX &&
                        (me != root || ((d_node_off && d_time && d_rule) || c->pn_N == 0)) && budget_bytes > 0;
  const int64_t mine[kMeta] = {c->pn_N, c->pn_E, local_ok ? 1 : 0, rule_base, cap, budget_bytes,
                               c->pn_time_ordered ? 1 : 0};
  std::vector<int64_t> meta(size_t(kMeta * W));
  if ((rc = allgather_locked(m, mine, kMeta, meta.data()))) return rc;
  const int64_t N = c->pn_N;
  int64_t total = 0;
  for (int q = 0; q < W; q++) {
    const int64_t* mq = &meta[size_t(kMeta * q)];
    if (!mq[2])
      return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: rank " + std::to_string(q) +
                                    " has no gatherable result (none yet, a failed call, pending windows, a bad "
                                    "rule_base or budget, or null output buffers on root)");
    if (mq[0] != N) return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: ranks differ in node count");
    if (mq[6] != meta[6])
      return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: ranks differ in list order (some results time-ordered)");
    total += mq[1];
  }
  const bool timed = meta[6] != 0;
  if (timed && W > kMergeMaxRanks)  // refused here, on every rank, before any transfer
    return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: time-ordered results of more than " +
                                  std::to_string(kMergeMaxRanks) + " ranks");
  if (timed) {
    // the merge breaks (time) ties by rank: that is (time, global rule) order
    // only when the ranks' job-ID ranges ascend with the rank
    int64_t prev = -1;
    for (int q = 0; q < W; q++) {
      const int64_t* mq = &meta[size_t(kMeta * q)];
      if (mq[1] == 0) continue;  // no events: no ties to order
      if (mq[3] <= prev)
        return cg_fail(CG_EINVAL, "cg_comm_gather_node_csr: rule_base of rank " + std::to_string(q) +
                                      " does not ascend with the rank (time-ordered results merge by rank)");
      prev = mq[3];
    }
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
  if ((rc = node_counts_locked(m, N, cnt))) return rc;  // a collective: every rank reaches it
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
  const std::vector<Chunk> plan = gather_plan(cnt.data(), W, N, root, cap_ev);
  // peer q's piece of a chunk: its events [lo, hi) of its own CSR
  auto piece = [&](const Chunk& ch, int q, int64_t* lo, int64_t* hi) {
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
  hipStream_t s = c->st;
  // Root prepares everything before the transfers: staging (also the merge's
  // scratch), node offsets, slice destinations, its own slice.  Agreement 2
  // carries every rank's status of that step, so no rank starts a transfer
  // its peers will not join.
  int prep = CG_OK;
  std::string prep_msg;
  if (me == root) {
    int64_t stage = 1;
    for (const Chunk& ch : plan) {
      int64_t ev = 0;
      for (int q = 0; q < W; q++) {
        if (q == root) continue;
        int64_t lo, hi;
        piece(ch, q, &lo, &hi);
        ev += hi - lo;
      }
      stage = std::max(stage, ev);
    }
    if (timed && W > 1) {  // the merge's scratch: at least the largest node
      for (int64_t n = 0; n < N; n++) stage = std::max(stage, base[size_t(n + 1)] - base[size_t(n)]);
      stage = std::max(stage, std::min(cap_ev, total));
      prep = c->mr_rb.ensure(size_t(N) * (W + 1));
      if (!prep) prep = c->mr_tp.ensure(size_t(N) * W + 1);
    }
    if (!prep && N > 0) prep = m->off_all.ensure(size_t(W * (N + 1)));
    if (!prep && N > 0) prep = m->starts.ensure(size_t(W * N));
    if (!prep && (!plan.empty() || (timed && W > 1))) prep = m->stage_t.ensure(size_t(stage));
    if (!prep && (!plan.empty() || (timed && W > 1))) prep = m->stage_r.ensure(size_t(stage));
    if (!prep && N > 0) {
      prep = cg_hip_check(hipMemcpyAsync(m->off_all.p, off.data(), off.size() * 8, hipMemcpyHostToDevice, s), "copy");
      if (!prep)
        prep = cg_hip_check(hipMemcpyAsync(m->starts.p, st.data(), st.size() * 8, hipMemcpyHostToDevice, s), "copy");
      if (!prep)
        prep = cg_hip_check(hipMemcpyAsync(d_node_off, base.data(), base.size() * 8, hipMemcpyHostToDevice, s), "copy");
      // root's own slice, straight from its result
      if (!prep)
        prep = launch_node_place(c, s, int32_t(N), c->node_off.p, 0, c->node_time.p, c->node_rule.p,
                                 int32_t(rule_base), m->starts.p + int64_t(root) * N, d_time, d_rule);
    }
    if (prep) prep_msg = cg_last_error();
  }
  {
    const int64_t mine2[1] = {prep};
    std::vector<int64_t> st2(static_cast<size_t>(W));
    if ((rc = allgather_locked(m, mine2, 1, st2.data()))) return rc;
    for (int q = 0; q < W; q++)
      if (st2[size_t(q)] != CG_OK)
        return q == me ? cg_fail(int(st2[size_t(q)]), prep_msg)
                       : cg_fail(int(st2[size_t(q)]), "cg_comm_gather_node_csr: root (rank " + std::to_string(q) +
                                                          ") could not prepare the gather");
  }
  // The transfers.  From here on no rank returns before it has issued every
  // send / receive of the plan: a failure only stops root's placements (and
  // aborts the communicator when RCCL itself failed).
  int post = CG_OK;
  for (const Chunk& ch : plan) {
    int rc2 = nccl_check(rccl().GroupStart(), "ncclGroupStart");
    if (me == root) {
      int64_t o = 0;
      for (int q = 0; q < W && !rc2; q++) {
        if (q == root) continue;
        int64_t lo, hi;
        piece(ch, q, &lo, &hi);
        if (hi > lo) {
          rc2 = nccl_check(rccl().Recv(m->stage_t.p + o, size_t(hi - lo), ncclInt64, q, m->nc, s), "ncclRecv");
          if (!rc2) rc2 = nccl_check(rccl().Recv(m->stage_r.p + o, size_t(hi - lo), ncclInt32, q, m->nc, s), "ncclRecv");
        }
        o += hi - lo;
      }
    } else if (!rc2) {
      int64_t lo, hi;
      piece(ch, me, &lo, &hi);
      if (hi > lo) {
        rc2 = nccl_check(rccl().Send(c->node_time.p + lo, size_t(hi - lo), ncclInt64, root, m->nc, s), "ncclSend");
        if (!rc2) rc2 = nccl_check(rccl().Send(c->node_rule.p + lo, size_t(hi - lo), ncclInt32, root, m->nc, s), "ncclSend");
      }
    }
    const int rc3 = nccl_check(rccl().GroupEnd(), "ncclGroupEnd");  // always closes the group
    if (rc2 || rc3) {
      post = rc2 ? rc2 : rc3;
      abort_comm(m);
      break;
    }
    if (me != root || post) continue;
    // place the chunk (same stream: after the receives, before the next chunk's)
    int64_t o = 0;
    for (int q = 0; q < W && !post; q++) {
      if (q == root) continue;
      int64_t lo, hi;
      piece(ch, q, &lo, &hi);
      const int32_t add = int32_t(meta[size_t(kMeta * q + 3)]);
      if (hi > lo) {
        if (ch.k == 1)  // peer positions [lo, hi) staged at stage[o ..]
          post = launch_node_place(c, s, int32_t(ch.n1 - ch.n0), m->off_all.p + int64_t(q) * (N + 1) + ch.n0, lo - o,
                                   m->stage_t.p, m->stage_r.p, add, m->starts.p + int64_t(q) * N + ch.n0, d_time,
                                   d_rule);
        else {
          const int64_t dst = st[size_t(q * N + ch.n0)] + (lo - off[size_t(q * (N + 1) + ch.n0)]);
          post = launch_span_place(c, s, hi - lo, m->stage_t.p + o, m->stage_r.p + o, add, d_time + dst, d_rule + dst);
        }
      }
      o += hi - lo;
    }
  }
  if (post) {
    (void)hipStreamSynchronize(s);
    return post;
  }
  if (me == root && timed && W > 1 && N > 0) {
    // every node's slices are in (time, rule) order: merge them in place
    std::vector<int64_t> rb(size_t(N) * (W + 1));
    for (int64_t n = 0; n < N; n++) {
      for (int q = 0; q < W; q++) rb[size_t(n * (W + 1) + q)] = st[size_t(q * N + n)];
      rb[size_t(n * (W + 1) + W)] = base[size_t(n + 1)];
    }
    return merge_ranks_locked(c, s, int32_t(N), W, rb.data(), d_time, d_rule, int64_t(m->stage_t.cap), m->stage_t,
                              m->stage_r);
  }
  return cg_hip_check(hipStreamSynchronize(s), "gather sync");
}

}  // extern "C"
