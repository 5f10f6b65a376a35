// cg_dispatch.cpp -- GPU-resident cron dispatcher: the state of Cron.run
// (node/cron/cron.go:210-275) kept in HBM.
//
// The reference keeps []*Entry, re-sorts it by Next on every wake
// (sort.Sort(byTime), cron.go:220) and calls Schedule.Next for each entry that
// fired.  Here every entry is a slot (its Entry ID maps to a slot index on the
// host side) with three HBM arrays: the packed spec (32 B), Next and Prev
// (int64 unix seconds).  A wake is a streaming scan (due bitmap + the minimum
// over the entries that stay), an ordered compaction of the due slots, and a
// dense pass that advances the due entries with Next(now) and folds them into
// the minimum.  No sort: the run loop only ever needs the minimum and the
// entries equal to it.
#include <algorithm>
#include <cstring>
#include <vector>

#include "cg_api_internal.h"

using namespace cg;

namespace {

constexpr int64_t kDay = 86400;
// Next(now) walks back at most a month and forward at most five years
constexpr int64_t kBack = 64 * kDay;
constexpr int64_t kAhead = (6 * 366 + 64) * kDay;
constexpr int64_t kTableSpan = 16 * 366 * kDay;

// reallocate to `cap` elements keeping the first `used`
template <class T>
int grow_keep(T** p, size_t used, size_t cap, hipStream_t st) {
  T* q = nullptr;
  hipError_t e = hipMalloc(&q, cap * sizeof(T));
  if (e != hipSuccess) return cg_hip_check(e, "hipMalloc(dispatcher)");
  if (*p && used) {
    e = hipMemcpyAsync(q, *p, used * sizeof(T), hipMemcpyDeviceToDevice, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) {
      (void)hipFree(q);
      return cg_hip_check(e, "hipMemcpy(dispatcher grow)");
    }
  }
  if (*p) (void)hipFree(*p);
  *p = q;
  return CG_OK;
}

}  // namespace

struct cg_dispatcher {
  cg_ctx* ctx = nullptr;
  ZoneRules zone;
  // slots
  int64_t n = 0;
  size_t cap = 0;  // slots allocated
  DSpec* specs = nullptr;
  int64_t* next = nullptr;
  int64_t* prev = nullptr;
  std::vector<uint8_t> live;
  // wake scratch
  unsigned long long* due_bits = nullptr;
  uint32_t* tile_cnt = nullptr;
  unsigned long long* tile_min = nullptr;
  int32_t* due = nullptr;
  DispatchState* st = nullptr;
  int64_t n_due = 0;
  // the min over Next, host copy (CG_ZERO_TIME = no entry can fire)
  int64_t effective = CG_ZERO_TIME;
  // zone table covering [tab_lo, tab_hi], own buffer (the ctx plan buffer is shared)
  DBuf<char> tab_dev;
  PlanArgs pa{};
  int64_t tab_lo = 1, tab_hi = 0;
  // staging for set/remove
  DBuf<int64_t> idx_dev;
  DBuf<DSpec> src_dev;

  void release() {
    for (void* p : {(void*)specs, (void*)next, (void*)prev, (void*)due_bits, (void*)tile_cnt,
                    (void*)tile_min, (void*)due, (void*)st})
      if (p) (void)hipFree(p);
    specs = nullptr;
    next = prev = nullptr;
    due_bits = nullptr;
    tile_cnt = nullptr;
    tile_min = nullptr;
    due = nullptr;
    st = nullptr;
    tab_dev.release();
    idx_dev.release();
    src_dev.release();
  }

  // the zone table for Next walks from `now`
  int ensure_table(int64_t now) {
    if (now - kBack >= tab_lo && now + kAhead <= tab_hi) return CG_OK;
    if (now < -(int64_t(1) << 45) || now > (int64_t(1) << 45))
      return cg_fail(CG_ERANGE, "time outside +-1.1M years");
    ZoneTable t = build_table(zone, now - kBack, now + kTableSpan);
    const int32_t zn = int32_t(t.when.size());
    const size_t o_off = size_t(zn) * 8, bytes = o_off + size_t(zn) * 4 + 16;
    std::vector<char> h(bytes, 0);
    std::memcpy(h.data(), t.when.data(), size_t(zn) * 8);
    std::memcpy(h.data() + o_off, t.off.data(), size_t(zn) * 4);
    int rc = tab_dev.ensure(bytes);
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(tab_dev.p, h.data(), bytes, hipMemcpyHostToDevice, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    pa = PlanArgs{};
    pa.zwhen = reinterpret_cast<const int64_t*>(tab_dev.p);
    pa.zoff = reinterpret_cast<const int32_t*>(tab_dev.p + o_off);
    pa.zn = zn;
    if (plan_lds_bytes(pa) > 60 * 1024) return cg_fail(CG_ERANGE, "zone table too large for LDS");
    tab_lo = now - kBack;
    tab_hi = now + kTableSpan;
    return CG_OK;
  }

  // every per-slot array sized together, contents of [0, n) kept
  int reserve(int64_t want) {
    const size_t w = size_t(want);
    if (w <= cap) return CG_OK;
    const size_t nc = std::max(w, cap * 2);
    const size_t tiles = (nc + kDispatchTile - 1) / kDispatchTile;
    int rc;
    if ((rc = grow_keep(&specs, size_t(n), nc, ctx->st)) ||
        (rc = grow_keep(&next, size_t(n), nc, ctx->st)) ||
        (rc = grow_keep(&prev, size_t(n), nc, ctx->st)) ||
        (rc = grow_keep(&due_bits, 0, tiles * (kDispatchTile / 64), ctx->st)) ||
        (rc = grow_keep(&tile_cnt, 0, tiles, ctx->st)) ||
        (rc = grow_keep(&tile_min, 0, tiles, ctx->st)) || (rc = grow_keep(&due, 0, nc, ctx->st)))
      return rc;
    if (!st) HIPCHK(hipMalloc(&st, sizeof(DispatchState)));
    cap = nc;
    live.resize(nc, 0);
    return CG_OK;
  }

  int reset_state() {
    HIPCHK(hipMemsetAsync(st, 0xFF, sizeof(DispatchState), ctx->st));
    HIPCHK(hipMemsetAsync(&st->n_due, 0, sizeof(unsigned long long), ctx->st));
    return CG_OK;
  }

  // read the state back; CG_ERANGE if some entry's Next never returns
  int read_state(DispatchState* h) {
    HIPCHK(hipMemcpyAsync(h, st, sizeof *h, hipMemcpyDeviceToHost, ctx->st));
    HIPCHK(hipStreamSynchronize(ctx->st));
    effective = h->min_key == ~0ull ? CG_ZERO_TIME : int64_t(h->min_key ^ (uint64_t(1) << 63));
    if (h->stuck != ~0ull)
      return cg_fail(CG_ERANGE, "entry " + std::to_string(h->stuck) +
                                    ": Schedule.Next never returns for it (the reference run "
                                    "loop blocks forever); its Next is left unset");
    return CG_OK;
  }

  int recompute_min() {
    int rc = reset_state();
    if (rc) return rc;
    launch_dispatch_min(next, n, st, ctx->st);
    HIPCHK(hipGetLastError());
    DispatchState h;
    return read_state(&h);
  }
};

extern "C" {

int cg_dispatcher_new(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t now,
                      cg_dispatcher** out) {
  if (!c || !s || !z || !out) return cg_fail(CG_EINVAL, "cg_dispatcher_new: null");
  if (s->n > size_t(INT32_MAX)) return cg_fail(CG_ERANGE, "more than 2^31-1 entries");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  cg_dispatcher* d = new cg_dispatcher();
  d->ctx = c;
  d->zone = z->rules;
  int rc = d->reserve(std::max<int64_t>(int64_t(s->n), 1024));
  if (!rc) rc = d->ensure_table(now);
  if (rc) {
    d->release();
    delete d;
    return rc;
  }
  d->n = int64_t(s->n);
  if (d->n) {
    HIPCHK(hipMemcpyAsync(d->specs, s->d, s->n * sizeof(DSpec), hipMemcpyDeviceToDevice, c->st));
    std::fill(d->live.begin(), d->live.begin() + d->n, 1);
  }
  *out = d;
  // run(): entry.Next = entry.Schedule.Next(now) for every entry (cron.go:212-215)
  if ((rc = d->reset_state())) return rc;
  launch_dispatch_place(d->specs, nullptr, nullptr, 0, d->n, d->pa, now, d->next, d->prev, d->st,
                        c->st);
  launch_dispatch_min(d->next, d->n, d->st, c->st);
  HIPCHK(hipGetLastError());
  DispatchState h;
  return d->read_state(&h);
}

void cg_dispatcher_free(cg_dispatcher* d) {
  if (!d) return;
  {
    std::lock_guard<std::mutex> g(d->ctx->mu);
    (void)hipSetDevice(d->ctx->device);
    (void)hipStreamSynchronize(d->ctx->st);
    d->release();
  }
  delete d;
}

int64_t cg_dispatcher_count(const cg_dispatcher* d) { return d ? d->n : 0; }

int cg_dispatcher_effective(const cg_dispatcher* d, int64_t* effective) {
  if (!d || !effective) return cg_fail(CG_EINVAL, "cg_dispatcher_effective: null");
  *effective = d->effective;
  return CG_OK;
}

int cg_dispatcher_fire(cg_dispatcher* d, int64_t now, int64_t* n_due, int64_t* effective) {
  if (!d || !n_due || !effective) return cg_fail(CG_EINVAL, "cg_dispatcher_fire: null");
  cg_ctx* c = d->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  d->n_due = 0;
  *n_due = 0;
  *effective = d->effective;
  if (d->effective == CG_ZERO_TIME) return CG_OK;  // nothing can fire: the loop just sleeps
  if (now < d->effective)
    return cg_fail(CG_EINVAL, "cg_dispatcher_fire: now is before the effective time "
                              "(the run loop's timer fires at or after it)");
  int rc = d->ensure_table(now);
  if (rc) return rc;
  // (k_dispatch_compact writes the whole DispatchState: no reset)
  (void)hipEventRecord(c->pev[0], c->st);
  launch_dispatch_scan(d->next, d->n, d->effective, d->due_bits, d->tile_cnt, d->tile_min, c->st);
  (void)hipEventRecord(c->pev[1], c->st);
  launch_dispatch_compact(d->due_bits, d->tile_cnt, d->tile_min, d->n, d->due, d->st, c->st);
  (void)hipEventRecord(c->pev[2], c->st);
  launch_dispatch_advance(d->specs, d->due, d->n, d->pa, now, d->next, d->prev, d->st, c->st);
  (void)hipEventRecord(c->pev[3], c->st);
  HIPCHK(hipGetLastError());
  DispatchState h;
  rc = d->read_state(&h);
  (void)hipEventElapsedTime(&c->kt[9], c->pev[0], c->pev[1]);
  (void)hipEventElapsedTime(&c->kt[10], c->pev[1], c->pev[2]);
  (void)hipEventElapsedTime(&c->kt[11], c->pev[2], c->pev[3]);
  d->n_due = int64_t(h.n_due);
  *n_due = d->n_due;
  *effective = d->effective;
  return rc;
}

int cg_dispatcher_due(const cg_dispatcher* d, int64_t first, int64_t count, int32_t* out) {
  if (!d || (count && !out)) return cg_fail(CG_EINVAL, "cg_dispatcher_due: null");
  if (first < 0 || count < 0 || first + count > d->n_due)
    return cg_fail(CG_ERANGE, "cg_dispatcher_due: range outside the last wake's due list");
  if (!count) return CG_OK;
  cg_ctx* c = d->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipMemcpyAsync(out, d->due + first, size_t(count) * 4, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return CG_OK;
}

int cg_dispatcher_due_device(const cg_dispatcher* d, const int32_t** due, int64_t* n_due) {
  if (!d || !due || !n_due) return cg_fail(CG_EINVAL, "cg_dispatcher_due_device: null");
  *due = d->due;
  *n_due = d->n_due;
  return CG_OK;
}

int cg_dispatcher_set(cg_dispatcher* d, const int64_t* idx, const cg_schedule* s, size_t k,
                      int64_t now) {
  if (!d || (k && (!idx || !s))) return cg_fail(CG_EINVAL, "cg_dispatcher_set: null");
  if (!k) return CG_OK;
  std::vector<DSpec> h(k);
  int64_t top = d->n;
  {
    std::vector<int64_t> sorted(idx, idx + k);
    std::sort(sorted.begin(), sorted.end());
    if (sorted[0] < 0) return cg_fail(CG_EINVAL, "cg_dispatcher_set: negative slot");
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      return cg_fail(CG_EINVAL, "cg_dispatcher_set: a slot appears twice");
    top = std::max(top, sorted.back() + 1);
  }
  if (top > INT32_MAX) return cg_fail(CG_ERANGE, "more than 2^31-1 entries");
  for (size_t j = 0; j < k; j++) {
    int rc = pack_spec(s[j], &h[j]);
    if (rc) return rc;
  }
  cg_ctx* c = d->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = d->ensure_table(now);
  if (!rc && top > d->n) rc = d->reserve(top);
  if (!rc) rc = d->idx_dev.ensure(k);
  if (!rc) rc = d->src_dev.ensure(k);
  if (rc) return rc;
  if (top > d->n) {  // new slots start empty (Next = Prev = zero)
    launch_dispatch_clear(nullptr, d->n, top - d->n, d->next, d->prev, c->st);
    d->n = top;
  }
  HIPCHK(hipMemcpyAsync(d->idx_dev.p, idx, k * 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipMemcpyAsync(d->src_dev.p, h.data(), k * sizeof(DSpec), hipMemcpyHostToDevice, c->st));
  if ((rc = d->reset_state())) return rc;
  // newEntry.Next = newEntry.Schedule.Next(time.Now()) (cron.go:246-252)
  launch_dispatch_place(d->specs, d->idx_dev.p, d->src_dev.p, 0, int64_t(k), d->pa, now, d->next,
                        d->prev, d->st, c->st);
  launch_dispatch_min(d->next, d->n, d->st, c->st);
  HIPCHK(hipGetLastError());
  for (size_t j = 0; j < k; j++) d->live[size_t(idx[j])] = 1;
  DispatchState hs;
  return d->read_state(&hs);
}

int cg_dispatcher_remove(cg_dispatcher* d, const int64_t* idx, size_t k) {
  if (!d || (k && !idx)) return cg_fail(CG_EINVAL, "cg_dispatcher_remove: null");
  for (size_t j = 0; j < k; j++)
    if (idx[j] < 0 || idx[j] >= d->n) return cg_fail(CG_EINVAL, "cg_dispatcher_remove: bad slot");
  if (!k) return CG_OK;
  cg_ctx* c = d->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = d->idx_dev.ensure(k);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(d->idx_dev.p, idx, k * 8, hipMemcpyHostToDevice, c->st));
  launch_dispatch_clear(d->idx_dev.p, 0, int64_t(k), d->next, d->prev, c->st);
  for (size_t j = 0; j < k; j++) d->live[size_t(idx[j])] = 0;
  return d->recompute_min();
}

int cg_dispatcher_snapshot(const cg_dispatcher* d, int64_t* next, int64_t* prev, uint8_t* live) {
  if (!d) return cg_fail(CG_EINVAL, "cg_dispatcher_snapshot: null");
  cg_ctx* c = d->ctx;
  std::lock_guard<std::mutex> g(c->mu);
  HIPCHK(hipSetDevice(c->device));
  if (d->n && next)
    HIPCHK(hipMemcpyAsync(next, d->next, size_t(d->n) * 8, hipMemcpyDeviceToHost, c->st));
  if (d->n && prev)
    HIPCHK(hipMemcpyAsync(prev, d->prev, size_t(d->n) * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  if (live) std::copy(d->live.begin(), d->live.begin() + d->n, live);
  return CG_OK;
}

}  // extern "C"
