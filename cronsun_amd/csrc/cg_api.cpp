// cg_api.cpp -- the C-ABI of include/cronsun_gpu.h: contexts, device memory,
// zones, spec upload, Next batches and the expansion pipeline.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"
#include "cg_kernels.h"
#include "cg_parse.h"
#include "cg_zone.h"

using namespace cg;

namespace {
thread_local std::string g_err;
}

int cg_fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int cg_hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return CG_OK;
  return cg_fail(e == hipErrorOutOfMemory ? CG_ENOMEM : CG_EHIP,
                 std::string(what) + ": " + hipGetErrorString(e));
}



static uint64_t next_serial() {
  static std::mutex m;
  static uint64_t s = 0;
  std::lock_guard<std::mutex> g(m);
  return ++s;
}

extern "C" {

int cg_abi_version(void) { return CG_ABI_VERSION; }

const char* cg_last_error(void) { return g_err.c_str(); }

int cg_build_info(void) {
#ifdef CG_DIAG
  return CG_BUILD_DIAG;
#else
  return 0;
#endif
}

int cg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int ok = 0;
  for (int i = 0; i < n; i++) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ok++;
  }
  return ok;
}

// ------------------------------------------------------------------ zones
int cg_zone_from_tzif(const uint8_t* data, size_t len, cg_zone** out) {
  if (!data || !out) return cg_fail(CG_EINVAL, "cg_zone_from_tzif: null");
  ZoneRules r;
  std::string e;
  if (!zone_from_tzif(data, len, &r, &e)) return cg_fail(CG_EINVAL, "TZif: " + e);
  *out = new cg_zone{std::move(r), next_serial()};
  return CG_OK;
}

int cg_zone_fixed(int32_t off, cg_zone** out) {
  if (!out) return cg_fail(CG_EINVAL, "cg_zone_fixed: null");
  *out = new cg_zone{zone_fixed(off), next_serial()};
  return CG_OK;
}

int cg_zone_utc(cg_zone** out) {
  if (!out) return cg_fail(CG_EINVAL, "cg_zone_utc: null");
  *out = new cg_zone{zone_utc(), next_serial()};
  return CG_OK;
}

void cg_zone_free(cg_zone* z) { delete z; }

int cg_zone_offset(const cg_zone* z, int64_t t, int32_t* off) {
  if (!z || !off) return cg_fail(CG_EINVAL, "cg_zone_offset: null");
  *off = z->rules.offset(t);
  return CG_OK;
}

int cg_zone_table(const cg_zone* z, int64_t lo, int64_t hi, int64_t* when, int32_t* off, int cap) {
  if (!z) return cg_fail(CG_EINVAL, "cg_zone_table: null");
  ZoneTable t = build_table(z->rules, lo, hi);
  int n = int(t.when.size());
  for (int i = 0; i < n && i < cap; i++) {
    if (when) when[i] = t.when[i];
    if (off) off[i] = t.off[i];
  }
  return n;
}

// ---------------------------------------------------------------- context
int cg_init(int device, cg_ctx** out) {
  if (!out) return cg_fail(CG_EINVAL, "cg_init: null");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return cg_fail(CG_ENODEV, "no HIP device visible (this engine has no CPU fallback)");
  if (device < 0 || device >= n) return cg_fail(CG_ENODEV, "device index out of range");
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return cg_fail(CG_ENODEV, std::string("device is ") + prop.gcnArchName + ", need gfx950");
  HIPCHK(hipSetDevice(device));
  cg_ctx* c = new cg_ctx();
  c->device = device;
  int per_cu = kWriteBlocksPerCU;
#ifdef CG_DIAG
  if (const char* e = getenv("CG_WRITE_BLOCKS_PER_CU")) per_cu = std::max(1, atoi(e));
#endif
  c->write_blocks = std::max(1, prop.multiProcessorCount) * per_cu;
  if (hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return cg_fail(CG_EHIP, "hipStreamCreate failed");
  }
  // timing-only events (read after a stream sync): no system-scope fence
  // when they complete -- a fenced event between two kernels idles the GPU
  // for several us (cache writeback + invalidate)
  for (auto& e : c->ev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  for (auto& e : c->pev) (void)hipEventCreateWithFlags(&e, hipEventDisableSystemFence);
  *out = c;
  return CG_OK;
}

void cg_destroy(cg_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->st);
  if (c->st_cs) (void)hipStreamSynchronize(c->st_cs);
  c->free_all();
  for (auto& e : c->ev) (void)hipEventDestroy(e);
  for (auto& e : c->pev) (void)hipEventDestroy(e);
  (void)hipStreamDestroy(c->st);
  delete c;
}

int cg_sync(cg_ctx* c) {
  if (!c) return cg_fail(CG_EINVAL, "cg_sync: null");
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->st));
  return CG_OK;
}

// ------------------------------------------------------------------ specs
}  // extern "C"

int pack_spec(const cg_schedule& s, DSpec* d) {
  std::memset(d, 0, sizeof *d);
  if (s.kind == 1) {
    if (s.delay_ns <= 0 || s.delay_ns % 1000000000LL != 0)
      return cg_fail(CG_EINVAL,
                     "ConstantDelaySchedule.Delay must be a positive whole number of seconds "
                     "(cron.Every guarantees this)");
    d->kind = KIND_EVERY;
    d->sec = uint64_t(s.delay_ns / 1000000000LL);
    return CG_OK;
  }
  if (s.kind != 0) return cg_fail(CG_EINVAL, "unknown schedule kind");
  d->kind = KIND_SPEC;
  d->sec = s.second & 0x0FFFFFFFFFFFFFFFull;
  d->min = s.minute & 0x0FFFFFFFFFFFFFFFull;
  d->hour = uint32_t(s.hour & 0xFFFFFFu);
  d->dom = uint32_t(s.dom & 0xFFFFFFFEu) | uint32_t((s.dom >> 63) & 1u);
  d->mondow = uint32_t(s.month & 0x1FFEu) | (uint32_t(s.dow & 0x7Fu) << 16) |
              (uint32_t((s.dow >> 63) & 1u) << 23);
  return CG_OK;
}

extern "C" {

static int upload_packed(cg_ctx* c, const std::vector<DSpec>& h, cg_specs** out) {
  HIPCHK(hipSetDevice(c->device));
  cg_specs* s = new cg_specs();
  s->ctx = c;
  s->n = h.size();
  s->owner = true;
  if (!h.empty()) {
    hipError_t e = hipMalloc(&s->d, h.size() * sizeof(DSpec));
    if (e != hipSuccess) {
      delete s;
      return cg_hip_check(e, "hipMalloc(specs)");
    }
    e = hipMemcpy(s->d, h.data(), h.size() * sizeof(DSpec), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
      (void)hipFree(s->d);
      delete s;
      return cg_hip_check(e, "hipMemcpy(specs)");
    }
  }
  *out = s;
  return CG_OK;
}

int cg_specs_upload(cg_ctx* c, const cg_spec_soa* soa, size_t n, cg_specs** out) {
  if (!c || !soa || !out) return cg_fail(CG_EINVAL, "cg_specs_upload: null");
  std::vector<DSpec> h(n);
  for (size_t i = 0; i < n; i++) {
    cg_schedule s;
    std::memset(&s, 0, sizeof s);
    if (soa->delay_ns && soa->delay_ns[i] > 0) {
      s.kind = 1;
      s.delay_ns = soa->delay_ns[i];
    } else {
      s.second = soa->second ? soa->second[i] : 0;
      s.minute = soa->minute ? soa->minute[i] : 0;
      s.hour = soa->hour ? soa->hour[i] : 0;
      s.dom = soa->dom ? soa->dom[i] : 0;
      s.month = soa->month ? soa->month[i] : 0;
      s.dow = soa->dow ? soa->dow[i] : 0;
    }
    int rc = pack_spec(s, &h[i]);
    if (rc) return rc;
  }
  return upload_packed(c, h, out);
}

int cg_specs_upload_schedules(cg_ctx* c, const cg_schedule* s, size_t n, cg_specs** out) {
  if (!c || (!s && n) || !out) return cg_fail(CG_EINVAL, "cg_specs_upload_schedules: null");
  std::vector<DSpec> h(n);
  for (size_t i = 0; i < n; i++) {
    int rc = pack_spec(s[i], &h[i]);
    if (rc) return rc;
  }
  return upload_packed(c, h, out);
}

int cg_specs_slice(cg_specs* p, size_t first, size_t count, cg_specs** out) {
  if (!p || !out) return cg_fail(CG_EINVAL, "cg_specs_slice: null");
  if (first > p->n || count > p->n - first) return cg_fail(CG_EINVAL, "slice out of range");
  cg_specs* s = new cg_specs();
  s->ctx = p->ctx;
  s->d = p->d + first;
  s->n = count;
  s->owner = false;
  *out = s;
  return CG_OK;
}

size_t cg_specs_count(const cg_specs* s) { return s ? s->n : 0; }

void cg_specs_free(cg_specs* s) {
  if (!s) return;
  if (s->owner && s->d) {
    (void)hipSetDevice(s->ctx->device);
    (void)hipFree(s->d);
  }
  delete s;
}

}  // extern "C"

// ----------------------------------------------------------- plan upload
// one packed upload: when | off | segs | dtab
PlanLayout plan_layout(const Plan& plan) {
  PlanLayout L;
  const size_t zn = plan.table.when.size(), G = plan.segs.size(), nd = plan.dtab.size();
  L.o_when = 0;
  L.o_off = L.o_when + zn * 8;
  L.o_seg = (L.o_off + zn * 4 + 15) / 16 * 16;
  L.o_dt = L.o_seg + G * sizeof(Segment);
  L.bytes = L.o_dt + nd * 4 + 16;
  return L;
}

void plan_pack(const Plan& plan, const PlanLayout& L, char* h) {
  std::memset(h, 0, L.bytes);
  std::memcpy(h + L.o_when, plan.table.when.data(), plan.table.when.size() * 8);
  std::memcpy(h + L.o_off, plan.table.off.data(), plan.table.off.size() * 4);
  if (!plan.segs.empty()) std::memcpy(h + L.o_seg, plan.segs.data(), plan.segs.size() * sizeof(Segment));
  if (!plan.dtab.empty()) std::memcpy(h + L.o_dt, plan.dtab.data(), plan.dtab.size() * 4);
}

int plan_args(const Plan& plan, const PlanLayout& L, char* base, int64_t t0, int64_t t1, PlanArgs* pa) {
  const int32_t G = int32_t(plan.segs.size());
  if (G > kMaxSegments)
    return cg_fail(CG_ERANGE, "plan has more than " + std::to_string(kMaxSegments) +
                                  " segments (horizon too long for this zone)");
  pa->zwhen = reinterpret_cast<const int64_t*>(base + L.o_when);
  pa->zoff = reinterpret_cast<const int32_t*>(base + L.o_off);
  pa->segs = reinterpret_cast<const Segment*>(base + L.o_seg);
  pa->dtab = reinterpret_cast<const uint32_t*>(base + L.o_dt);
  pa->zn = int32_t(plan.table.when.size());
  pa->G = G;
  pa->nd = int32_t(plan.dtab.size());
  pa->dtab_global = 0;
  pa->flags = plan.flags;
  pa->t0 = t0;
  pa->t1 = t1;
  // long horizons: the day table (4 B per local day) stays in HBM and the
  // zone table + segments alone are staged
  if (plan_lds_bytes(*pa) > kPlanLdsBytes) pa->dtab_global = 1;
  if (plan_lds_bytes(*pa) > kPlanLdsBytes)
    return cg_fail(CG_ERANGE, "zone table too large for LDS staging (narrow the time range)");
  return CG_OK;
}

int upload_plan(cg_ctx* c, const Plan& plan, int64_t t0, int64_t t1, PlanArgs* pa) {
  if (plan.segs.size() > size_t(kMaxSegments))
    return cg_fail(CG_ERANGE, "plan has more than " + std::to_string(kMaxSegments) +
                                  " segments (horizon too long for this zone)");
  // plan_dev is shared by every entry point: whatever it held is gone, so the
  // expansion's plan cache must not be trusted after this (expand re-validates)
  c->plan_valid = false;
  const PlanLayout L = plan_layout(plan);
  std::vector<char>& h = c->plan_host;
  h.assign(L.bytes, 0);
  plan_pack(plan, L, h.data());
  int rc = c->plan_dev.ensure(L.bytes);
  if (rc) return rc;
  HIPCHK(hipMemcpyAsync(c->plan_dev.p, h.data(), L.bytes, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipStreamSynchronize(c->st));  // h is reused by the next call
  return plan_args(plan, L, c->plan_dev.p, t0, t1, pa);
}

extern "C" {

// ------------------------------------------------------------------ Next()
int cg_next_batch(cg_ctx* c, const cg_specs* s, const cg_zone* z, const int64_t* t_in,
                  int64_t* t_out) {
  if (!c || !s || !z || (s->n && (!t_in || !t_out))) return cg_fail(CG_EINVAL, "cg_next_batch: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  HIPCHK(hipSetDevice(c->device));
  const int64_t n = int64_t(s->n);
  if (n == 0) return CG_OK;
  int64_t lo = t_in[0], hi = t_in[0];
  for (int64_t i = 1; i < n; i++) {
    lo = std::min(lo, t_in[i]);
    hi = std::max(hi, t_in[i]);
  }
  const int64_t kDay = 86400;
  if (lo < -(int64_t(1) << 45) || hi > (int64_t(1) << 45))
    return cg_fail(CG_ERANGE, "input time outside +-1.1M years");
  Plan plan;
  // Next walks back to the month start of t+1 and forward at most ~6 years
  plan.table = build_table(z->rules, lo - 64 * kDay, hi + (6 * 366 + 64) * kDay);
  PlanArgs pa;
  int rc = upload_plan(c, plan, 0, 0, &pa);
  if (rc) return rc;
  if ((rc = c->nb_in.ensure(n))) return rc;
  if ((rc = c->nb_out.ensure(n))) return rc;
  HIPCHK(hipMemcpyAsync(c->nb_in.p, t_in, n * 8, hipMemcpyHostToDevice, c->st));
  launch_next_batch(s->d, n, pa, c->nb_in.p, c->nb_out.p, c->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(t_out, c->nb_out.p, n * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return CG_OK;
}

// ---------------------------------------------------------- Cmd.lockTtl()
int cg_lock_ttl_batch(cg_ctx* c, const cg_specs* s, const cg_zone* z, const int64_t* now,
                      const int32_t* kind, const int64_t* avg_time_ms, int64_t lock_ttl,
                      int64_t* ttl_out) {
  if (!c || !s || !z || (s->n && (!now || !kind || !avg_time_ms || !ttl_out)))
    return cg_fail(CG_EINVAL, "cg_lock_ttl_batch: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  const int64_t n = int64_t(s->n);
  if (n == 0) return CG_OK;
  int64_t lo = now[0], hi = now[0];
  for (int64_t i = 1; i < n; i++) {
    lo = std::min(lo, now[i]);
    hi = std::max(hi, now[i]);
  }
  if (lo < -(int64_t(1) << 45) || hi > (int64_t(1) << 45))
    return cg_fail(CG_ERANGE, "input time outside +-1.1M years");
  const int64_t kDay = 86400;
  // prev may be the zero time (no fire within five years), and Next(prev) then
  // walks from year 1; otherwise the two walks end within ~12 years of now.
  Plan plan;
  plan.table = build_table(z->rules, std::min(lo, int64_t(CG_ZERO_TIME)) - 64 * kDay,
                           hi + (12 * 366 + 64) * kDay);
  PlanArgs pa;
  int rc = upload_plan(c, plan, 0, 0, &pa);
  if (rc) return rc;
  if ((rc = c->nb_in.ensure(n)) || (rc = c->nb_out.ensure(n)) || (rc = c->lt_avg.ensure(n)) ||
      (rc = c->lt_kind.ensure(n)))
    return rc;
  HIPCHK(hipMemcpyAsync(c->nb_in.p, now, n * 8, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipMemcpyAsync(c->lt_kind.p, kind, n * 4, hipMemcpyHostToDevice, c->st));
  HIPCHK(hipMemcpyAsync(c->lt_avg.p, avg_time_ms, n * 8, hipMemcpyHostToDevice, c->st));
  launch_lock_ttl(s->d, n, pa, c->nb_in.p, c->lt_kind.p, c->lt_avg.p, lock_ttl, c->nb_out.p, c->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(ttl_out, c->nb_out.p, n * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return CG_OK;
}

}  // extern "C"

// --------------------------------------------------------------- expansion
// plan (cached) + k_count + scan of the run counts: c->run_off holds the run
// offsets afterwards.  *empty = true when there is nothing to count.
// map_cap > 0: the scan also builds k_write_cf's slice map in c->block_run
// for an output capacity of map_cap events (no k_chunk_map launch).
static int count_phase(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                       bool* empty, int64_t map_cap = 0) {
  // no readable result until this call succeeds (the accessors check last_R/E).
  // Asynchronous calls still pending are drained and their results and errors
  // discarded: this call's result replaces them (cronsun_gpu.h).
  int rc0 = async_drain(c);
  if (rc0) return rc0;
  c->async_rc = 0;
  c->async_msg.clear();
  if ((rc0 = pn_async_drain(c))) return rc0;  // the same for pipelined per-node windows
  c->pa_rc = 0;
  c->pa_msg.clear();
  c->pa_last = -1;
  c->pa_en_sum = 0;
  c->as_last = -1;
  c->last_R = 0;
  c->last_E = 0;
  HIPCHK(hipSetDevice(c->device));
  if (t1 - t0 > CG_MAX_HORIZON || t0 < -(int64_t(1) << 45) || t1 > (int64_t(1) << 45))
    return cg_fail(CG_ERANGE, "horizon must satisfy t1 - t0 <= CG_MAX_HORIZON (40 years)");
  const int64_t R = int64_t(s->n);
  int rc;
  // plan (cached across identical calls)
  if (!(c->plan_valid && c->plan_zone == z->serial && c->plan_t0 == t0 && c->plan_t1 == t1)) {
    c->plan = build_plan(z->rules, t0, t1);
    if ((rc = upload_plan(c, c->plan, t0, t1, &c->pa))) {
      c->plan_valid = false;
      return rc;
    }
    c->plan_valid = true;
    c->plan_zone = z->serial;
    c->plan_t0 = t0;
    c->plan_t1 = t1;
  }
  const PlanArgs& pa = c->pa;
  const int64_t G = pa.G;
  c->last_G = G;
  for (int i = 0; i < 6; i++) c->kt[i] = 0;
  if ((rc = c->offsets.ensure(R + 1))) return rc;
  if (R == 0 || G == 0) {
    HIPCHK(hipMemsetAsync(c->offsets.p, 0, (R + 1) * 8, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    *empty = true;
    return CG_OK;
  }
  const int64_t nruns = R * G;
  if ((rc = c->run_anchor.ensure(nruns))) return rc;
  if ((rc = c->run_count.ensure(nruns))) return rc;
  if ((rc = c->run_dmask.ensure(nruns))) return rc;
  if ((rc = c->run_off.ensure(nruns + 1))) return rc;
  if ((rc = c->scan_tmp.ensure(scan_temp_bytes(nruns)))) return rc;

  if ((rc = c->stuck.ensure(1))) return rc;
  if (!c->res_host) {
    // mapped, coherent pinned memory: the scan kernel stores the 16-B record
    // straight into it (no D2H copy launch); read after the stream sync
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->res_host), 16,
                         hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->res_dev), c->res_host, 0));
  }
  if (!c->stuck_armed) HIPCHK(hipMemsetAsync(c->stuck.p, 0xFF, sizeof(unsigned long long), c->st));
  c->stuck_armed = false;  // until this call's scan re-arms it
  const bool all_phases = c->phase_timing >= 2;
  if (all_phases) (void)hipEventRecord(c->ev[0], c->st);
  launch_count(s->d, R, pa, c->run_anchor.p, c->run_count.p, c->run_dmask.p, c->stuck.p, c->st);
  if (all_phases) (void)hipEventRecord(c->ev[1], c->st);
  if (map_cap > 0 && (rc = c->block_run.ensure(slice_map_words(map_cap)))) return rc;
  launch_scan_runs(c->run_count.p, c->run_off.p, R, int32_t(G), c->scan_tmp.p, c->offsets.p, c->res_dev,
                   c->stuck.p, map_cap > 0 ? c->block_run.p : nullptr, map_cap, c->st);
  if (all_phases) (void)hipEventRecord(c->ev[2], c->st);
  HIPCHK(hipGetLastError());
  *empty = false;
  return CG_OK;
}

static int stuck_error(unsigned long long stuck) {
  return cg_fail(CG_ERANGE, "rule " + std::to_string(stuck) +
                                ": the reference Next loop never terminates inside this horizon "
                                "(Next does not return, or returns a time <= its input and cycles)");
}

int expand_device_locked(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                         int64_t* n_events) {
  bool empty = true;
  // steady state: the output buffer exists, so the scan builds the writer's
  // slice map for its capacity (a first or a growing call maps separately)
  const int64_t cap0 = int64_t(c->times.cap);
  int rc = count_phase(c, s, z, t0, t1, &empty, cap0);
  if (rc) return rc;
  const int64_t R = int64_t(s->n);
  if (empty) {
    c->last_R = R;  // offsets are all zero
    c->last_E = 0;
    *n_events = 0;
    return CG_OK;
  }
  const PlanArgs& pa = c->pa;
  const int64_t G = pa.G;
  const int64_t nruns = R * G;
  // Write phase without a host round trip: the chunk map and writers read the
  // event total from device memory and size their work from it.  Output
  // capacity comes from earlier calls; the first call (or a larger result)
  // syncs once to size the buffers and relaunches the write phase.
  if (c->times.cap == 0) {
    int64_t E0 = 0;
    HIPCHK(hipMemcpyAsync(&E0, c->run_off.p + nruns, 8, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if ((rc = c->times.ensure(std::max<int64_t>(E0, 1)))) return rc;
  }
  // walked runs: WALK windows, or CF segments whose entry fire does not fully
  // match (only possible when the plan has zone transitions)
  const bool all_phases = c->phase_timing >= 2;
  // (a CF run is entered by the exact walk only after a WALK segment, or from
  // T0 when a transition lies in the 40 days before it)
  const bool has_walk = (c->plan.flags & (kPlanT0Walk | kPlanWalkSegs)) != 0;
  int64_t E = 0;
  unsigned long long stuck = 0;
  for (int attempt = 0; attempt < 2; attempt++) {
    const int64_t cap = int64_t(c->times.cap);
    if ((rc = c->block_run.ensure(slice_map_words(cap)))) return rc;
    if (all_phases) (void)hipEventRecord(c->ev[3], c->st);
    if (!(cap0 > 0 && cap == cap0))
      launch_chunk_map(c->run_off.p, nruns, cap, c->block_run.p, c->st);
    (void)hipEventRecord(c->ev[4], c->st);
    launch_write_cf(s->d, pa, c->run_anchor.p, c->run_count.p, c->run_dmask.p, c->run_off.p, nruns,
                    c->block_run.p, cap, c->times.p, c->write_blocks, c->st);
    (void)hipEventRecord(c->ev[5], c->st);
    if (has_walk)
      launch_write_walk(s->d, R, pa, c->run_anchor.p, c->run_count.p, c->run_dmask.p,
                        c->run_off.p, cap, c->times.p, c->st);
    if (all_phases) (void)hipEventRecord(c->ev[6], c->st);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->st));
    c->stuck_armed = true;
    E = c->res_host[0];
    stuck = static_cast<unsigned long long>(c->res_host[1]);
    if (stuck != ~0ULL) return stuck_error(stuck);
    if (E <= cap) break;
    if ((rc = c->times.ensure(E))) return rc;  // grow and redo the write phase
  }
  (void)hipEventElapsedTime(&c->kt[3], c->ev[4], c->ev[5]);
  if (all_phases) {
    (void)hipEventElapsedTime(&c->kt[0], c->ev[0], c->ev[1]);
    (void)hipEventElapsedTime(&c->kt[1], c->ev[1], c->ev[2]);
    (void)hipEventElapsedTime(&c->kt[2], c->ev[3], c->ev[4]);
    (void)hipEventElapsedTime(&c->kt[4], c->ev[5], c->ev[6]);
    c->kt[5] = 0.f;  // per-rule offsets: written by the scan (k_scan_apply)
  } else {
    c->kt[0] = c->kt[1] = c->kt[2] = c->kt[4] = c->kt[5] = -1.f;
  }
  c->last_R = R;
  c->last_E = E;
  *n_events = E;
  return CG_OK;
}

extern "C" int cg_count(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                        int64_t* counts, int64_t* total) {
  if (!c || !s || !z || !total || (s->n && !counts)) return cg_fail(CG_EINVAL, "cg_count: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  bool empty = true;
  int rc = count_phase(c, s, z, t0, t1, &empty);
  if (rc) return rc;
  const int64_t R = int64_t(s->n);
  if (empty) {
    for (int64_t r = 0; r < R; r++) counts[r] = 0;
    *total = 0;
    return CG_OK;
  }
  HIPCHK(hipGetLastError());
  std::vector<int64_t> off(size_t(R) + 1);
  HIPCHK(hipMemcpyAsync(off.data(), c->offsets.p, (R + 1) * 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  c->stuck_armed = true;
  const unsigned long long stuck = static_cast<unsigned long long>(c->res_host[1]);
  if (stuck != ~0ULL) return stuck_error(stuck);
  for (int64_t r = 0; r < R; r++) counts[r] = off[size_t(r) + 1] - off[size_t(r)];
  *total = off[size_t(R)];
  return CG_OK;  // (no expansion result to read after a count: last_R = last_E = 0)
}

extern "C" {

int cg_expand_device(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                     int64_t* n_events) {
  if (!c || !s || !z || !n_events) return cg_fail(CG_EINVAL, "cg_expand_device: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  return expand_device_locked(c, s, z, t0, t1, n_events);
}

int cg_expand(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
              cg_csr* out) {
  if (!c || !s || !z || !out) return cg_fail(CG_EINVAL, "cg_expand: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  int64_t E = 0;
  int rc = expand_device_locked(c, s, z, t0, t1, &E);
  if (rc) return rc;
  out->n_events = E;
  if (out->offsets)
    HIPCHK(hipMemcpy(out->offsets, c->offsets.p, (s->n + 1) * 8, hipMemcpyDeviceToHost));
  if (out->times) {
    if (out->times_cap < E) return cg_fail(CG_ECAPACITY, "times buffer too small; see n_events");
    if (E) HIPCHK(hipMemcpy(out->times, c->times.p, E * 8, hipMemcpyDeviceToHost));
  }
  return CG_OK;
}

static int refuse_pending(cg_ctx* c, const char* what) {
  if (!async_pending(c)) return CG_OK;
  return cg_fail(CG_EINVAL, std::string(what) + ": asynchronous expansions pending (call cg_expand_wait first)");
}

int cg_result_device(cg_ctx* c, const int64_t** d_off, const int64_t** d_times, int64_t* n) {
  if (!c) return cg_fail(CG_EINVAL, "cg_result_device: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (int rc = refuse_pending(c, "cg_result_device")) return rc;
  if (d_off) *d_off = c->as_last >= 0 ? c->as[c->as_last].offsets.p : c->offsets.p;
  if (d_times) *d_times = c->times.p;
  if (n) *n = c->last_E;
  return CG_OK;
}

int cg_result_copy_times(cg_ctx* c, int64_t first, int64_t count, int64_t* host) {
  if (!c || (count && !host)) return cg_fail(CG_EINVAL, "cg_result_copy_times: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (int rc = refuse_pending(c, "cg_result_copy_times")) return rc;
  if (first < 0 || count < 0 || first + count > c->last_E)
    return cg_fail(CG_EINVAL, "range outside the last result");
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  HIPCHK(hipSetDevice(c->device));
  if (count) HIPCHK(hipMemcpy(host, c->times.p + first, count * 8, hipMemcpyDeviceToHost));
  return CG_OK;
}

int cg_result_copy_offsets(cg_ctx* c, int64_t* host) {
  if (!c || !host) return cg_fail(CG_EINVAL, "cg_result_copy_offsets: null");
  std::lock_guard<std::mutex> g(c->mu);
  if (int rc = refuse_pending(c, "cg_result_copy_offsets")) return rc;
  (void)hipGetLastError();  // clear a stale error so launch checks see only their own
  HIPCHK(hipSetDevice(c->device));
  const int64_t* off = c->as_last >= 0 ? c->as[c->as_last].offsets.p : c->offsets.p;
  HIPCHK(hipMemcpy(host, off, (c->last_R + 1) * 8, hipMemcpyDeviceToHost));
  return CG_OK;
}

int cg_checksum_device(cg_ctx* c, const void* d_ptr, int64_t n, int elem_bytes, int64_t first_index,
                       int64_t add, uint64_t* out) {
  if (!c || !out || (n > 0 && !d_ptr) || n < 0 || (elem_bytes != 8 && elem_bytes != 4))
    return cg_fail(CG_EINVAL, "cg_checksum_device: bad argument");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = c->cksum.ensure(1);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(c->cksum.p, 0, 8, c->st));
  launch_checksum(d_ptr, n, elem_bytes, first_index, add, c->cksum.p, c->st);
  HIPCHK(hipGetLastError());
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, c->cksum.p, 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  *out = v;
  return CG_OK;
}

int cg_fill_device(cg_ctx* c, void* d_ptr, int64_t bytes, int byte_value) {
  if (!c || bytes < 0 || (bytes > 0 && !d_ptr)) return cg_fail(CG_EINVAL, "cg_fill_device: bad argument");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  if (bytes) HIPCHK(hipMemsetAsync(d_ptr, byte_value & 0xFF, size_t(bytes), c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  return CG_OK;
}

int cg_fill_rate_device(cg_ctx* c, void* d_ptr, int64_t bytes, int reps, float* ms) {
  if (!c || !ms || bytes <= 0 || bytes % 16 != 0 || !d_ptr || reps < 1)
    return cg_fail(CG_EINVAL, "cg_fill_rate_device: bad argument (bytes a positive multiple of 16, reps >= 1)");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipStreamSynchronize(c->st));
  for (int kind = 0; kind < 3; kind++) {
    auto fill = [&]() -> hipError_t {
      if (kind == 2) return hipMemsetAsync(d_ptr, 0x5E, size_t(bytes), c->st);
      launch_fill_stream(d_ptr, bytes / 16, kind == 0, c->st);
      return hipGetLastError();
    };
    HIPCHK(fill());  // warm-up
    HIPCHK(hipEventRecord(c->ev[0], c->st));
    for (int r = 0; r < reps; r++) HIPCHK(fill());
    HIPCHK(hipEventRecord(c->ev[1], c->st));
    HIPCHK(hipEventSynchronize(c->ev[1]));
    float t = 0.f;
    HIPCHK(hipEventElapsedTime(&t, c->ev[0], c->ev[1]));
    ms[kind] = t / float(reps);
  }
  return CG_OK;
}

int cg_count_value_device(cg_ctx* c, const void* d_ptr, int64_t n, int elem_bytes, int64_t value,
                          int64_t* count) {
  if (!c || !count || (n > 0 && !d_ptr) || n < 0 || (elem_bytes != 8 && elem_bytes != 4))
    return cg_fail(CG_EINVAL, "cg_count_value_device: bad argument");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = c->cksum.ensure(1);
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(c->cksum.p, 0, 8, c->st));
  launch_count_eq(d_ptr, n, elem_bytes, value, c->cksum.p, c->st);
  HIPCHK(hipGetLastError());
  unsigned long long v = 0;
  HIPCHK(hipMemcpyAsync(&v, c->cksum.p, 8, hipMemcpyDeviceToHost, c->st));
  HIPCHK(hipStreamSynchronize(c->st));
  *count = int64_t(v);
  return CG_OK;
}

int cg_set_phase_timing(cg_ctx* c, int level) {
  if (!c || level < 1 || level > 2) return cg_fail(CG_EINVAL, "cg_set_phase_timing: level 1 or 2");
  std::lock_guard<std::mutex> g(c->mu);
  c->phase_timing = level;
  return CG_OK;
}

int cg_set_node_order(cg_ctx* c, int order) {
  if (!c || (order != CG_NODE_ORDER_RULE && order != CG_NODE_ORDER_TIME))
    return cg_fail(CG_EINVAL, "cg_set_node_order: CG_NODE_ORDER_RULE or CG_NODE_ORDER_TIME");
  std::lock_guard<std::mutex> g(c->mu);
  c->node_order = order;
  return CG_OK;
}

int cg_last_kernel_times(cg_ctx* c, float* ms, int n) {
  if (!c || !ms) return cg_fail(CG_EINVAL, "cg_last_kernel_times: null");
  int k = std::min(n, int(sizeof(c->kt) / sizeof(c->kt[0])));
  for (int i = 0; i < k; i++) ms[i] = c->kt[i];
  return k;
}

}  // extern "C"
