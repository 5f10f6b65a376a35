// cg_async.cpp -- pipelined expansion for back-to-back calls (a scheduler's
// tick loop, SURVEY.md §8 a11: cron.go:212-215,242-243 batched per tick).
//
// A synchronous cg_expand_device ends every call with a stream sync (the
// caller reads the event total) and runs count -> scan -> write in series.
// cg_expand_device_async enqueues the same kernels and returns: the count and
// scan of call k run on a second stream, into a run set no queued writer
// reads (three sets), while call k-1's writer streams its output; call k's writer then
// follows call k-1's on the ctx stream.  The plan of each call (zone table,
// segments, day table) is staged through pinned memory of its run set, so a
// moving T0 costs no stream sync either.  cg_expand_wait drains the pipeline
// and reports the calls' errors: a rule whose reference Next loop never ends
// (CG_ERANGE), or a result larger than the output capacity sized by an
// earlier synchronous call (CG_ECAPACITY: the writer then wrote nothing).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "../../include/cronsun_gpu.h"
#include "cg_api_internal.h"
#include "cg_kernels.h"
#include "cg_zone.h"

using namespace cg;

#ifndef CG_ASYNC_ONE_EVENT
#define CG_ASYNC_ONE_EVENT 1
#endif
#ifndef CG_ASYNC_NO_TIMING
#define CG_ASYNC_NO_TIMING 0  // diagnostic: no writer timing events (kernel_ms then meaningless)
#endif

namespace {

// the record of a finished call on set a: fold its errors and writer time in
void check_set(cg_ctx* c, AsyncSet& a) {
  if (!a.pending) return;
  a.pending = false;
  float ms = 0.f;
  if (!CG_ASYNC_NO_TIMING && hipEventElapsedTime(&ms, a.w0, a.w1) == hipSuccess) {
    c->wr_ms_sum += ms;
    c->wr_n++;
  }
  const int64_t E = a.res_host[0];
  const unsigned long long stuck = static_cast<unsigned long long>(a.res_host[1]);
  if (c->async_rc) return;  // keep the first error
  if (stuck != ~0ULL) {
    c->async_rc = CG_ERANGE;
    c->async_msg = "rule " + std::to_string(stuck) +
                   ": the reference Next loop never terminates inside this horizon "
                   "(Next does not return, or returns a time <= its input and cycles)";
  } else if (E > a.cap) {
    c->async_rc = CG_ECAPACITY;
    c->async_msg = "async expansion: " + std::to_string(E) + " events exceed the output capacity " +
                   std::to_string(a.cap) + " (run a synchronous cg_expand_device to grow it)";
  }
}

}  // namespace

int ensure_async(cg_ctx* c) {
  if (c->st_cs) return CG_OK;
  HIPCHK(hipStreamCreateWithFlags(&c->st_cs, hipStreamNonBlocking));
  for (hipEvent_t& e : c->cs_done) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (AsyncSet& a : c->as) {
    HIPCHK(hipEventCreateWithFlags(&a.written, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&a.w0, hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&a.w1, hipEventDisableSystemFence));
    HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&a.res_host), 16, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.res_dev), a.res_host, 0));
    a.res_host[0] = 0;
    a.res_host[1] = -1;
  }
  return CG_OK;
}

bool async_pending(const cg_ctx* c) {
  for (const AsyncSet& a : c->as)
    if (a.pending) return true;
  return false;
}

// every pending async call finished and checked (errors kept for the next wait)
int async_drain(cg_ctx* c) {
  bool any = false;
  for (const AsyncSet& a : c->as) any = any || a.pending;
  if (!any) return CG_OK;
  HIPCHK(hipStreamSynchronize(c->st));
  for (AsyncSet& a : c->as) check_set(c, a);
  return CG_OK;
}

// Stages call (t0, t1]'s plan into run set a (pinned memory, no stream sync)
// and enqueues its count and scan on the ctx's second stream, building the
// writer's slice map for an output capacity of cap events.  *empty: R or G
// is 0 (nothing enqueued).
int async_count_scan(cg_ctx* c, AsyncSet& a, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                     int64_t cap, bool* empty) {
  int rc;
  const int64_t R = int64_t(s->n);
  if (!(a.plan_valid && a.plan_zone == z->serial && a.plan_t0 == t0 && a.plan_t1 == t1)) {
    a.plan_valid = false;
    a.plan = build_plan(z->rules, t0, t1);
    const PlanLayout L = plan_layout(a.plan);
    if (a.plan_pin_cap < L.bytes) {
      if (a.plan_pin) (void)hipHostFree(a.plan_pin);
      a.plan_pin = nullptr;
      a.plan_pin_cap = 0;
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&a.plan_pin), L.bytes));
      a.plan_pin_cap = L.bytes;
    }
    plan_pack(a.plan, L, a.plan_pin);
    if ((rc = a.plan_dev.ensure(L.bytes))) return rc;
    if ((rc = plan_args(a.plan, L, a.plan_dev.p, t0, t1, &a.pa))) return rc;
    HIPCHK(hipMemcpyAsync(a.plan_dev.p, a.plan_pin, L.bytes, hipMemcpyHostToDevice, c->st_cs));
    a.plan_valid = true;
    a.plan_zone = z->serial;
    a.plan_t0 = t0;
    a.plan_t1 = t1;
  }
  const PlanArgs& pa = a.pa;
  const int64_t G = pa.G;
  if ((rc = a.offsets.ensure(R + 1))) return rc;
  if (R == 0 || G == 0) {
    *empty = true;
    return CG_OK;
  }
  const int64_t nruns = R * G;
  if ((rc = a.run_anchor.ensure(nruns)) || (rc = a.run_count.ensure(nruns)) || (rc = a.run_dmask.ensure(nruns)) ||
      (rc = a.run_off.ensure(nruns + 1)) || (rc = a.scan_tmp.ensure(scan_temp_bytes(nruns))) ||
      (rc = a.block_run.ensure(slice_map_words(cap))) || (rc = a.stuck.ensure(1)))
    return rc;
  // count + scan on the second stream (the scan re-arms the stuck flag and
  // builds the writer's slice map for the output capacity)
  if (!a.armed) HIPCHK(hipMemsetAsync(a.stuck.p, 0xFF, sizeof(unsigned long long), c->st_cs));
  a.armed = true;  // from here on every scan re-arms it
  launch_count(s->d, R, pa, a.run_anchor.p, a.run_count.p, a.run_dmask.p, a.stuck.p, c->st_cs);
  launch_scan_runs(a.run_count.p, a.run_off.p, R, int32_t(G), a.scan_tmp.p, a.offsets.p, a.res_dev, a.stuck.p,
                   a.block_run.p, cap, c->st_cs);
  a.R = R;
  a.cap = cap;
  *empty = false;
  return CG_OK;
}

extern "C" {

int cg_expand_device_async(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1) {
  if (!c || !s || !z) return cg_fail(CG_EINVAL, "cg_expand_device_async: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  if (t1 - t0 > CG_MAX_HORIZON || t0 < -(int64_t(1) << 45) || t1 > (int64_t(1) << 45))
    return cg_fail(CG_ERANGE, "horizon must satisfy t1 - t0 <= CG_MAX_HORIZON (40 years)");
  const int64_t cap = int64_t(c->times.cap);
  if (cap == 0)
    return cg_fail(CG_ECAPACITY, "cg_expand_device_async: no output capacity yet (run cg_expand_device once)");
  int rc = ensure_async(c);
  if (rc) return rc;
  const int k = c->as_next;
  AsyncSet& a = c->as[k];
  // the set was last used kAsyncSets calls ago: its writer must be done
  // before the host restages its plan or the count stream rewrites its runs
  HIPCHK(hipEventSynchronize(a.written_w1 ? a.w1 : a.written));
  check_set(c, a);
  const int64_t R = int64_t(s->n);
  bool empty = false;
  if ((rc = async_count_scan(c, a, s, z, t0, t1, cap, &empty))) return rc;
  if (empty) {  // nothing to count: zero offsets, an empty result
    HIPCHK(hipMemsetAsync(a.offsets.p, 0, (R + 1) * 8, c->st));
    a.res_host[0] = 0;
    a.res_host[1] = -1;
    a.R = R;
    c->as_next = (k + 1) % cg_ctx::kAsyncSets;
    c->as_last = k;
    c->last_R = R;
    c->last_E = 0;
    return CG_OK;
  }
  const PlanArgs& pa = a.pa;
  const int64_t nruns = R * int64_t(pa.G);
  HIPCHK(hipEventRecord(c->cs_done[k], c->st_cs));
  // the writer after the previous call's writer, once this call's scan is done
  HIPCHK(hipStreamWaitEvent(c->st, c->cs_done[k], 0));
  const bool has_walk = (a.plan.flags & (kPlanT0Walk | kPlanWalkSegs)) != 0;
  if (!CG_ASYNC_NO_TIMING) (void)hipEventRecord(a.w0, c->st);
  launch_write_cf(s->d, pa, a.run_anchor.p, a.run_count.p, a.run_dmask.p, a.run_off.p, nruns, a.block_run.p, cap,
                  c->times.p, c->write_blocks, c->st);
  if (!CG_ASYNC_NO_TIMING) (void)hipEventRecord(a.w1, c->st);
  if (has_walk)
    launch_write_walk(s->d, R, pa, a.run_anchor.p, a.run_count.p, a.run_dmask.p, a.run_off.p, cap, c->times.p,
                      c->st);
  // the set is free again once its writer is done: without a walk that is w1
  // (one event packet fewer between back-to-back writers)
  a.written_w1 = CG_ASYNC_ONE_EVENT && !has_walk && !CG_ASYNC_NO_TIMING;
  if (!a.written_w1) HIPCHK(hipEventRecord(a.written, c->st));
  HIPCHK(hipGetLastError());
  a.R = R;
  a.cap = cap;
  a.pending = true;
  c->as_next = (k + 1) % cg_ctx::kAsyncSets;
  c->as_last = k;
  c->last_R = 0;  // nothing readable until cg_expand_wait (the accessors refuse while a call is pending)
  c->last_E = 0;
  return CG_OK;
}

int cg_expand_wait(cg_ctx* c, int64_t* n_events) {
  if (!c) return cg_fail(CG_EINVAL, "cg_expand_wait: null");
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipGetLastError();
  HIPCHK(hipSetDevice(c->device));
  int rc = async_drain(c);
  if (rc) return rc;
  if (c->wr_n > 0) {
    c->kt[3] = float(c->wr_ms_sum / c->wr_n);  // mean writer time of the calls checked
    for (int i : {0, 1, 2, 4, 5}) c->kt[i] = -1.f;
  }
  c->wr_ms_sum = 0;
  c->wr_n = 0;
  const int rc_async = c->async_rc;
  const std::string msg = c->async_msg;
  c->async_rc = 0;
  c->async_msg.clear();
  int64_t E = 0;
  if (c->as_last >= 0) {
    E = c->as[c->as_last].res_host[0];
    c->last_E = rc_async ? 0 : E;
    c->last_R = rc_async ? 0 : c->as[c->as_last].R;
  }
  if (n_events) *n_events = E;  // 0 when no asynchronous call was made since the last synchronous one
  if (rc_async) return cg_fail(rc_async, msg);
  return CG_OK;
}

}  // extern "C"
