// cg_api_internal.h -- context/specs objects behind the C-ABI handles.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>
#include <vector>

#include "../../include/cronsun_gpu.h"
#include "cg_kernels.h"
#include "cg_zone.h"

int cg_fail(int code, const std::string& msg);
int cg_hip_check(hipError_t e, const char* what);

#define HIPCHK(x)                    \
  do {                               \
    int _rc = cg_hip_check((x), #x); \
    if (_rc != CG_OK) return _rc;    \
  } while (0)

// Grow-only device buffer (grows by 1.25x so repeated calls settle).
// per-node writer record of one non-empty (node, rule) pair of a segment
// (cg_pernode.hip, k_seg_records): rule, first position in the segment, and
// x, st -- fire at position p = t0 + x + p * st (a progression rule), or
// band-relative fire-list index = x + p when st == 0
// per rule of a per-node window (k_rule_info): fire count, band-relative
// index of the first fire, and {first - t0, stride} of a progression (st 0:
// not one)
struct alignas(16) RuleInfo {
  int32_t cnt, off, first, st;
};

struct alignas(16) PairRec {
  int32_t rule, dst, x, st;
};

template <class T>
struct DBuf {
  T* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return CG_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    size_t want = std::max(n, cap + cap / 4);
    hipError_t e = hipMalloc(&p, want * sizeof(T));
    if (e != hipSuccess) {
      // retry at the exact size before giving up
      e = hipMalloc(&p, n * sizeof(T));
      if (e != hipSuccess) {
        p = nullptr;
        cap = 0;
        return cg_hip_check(e, "hipMalloc");
      }
      want = n;
    }
    cap = want;
    return CG_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

// An integer-interned rule set in device memory (cg_rules_in uploaded).
struct RulesStore {
  DBuf<int64_t> nid_off, gid_off, ex_off, group_off;
  DBuf<int32_t> nids, gids, ex, group_nodes, rule_job;
  // next_same[r]: the next rule of r's job with r's Cmd key (rule_key), or -1
  // (Job.Cmds keeps the last included rule per key, job.go:604-609); only
  // uploaded when some job repeats a key (has_dup); prev_same[r] the previous
  // one (k_rule_nodes sweeps each key's chain from its last rule back)
  DBuf<int32_t> next_same, prev_same;
  bool has_dup = false;
  DBuf<uint8_t> group_exists, job_pause;
  int32_t n_nodes = 0, n_groups = 0, n_rules = 0, n_jobs = 0;
  uint64_t serial = 0;  // unique per upload: keys the per-node transpose cache
  void release() {
    nid_off.release(); gid_off.release(); ex_off.release(); group_off.release();
    nids.release(); gids.release(); ex.release(); group_nodes.release(); rule_job.release();
    next_same.release(); prev_same.release();
    group_exists.release(); job_pause.release();
  }
};

// One run set of the pipelined expansion (cg_expand_device_async): what the
// count/scan of a call writes and its writer reads, so the count/scan of call
// k (on the ctx's second stream) can run while the writer of call k-1 does.
struct AsyncSet {
  DBuf<int64_t> run_anchor, run_off, offsets, block_run;
  DBuf<int32_t> run_count;
  DBuf<uint32_t> run_dmask;
  DBuf<char> scan_tmp, plan_dev;
  DBuf<unsigned long long> stuck;
  int64_t* res_host = nullptr;  // {E, stuck rule}: mapped pinned, written by the scan
  int64_t* res_dev = nullptr;
  char* plan_pin = nullptr;  // pinned staging of the plan upload
  size_t plan_pin_cap = 0;
  cg::Plan plan;
  cg::PlanArgs pa{};
  bool plan_valid = false;
  uint64_t plan_zone = 0;
  int64_t plan_t0 = 0, plan_t1 = 0;
  hipEvent_t written = nullptr, w0 = nullptr, w1 = nullptr;  // writer done; writer start/end
  bool written_w1 = false;  // the set's writer-done event is w1 (no walk kernel)
  bool pending = false;  // a call on this set whose record has not been checked
  bool armed = false;    // stuck flag holds ~0 (set once; every scan re-arms it)
  int64_t R = 0, cap = 0;
  void release() {
    run_anchor.release(); run_off.release(); offsets.release(); block_run.release();
    run_count.release(); run_dmask.release(); scan_tmp.release(); plan_dev.release(); stuck.release();
    if (res_host) (void)hipHostFree(res_host);
    if (plan_pin) (void)hipHostFree(plan_pin);
    res_host = res_dev = nullptr;
    plan_pin = nullptr;
    plan_pin_cap = 0;
    for (hipEvent_t* e : {&written, &w0, &w1})
      if (*e) (void)hipEventDestroy(*e), *e = nullptr;
  }
};

// One set of the pipelined per-node path (cg_expand_per_node_rules_device_async):
// the window's rule-major expansion (its own run set and fire times), rule
// infos and segment records, so window k+1's expansion and records are built
// on the second stream while window k's per-node writer streams on the first.
struct PnAsyncSet {
  AsyncSet rm;
  DBuf<int64_t> times, seg_cnt, seg_pos, node_off;
  DBuf<int32_t> seg_nrec;
  DBuf<RuleInfo> rule_info;
  DBuf<PairRec> recs;
  DBuf<uint32_t> tickets;
  DBuf<char> seg_tmp;
  int64_t* res_host = nullptr;  // {En, error}: mapped pinned, written by the records / node offsets
  int64_t* res_dev = nullptr;
  hipEvent_t side_done = nullptr, written = nullptr, nw0 = nullptr, nw1 = nullptr;
  bool pending = false;
  bool timed = false;  // the window's lists are written in (time, rule) order
  int64_t t0 = 0, t1 = 0, node_cap = 0, rm_cap = 0;
  int32_t N = 0;
  void release() {
    rm.release();
    times.release(); seg_cnt.release(); seg_pos.release(); node_off.release(); seg_nrec.release();
    rule_info.release(); recs.release(); tickets.release(); seg_tmp.release();
    if (res_host) (void)hipHostFree(res_host);
    res_host = res_dev = nullptr;
    for (hipEvent_t* e : {&side_done, &written, &nw0, &nw1})
      if (*e) (void)hipEventDestroy(*e), *e = nullptr;
  }
};

struct cg_ctx {
  int device = 0;
  int write_blocks = 1024;  // persistent k_write_cf grid (set from the CU count)
  hipStream_t st = nullptr;
  hipEvent_t ev[8] = {};
  hipEvent_t pev[4] = {};  // per-node phases
  std::mutex mu;
  // ms: [0..5] expansion phases (count, scan, map, write_cf, write_walk,
  // offsets), [6..8] per-node phases (rule->node join, transpose + per-node
  // offsets, k_node_write) of the last per-node call, [9..11] dispatcher
  // wake (scan, due compaction, advance) of the last cg_dispatcher_fire, [12]
  // the time-order pass of the last cg_node_result_order_by_time
  float kt[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  // expansion phase timing: 2 = an event between every phase (kt[0..5]);
  // 1 = events around k_write_cf only (kt[3]; the others read -1).  Each
  // event recorded between two kernels costs 6-12 us of idle GPU on this
  // stack, so throughput runs use 1 (cg_set_phase_timing).
  int phase_timing = 2;

  // plan cache
  cg::Plan plan;
  cg::PlanArgs pa{};
  bool plan_valid = false;
  uint64_t plan_zone = 0;
  int64_t plan_t0 = 0, plan_t1 = 0;
  std::vector<char> plan_host;
  DBuf<char> plan_dev;

  // expansion buffers
  DBuf<int64_t> run_anchor, run_off, offsets, times, block_run, nb_in, nb_out, lt_avg;
  DBuf<int32_t> run_count, lt_kind;
  DBuf<uint32_t> run_dmask;
  DBuf<char> scan_tmp;
  DBuf<unsigned long long> stuck;  // ~0 between calls (the expansion scan re-arms it)
  DBuf<unsigned long long> cksum;  // cg_checksum_device accumulator
  bool stuck_armed = false;        // false: memset it before the next k_count
  int64_t* res_host = nullptr;     // {E, stuck rule}: mapped pinned 16 B the scan writes
  int64_t* res_dev = nullptr;      // res_host's device address
  int64_t last_E = 0, last_R = 0, last_G = 0;

  // pipelined expansion (cg_async.cpp): two run sets used in turn, count +
  // scan on st_cs, writers on st; as_last = set of the last async result
  // (-1: the last result came from the synchronous path)
  // Three run sets: a call's count and scan are enqueued while the writer
  // two calls back is long done, so they sit ready in the hardware queue and
  // run in the previous writer's tail instead of racing the next writer's
  // start (two sets: the count alternately ran before and after that start,
  // 19 vs 50 us between writers, profiles/r02_ab_async_sets.json)
  static constexpr int kAsyncSets = 3;
  AsyncSet as[kAsyncSets];
  int as_next = 0, as_last = -1;
  hipStream_t st_cs = nullptr;
  hipEvent_t cs_done[kAsyncSets] = {};
  int async_rc = 0;  // first error of the calls since the last cg_expand_wait
  std::string async_msg;
  double wr_ms_sum = 0;  // writer (k_write_cf) time of the checked async calls
  int wr_n = 0;

  // pipelined per-node windows (cg_pernode.hip): three sets in turn
  static constexpr int kPnSets = 3;
  PnAsyncSet pns[kPnSets];
  int pa_next = 0, pa_last = -1;
  int pa_rc = 0;  // first error of the per-node calls since the last wait
  std::string pa_msg;
  double nw_ms_sum = 0;  // per-node writer time of the checked calls
  int nw_n = 0;
  int64_t pa_en_sum = 0;  // node events of the checked calls since the last wait

  // per-node buffers: the rule->node join (rule-major pairs), its node-major
  // transpose, the (node, rule band) segments and the node CSR
  DBuf<int64_t> rn_off, node_off, node_time, nt_off, rs_off, seg_pair, seg_cnt, seg_pos;
  DBuf<int32_t> rn_cnt, rn_nodes, pair_node, pair_rule, node_rule, nt_rule, rs_hist;
  DBuf<int32_t> seg_nrec;
  DBuf<PairRec> recs;  // per-call segment records (k_seg_records)
  DBuf<RuleInfo> rule_info;  // per-call, per rule (k_rule_info)
  DBuf<uint32_t> pn_tickets;
  // time-order pass (cg_node_order.hip): node-aligned tiles, per-pass
  // histograms/offsets, and the second buffers of the ping-pong
  DBuf<int32_t> ts_cnt, ts_tile_node, ts_hist, node_rule2;
  DBuf<int64_t> ts_base, ts_off, node_time2, ts_node_off;
  DBuf<int64_t> ts_start;  // per tile its first list position; [T] = the lists' end
  DBuf<int32_t> ts_hi;     // per tile the high rule bits (rule >> 20) all its events share
  int64_t pn_t0 = 0, pn_t1 = 0;  // window of the last per-node result
  RulesStore rules;  // rule set of the host-array entry points (re-uploaded per call)
  int64_t pn_E = 0, pn_nnz = 0, pn_N = 0;
  // a per-node result is readable (node_off [pn_N+1], pn_E events): cleared
  // when a per-node call starts or fails, set when one succeeds -- pn_N and
  // node_off may be stale otherwise (the gather / node offsets check it)
  bool pn_valid = false;
  int64_t pn_R = INT64_MAX;  // rule count of the per-node lists being ordered (the merge packs rules below 2^20)
  // time-ordered gather (merge_ranks_enqueue): per-node run bounds, the tile
  // prefix over runs, and a scratch copy of one node group
  DBuf<int64_t> mr_rb, mr_tp, mr_t;
  DBuf<int32_t> mr_r;
  int64_t* pn_res_host = nullptr;  // mapped pinned: per-node event total of the last call
  int64_t* pn_res_dev = nullptr;
  // the rule->node join + transpose depend only on (rule set, exclude mode):
  // kept across per-node calls on the same uploaded rule set (time windows);
  // the segment bounds also on the band width
  uint64_t pn_cache_serial = 0;
  int pn_cache_mode = -1;
  int node_order = CG_NODE_ORDER_RULE;  // cg_set_node_order
  bool pn_time_ordered = false;         // the last per-node result is in (time, rule) order
  int32_t pn_B = 0, pn_K = 0;  // rules per band, bands of the cached segment bounds (0: none)
  // the time-order merge's dense nodes run on their own stream beside the
  // sparse ones (fork / join events on st)
  hipStream_t st_ot = nullptr;
  hipEvent_t ot_fork = nullptr, ot_join = nullptr;

  void free_all() {
    for (AsyncSet& a : as) a.release();
    for (PnAsyncSet& a : pns) a.release();
    for (hipEvent_t& e : cs_done)
      if (e) (void)hipEventDestroy(e), e = nullptr;
    if (st_cs) (void)hipStreamDestroy(st_cs);
    st_cs = nullptr;
    if (ot_fork) (void)hipEventDestroy(ot_fork), ot_fork = nullptr;
    if (ot_join) (void)hipEventDestroy(ot_join), ot_join = nullptr;
    if (st_ot) (void)hipStreamDestroy(st_ot);
    st_ot = nullptr;
    plan_dev.release();
    run_anchor.release(); run_off.release(); offsets.release(); times.release();
    block_run.release(); nb_in.release(); nb_out.release(); run_count.release();
    lt_avg.release(); lt_kind.release();
    if (res_host) (void)hipHostFree(res_host);
    res_host = nullptr;
    res_dev = nullptr;
    run_dmask.release(); scan_tmp.release(); stuck.release(); cksum.release();
    rn_off.release(); node_off.release(); node_time.release(); nt_off.release(); rs_off.release();
    seg_pair.release(); seg_cnt.release(); seg_pos.release(); rn_cnt.release(); rn_nodes.release();
    pair_node.release(); pair_rule.release(); node_rule.release(); nt_rule.release();
    rs_hist.release(); pn_tickets.release(); rules.release();
    seg_nrec.release(); recs.release();
    rule_info.release();
    ts_cnt.release(); ts_tile_node.release(); ts_hist.release(); node_rule2.release();
    ts_start.release(); ts_hi.release();
    ts_base.release(); ts_off.release(); node_time2.release(); ts_node_off.release();
    mr_rb.release(); mr_tp.release(); mr_t.release(); mr_r.release();
    if (pn_res_host) (void)hipHostFree(pn_res_host);
    pn_res_host = nullptr;
    pn_res_dev = nullptr;
  }
};

struct cg_rules {
  cg_ctx* ctx = nullptr;
  RulesStore st;
};

struct cg_zone {
  cg::ZoneRules rules;
  uint64_t serial;
};

struct cg_specs {
  cg_ctx* ctx = nullptr;
  cg::DSpec* d = nullptr;
  size_t n = 0;
  bool owner = false;
};

// cg_schedule -> packed 32-byte device spec (validates @every delays)
int pack_spec(const cg_schedule& s, cg::DSpec* d);
int upload_plan(cg_ctx* c, const cg::Plan& plan, int64_t t0, int64_t t1, cg::PlanArgs* pa);
struct PlanLayout {
  size_t o_when, o_off, o_seg, o_dt, bytes;
};
PlanLayout plan_layout(const cg::Plan& plan);
void plan_pack(const cg::Plan& plan, const PlanLayout& L, char* dst);
int plan_args(const cg::Plan& plan, const PlanLayout& L, char* dev_base, int64_t t0, int64_t t1,
              cg::PlanArgs* pa);
int expand_device_locked(cg_ctx* c, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                         int64_t* n_events);
// finish and check every pending cg_expand_device_async call (cg_async.cpp);
// their errors are reported by the next cg_expand_wait
int async_drain(cg_ctx* c);
int ensure_async(cg_ctx* c);  // the second stream and the run sets' events / pinned records
// stage a call's plan into run set a and enqueue its count + scan on the second
// stream (cg_async.cpp); *empty when there is nothing to count
int async_count_scan(cg_ctx* c, AsyncSet& a, const cg_specs* s, const cg_zone* z, int64_t t0, int64_t t1,
                     int64_t cap, bool* empty);
bool async_pending(const cg_ctx* c);
// pipelined per-node calls (cg_pernode.hip): drain (errors kept for the next
// wait) / any pending
int pn_async_drain(cg_ctx* c);
bool pn_async_pending(const cg_ctx* c);  // an asynchronous expansion not yet waited for
// time-order tile sort + merge of c->node_time / c->node_rule (windows <= 4096 s;
// cg_node_order.hip), enqueued on st without a host sync
// in_mode: what the writer left in c->node_time / c->node_rule -- kInTimes
// int64 times + rules; kIn16 16-bit offsets t - t0 - 1 + rules
// (k_node_write<.., kOut16>); kInPacked one word per event, offset << 20 |
// (rule & 0xFFFFF), in c->node_rule (k_node_write<.., kOutPacked>; rules <
// 2^24: past 2^20 the tiles are cut where rule >> 20 changes and carry it)
constexpr int kInTimes = 0, kIn16 = 1, kInPacked = 2;
// the time-order writer may emit kInPacked for R rules (indices < 2^24)
bool pn_pack_ok(int64_t R);
// where every node's list crosses a multiple of 2^20 in rule index: the
// (node, band) segment offsets seg_pos [N*K+1] of bands of B rules (B a power
// of two <= 2^20, so 2^20 / B bands per block of 2^20 rules); null seg_pos:
// no cuts (rule indices < 2^20)
struct TileCut {
  const int64_t* seg_pos = nullptr;
  int32_t K = 1, B = 1;
  int64_t R = 0;
};
// err: a device word the kernels set when a sorted chunk is out of (time,
// rule) order (the sorts' ranks rest on lane-ordered LDS atomics; checked)
int order_merge_enqueue(cg_ctx* c, const int64_t* node_off, int32_t N, int64_t cap, int64_t t0, int64_t H,
                        hipStream_t st, int in_mode, int64_t* err, const TileCut& cut = TileCut());
constexpr const char* kOrderCheckMsg =
    "time-order pass: a sorted chunk came out of (time, rule) order (its LDS-atomic ranks were not in lane order)";
// the mapped pinned per-node result words: [0] node events, [1] size error, [2] order check
int pn_ensure_res(cg_ctx* c);
// the time-order pass over the last (rule-major) per-node result; c->mu held
int order_by_time_locked(cg_ctx* c, int in_mode = 0);
// kernels of the per-node CSR gather (cg_pernode.hip), enqueued on st:
// node n's events [src_off[n], src_off[n+1]) of src to dst_start[n] onwards /
// n contiguous events / the last per-node result's counts per node
// (event i of src_off's numbering at src_*[i - src_shift])
int launch_node_place(cg_ctx* c, hipStream_t st, int32_t N, const int64_t* src_off, int64_t src_shift,
                      const int64_t* src_time, const int32_t* src_rule, int32_t rule_add, const int64_t* dst_start,
                      int64_t* dst_time, int32_t* dst_rule);
int launch_span_place(cg_ctx* c, hipStream_t st, int64_t n, const int64_t* src_time, const int32_t* src_rule,
                      int32_t rule_add, int64_t* dst_time, int32_t* dst_rule);
int launch_node_counts(cg_ctx* c, hipStream_t st, int64_t* d_counts);
// Time-ordered gather: every node's list in d_time / d_rule holds W runs (the
// ranks' slices in rank = job-ID order, each in (time, rule) order); h_rb
// [N*(W+1)] (host) are the run bounds, node-major: run g of node n is
// [h_rb[n*(W+1)+g], h_rb[n*(W+1)+g+1]).  Merges every node's runs in place
// into (time, rule) order, one group of nodes of at most scratch_ev events at
// a time (a larger node alone) through a scratch copy (scr_t / scr_r), on st;
// returns after the stream has drained.
int merge_ranks_locked(cg_ctx* c, hipStream_t st, int32_t N, int32_t W, const int64_t* h_rb, int64_t* d_time,
                       int32_t* d_rule, int64_t scratch_ev, DBuf<int64_t>& scr_t, DBuf<int32_t>& scr_r);
constexpr int kMergeMaxRanks = 64;
// CG_ORDER_LSD set: order every window by the LSD passes (int64 times; the
// writer must not emit 16-bit offsets then)
bool order_lsd_only();
