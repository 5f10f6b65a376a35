/*
 * cronsun_gpu.h -- C-ABI of the MI355X fire-time expansion engine for
 * cronsun's scheduling path (library: cronsun_amd/libcronsun_gpu.so).
 *
 * This is the boundary a Go cgo package `node/cron/gpu` binds (see
 * INTEGRATION.md).  Plain pointers and sizes only; no C++ or torch types.
 * Every entry point names the reference interface it replaces
 * (paths relative to qlchan/cronsun).
 *
 * Conventions
 *   - Return value: CG_OK (0) or a negative CG_E* code; cg_last_error()
 *     returns a thread-local message for the last failure on this thread.
 *   - Times are int64 unix seconds.  Go's zero time.Time{} (the "never fires"
 *     result of Schedule.Next) is CG_ZERO_TIME = -62135596800.
 *   - Input buffers are owned by the caller and only read during the call;
 *     nothing is retained (cgo rule: Go memory is never kept).
 *   - A cg_ctx owns one HIP device, its stream and its device buffers.  Calls
 *     on one ctx are serialised internally; calls block the calling thread.
 *   - There is no CPU fallback: compute entry points fail with CG_ENODEV
 *     when no MI355X (gfx950) device is usable.
 */
#ifndef CRONSUN_GPU_H
#define CRONSUN_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: cg_rules_in.rule_key (Job.Cmds' Job.ID+Rule.ID map key)
 * 3: time-ordered per-node gather (cg_comm_gather_node_csr on time-ordered
 *    results, cg_node_csr_merge_ranks), cg_comm_gather_plan */
#define CG_ABI_VERSION 3

#define CG_OK 0
#define CG_EINVAL (-1)    /* bad argument */
#define CG_ENOMEM (-2)    /* host or device allocation failed */
#define CG_EHIP (-3)      /* HIP runtime error */
#define CG_ECAPACITY (-4) /* output buffer too small; required size reported */
#define CG_EPARSE (-5)    /* spec did not parse; message via cg_last_error */
#define CG_ERANGE (-6)    /* time range/horizon outside supported bounds */
#define CG_ENODEV (-7)    /* no usable gfx950 device */
#define CG_EPANIC (-8)    /* input on which the reference Go code panics */

#define CG_ZERO_TIME (-62135596800LL)

/* ParseOption bits -- node/cron/parser.go:17-26 */
#define CG_PARSE_SECOND 1
#define CG_PARSE_MINUTE 2
#define CG_PARSE_HOUR 4
#define CG_PARSE_DOM 8
#define CG_PARSE_MONTH 16
#define CG_PARSE_DOW 32
#define CG_PARSE_DOW_OPTIONAL 64
#define CG_PARSE_DESCRIPTOR 128
/* defaultParser, parser.go:171-173 (cron.Parse) */
#define CG_PARSE_DEFAULT (1 | 2 | 4 | 8 | 16 | 64 | 128)
/* standardParser, parser.go:155-157 (cron.ParseStandard) */
#define CG_PARSE_STANDARD (2 | 4 | 8 | 16 | 32 | 128)

#define CG_STAR_BIT (1ULL << 63) /* spec.go:48-51 */

/* A parsed cron.Schedule: *SpecSchedule (spec.go:7-9) or
 * ConstantDelaySchedule (constantdelay.go:7-9). */
typedef struct {
  int32_t kind; /* 0 = SpecSchedule, 1 = ConstantDelaySchedule */
  int32_t reserved;
  uint64_t second, minute, hour, dom, month, dow; /* SpecSchedule fields */
  int64_t delay_ns;                               /* ConstantDelaySchedule.Delay */
} cg_schedule;

typedef struct cg_ctx cg_ctx;
typedef struct cg_zone cg_zone;
typedef struct cg_specs cg_specs;
typedef struct cg_jobset cg_jobset;

/* ---------------------------------------------------------------- misc --- */
int cg_abi_version(void);
const char* cg_last_error(void);
/* number of gfx950 devices visible (0 on a host without one) */
int cg_device_count(void);
/* Build flags of the loaded library (instrumentation; no reference
 * counterpart).  CG_BUILD_DIAG: the diagnostic build (`make diag`), whose
 * writer honours probe/variant environment switches that replace or drop
 * output stores -- never a production or benchmark library. */
#define CG_BUILD_DIAG 1
int cg_build_info(void);

/* ------------------------------------------------------ parse (host) --- */
/* Parser{options}.Parse(spec) -- parser.go:78-136; cron.Parse is options =
 * CG_PARSE_DEFAULT (parser.go:181-183), cron.ParseStandard CG_PARSE_STANDARD
 * (parser.go:167-169).  On error returns CG_EPARSE and copies Go's message
 * into err (NUL-terminated, truncated to err_cap) and cg_last_error(). */
int cg_parse(int options, const char* spec, size_t len, cg_schedule* out, char* err,
             size_t err_cap);
/* Batch form: n specs, status[i] = 0 or a CG_E* code. */
int cg_parse_batch(int options, const char* const* specs, const size_t* lens, size_t n,
                   cg_schedule* out, int32_t* status, int nthreads);
/* Parser internals, exposed for the reference's parser KATs
 * (parser_test.go TestRange/TestField/TestBits): getRange (parser.go:204-267),
 * getField (parser.go:188-199), getBits (parser.go:293-306).  names: 0 none,
 * 1 month names, 2 day-of-week names. */
int cg_get_range(const char* expr, size_t len, unsigned min, unsigned max, int names,
                 uint64_t* bits, char* err, size_t err_cap);
int cg_get_field(const char* expr, size_t len, unsigned min, unsigned max, int names,
                 uint64_t* bits, char* err, size_t err_cap);
uint64_t cg_get_bits(unsigned min, unsigned max, unsigned step);
/* Every(d).Delay -- constantdelay.go:14-21 */
int64_t cg_every(int64_t duration_ns);
/* time.ParseDuration (used by "@every", parser.go:368-373) */
int cg_parse_duration(const char* s, size_t len, int64_t* out_ns);

/* ------------------------------------------------------------- zones --- */
/* time.LoadLocationFromTZData (TZif v1-v4 incl. the POSIX footer). */
int cg_zone_from_tzif(const uint8_t* data, size_t len, cg_zone** out);
/* time.FixedZone("", offset_sec) */
int cg_zone_fixed(int32_t offset_sec, cg_zone** out);
/* time.UTC */
int cg_zone_utc(cg_zone** out);
void cg_zone_free(cg_zone* z);
/* Location.lookup(unix).offset (host, for inspection/tests) */
int cg_zone_offset(const cg_zone* z, int64_t unix_sec, int32_t* offset_sec);
/* The flat breakpoint table the kernels use for [lo, hi]: when[0] is
 * INT64_MIN, then every instant in (lo, hi] where the offset changes.
 * Returns the entry count (writes at most cap). */
int cg_zone_table(const cg_zone* z, int64_t lo, int64_t hi, int64_t* when, int32_t* off,
                  int cap);

/* ----------------------------------------------------------- context --- */
int cg_init(int device, cg_ctx** out);
void cg_destroy(cg_ctx* ctx);
/* wait for all work queued on the ctx's stream */
int cg_sync(cg_ctx* ctx);

/* -------------------------------------------------- specs (HBM SoA) --- */
/* SoA upload of SpecSchedule/ConstantDelaySchedule values (spec.go:7-9,
 * constantdelay.go:7-9).  delay_ns[i] > 0 marks rule i as @every; the mask
 * arrays are then ignored for it. Any array may be NULL if unused. */
typedef struct {
  const uint64_t* second;
  const uint64_t* minute;
  const uint64_t* hour;
  const uint64_t* dom;
  const uint64_t* month;
  const uint64_t* dow;
  const int64_t* delay_ns;
} cg_spec_soa;
int cg_specs_upload(cg_ctx* ctx, const cg_spec_soa* soa, size_t n_rules, cg_specs** out);
int cg_specs_upload_schedules(cg_ctx* ctx, const cg_schedule* s, size_t n_rules,
                              cg_specs** out);
/* rules [first, first+count) of an uploaded set, as a view (no copy) -- used
 * to shard rules by job-ID range across ranks.  Free views with
 * cg_specs_free as well; the view must not outlive its parent. */
int cg_specs_slice(cg_specs* specs, size_t first, size_t count, cg_specs** out);
size_t cg_specs_count(const cg_specs* specs);
void cg_specs_free(cg_specs* specs);

/* --------------------------------------------------------- Next() ------ */
/* out[i] = Schedule.Next(t_in[i]) for rule i, evaluated in zone z
 * (spec.go:55-145, constantdelay.go:25-27).  Host arrays of n = rule count.
 * Never-firing specs give CG_ZERO_TIME; a rule whose Next never returns
 * (AddDate stuck on a skipped local day) gives CG_NO_PROGRESS_TIME.  Replaces per-entry calls in
 * Cron.run (cron.go:212-215, 242-243) and Cmd.lockTtl (job.go:196-197). */
int cg_next_batch(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, const int64_t* t_in,
                  int64_t* t_out);

/* ---------------------------------------------------- Cmd.lockTtl() ---- */
/* ttl_out[i] = Cmd.lockTtl() (job.go:194-233) for rule i at time now[i]:
 *   prev = Next(now); ttl = Next(prev).Sub(prev) / Second (saturating);
 *   ttl == 0 -> 0 (lock() treats the rule as invalid, job.go:246-248);
 *   kind[i] == CG_JOB_INTERVAL -> clamp(ttl - 2, 1, lock_ttl);
 *   otherwise ttl -= cost when ttl >= cost, cost = avg_time_ms[i] / 1e3 in
 *   Go int64 arithmetic (so the ceiling at job.go:214 only fires for a
 *   negative AvgTime), then clamp to [2, lock_ttl].
 * kind = Job.Kind (job.go:30-34), avg_time_ms = Job.AvgTime,
 * lock_ttl = conf.Config.LockTtl (conf.go:136-138 defaults it to 300).
 * A rule whose Next never returns gets CG_NO_PROGRESS_TIME.  Host arrays of
 * n = rule count.  Replaces the per-Cmd call in newLock (job.go:235-241). */
#define CG_JOB_COMMON 0
#define CG_JOB_ALONE 1
#define CG_JOB_INTERVAL 2
#define CG_NO_PROGRESS_TIME (INT64_MIN + 1)
int cg_lock_ttl_batch(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, const int64_t* now,
                      const int32_t* kind, const int64_t* avg_time_ms, int64_t lock_ttl,
                      int64_t* ttl_out);

/* ------------------------------------------------------- dispatcher ---- */
/* The state of Cron.run (node/cron/cron.go:210-275) resident in HBM.  Entries
 * are slots 0..count-1 (the caller maps Entry IDs, cron.go:17-27 `indexes`,
 * to slots).  Each slot holds a schedule, Next and Prev (unix seconds;
 * CG_ZERO_TIME = zero time).
 *
 *   cg_dispatcher_new        run() start: Next = Schedule.Next(now) for every
 *                            entry of specs (cron.go:212-215); Prev = zero.
 *   cg_dispatcher_effective  entries[0].Next after sort.Sort(byTime)
 *                            (cron.go:220-230): the earliest non-zero Next, or
 *                            CG_ZERO_TIME when none (the loop then sleeps
 *                            ten years).
 *   cg_dispatcher_fire       the timer fired at `now` >= effective
 *                            (cron.go:234-244): every entry whose Next ==
 *                            effective is due; its Prev = Next and
 *                            Next = Schedule.Next(now).  Returns the due count
 *                            and the next effective time.
 *   cg_dispatcher_due        the last wake's due slots, ascending (the
 *                            reference runs them in byTime order, which is
 *                            unordered among equal Next values).
 *   cg_dispatcher_set        add or replace entries (cron.go:246-252,
 *                            125-142): slot idx[j] gets schedule s[j],
 *                            Next = Schedule.Next(now), Prev = zero.  Slots
 *                            past the current count extend it; skipped slots
 *                            stay empty.
 *   cg_dispatcher_remove     DelJob (cron.go:149-164, 254-262): the slot is
 *                            emptied and never fires.
 *   cg_dispatcher_snapshot   Entries() (cron.go:166-174, 296-308): Next, Prev
 *                            and liveness per slot (any pointer may be NULL).
 * A schedule whose Next never returns (the reference loop then blocks
 * forever) makes the call fail with CG_ERANGE naming the slot. */
typedef struct cg_dispatcher cg_dispatcher;
int cg_dispatcher_new(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t now,
                      cg_dispatcher** out);
void cg_dispatcher_free(cg_dispatcher* d);
int64_t cg_dispatcher_count(const cg_dispatcher* d);
int cg_dispatcher_effective(const cg_dispatcher* d, int64_t* effective);
int cg_dispatcher_fire(cg_dispatcher* d, int64_t now, int64_t* n_due, int64_t* effective);
int cg_dispatcher_due(const cg_dispatcher* d, int64_t first, int64_t count, int32_t* out);
/* the due list in HBM (valid until the next call on d) */
int cg_dispatcher_due_device(const cg_dispatcher* d, const int32_t** due, int64_t* n_due);
int cg_dispatcher_set(cg_dispatcher* d, const int64_t* idx, const cg_schedule* s, size_t k,
                      int64_t now);
int cg_dispatcher_remove(cg_dispatcher* d, const int64_t* idx, size_t k);
int cg_dispatcher_snapshot(const cg_dispatcher* d, int64_t* next, int64_t* prev, uint8_t* live);

/* --------------------------------------------------------- expansion --- */
/* counts[r] = number of fires of rule r in (t0, t1] (the expansion's count
 * pass alone: plan + k_count + scan; no times are written), *total = their
 * sum.  The cheap pass that balances job-ID-range shards by estimated events
 * (SURVEY.md §8e).  Leaves no expansion result behind. */
int cg_count(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0, int64_t t1,
             int64_t* counts, int64_t* total);

/* Fire times of every rule over (t0, t1]: for each rule,
 *   t = t0; loop { t = Next(t); if t.IsZero() || t > t1 break; emit t }
 * i.e. the reference Next loop, batched.  Output is a rule-major CSR:
 *   offsets[R+1] (int64), times[offsets[R]] (int64, ascending per rule).
 * The reference loop takes any horizon (its only limit is Next's own: no
 * match within five calendar years of t returns the zero time and ends the
 * rule, spec.go:70-76 -- reproduced).  Internally the horizon is cut into
 * closed-form segments of <= 30 days, each continuing from the previous
 * segment's last fire; t1 - t0 may be up to CG_MAX_HORIZON seconds (40
 * years; CG_ERANGE beyond, or if a zone's transitions need more than 1024
 * segments). */
#define CG_MAX_HORIZON (14610LL * 86400)
typedef struct {
  int64_t* offsets;  /* [R+1], caller-allocated (may be NULL) */
  int64_t* times;    /* [times_cap], caller-allocated (may be NULL) */
  int64_t times_cap;
  int64_t n_events;  /* out: total events (always set, also on CG_ECAPACITY) */
} cg_csr;
int cg_expand(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0, int64_t t1,
              cg_csr* out);

/* Device-resident variant: runs the whole expansion on the ctx's stream and
 * leaves offsets/times in device memory owned by the ctx (valid until the next
 * expansion call on this ctx).  *n_events is set.  Used for benchmarks and by
 * multi-GPU drivers that keep results in HBM. */
int cg_expand_device(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0,
                     int64_t t1, int64_t* n_events);
/* Pipelined variant for back-to-back calls (a scheduler's tick loop over
 * consecutive windows, cron.go:212-215 per tick): enqueues the expansion and
 * returns without waiting.  The count/scan of a call overlap the previous
 * call's output write; each call's plan is staged without a stream sync, so
 * T0 may move every call.  Needs the output capacity left by an earlier
 * cg_expand_device large enough for every call's result: a call that would
 * exceed it writes nothing and cg_expand_wait returns CG_ECAPACITY.  Results
 * and errors are known only after cg_expand_wait, which waits for every
 * call issued since the last wait, returns the first error among them (a
 * rule whose reference loop never ends: CG_ERANGE, as cg_expand_device), and
 * sets *n_events of the last call, whose result the accessors below then
 * read.  cg_last_kernel_times [3] = the mean write time of those calls.
 * Every call writes into the same output buffer: after the wait only the
 * LAST call's result is readable (earlier calls leave nothing readable), and
 * a returned error may belong to any call since the previous wait (its
 * message names the rule or the sizes).  *n_events is always set (0 when no
 * asynchronous call was made).  While calls are pending the result accessors
 * below refuse with CG_EINVAL.  A synchronous expansion (cg_expand,
 * cg_expand_device, cg_count, cg_expand_per_node*) made while calls are
 * pending drains them and discards their results and errors: call
 * cg_expand_wait first to observe them. */
int cg_expand_device_async(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0,
                           int64_t t1);
int cg_expand_wait(cg_ctx* ctx, int64_t* n_events);
/* device pointers of the last device-resident result */
int cg_result_device(cg_ctx* ctx, const int64_t** d_offsets, const int64_t** d_times,
                     int64_t* n_events);
/* copy [first, first+count) of the last result's times to host */
int cg_result_copy_times(cg_ctx* ctx, int64_t first, int64_t count, int64_t* host_out);
int cg_result_copy_offsets(cg_ctx* ctx, int64_t* host_offsets /* [R+1] */);

/* Per-kernel device time of the last expansion (ms, HIP events on the ctx
 * stream): [0] count, [1] scan, [2] block map, [3] write (closed form),
 * [4] write (walk), [5] offsets; of the last per-node call: [6] rule->node
 * join, [7] transpose (when the join is rebuilt) + segment records + per-node
 * offsets, [8] per-node write; [12] the last time-order pass; of the last
 * dispatcher wake: [9] scan, [10] due compaction, [11] advance.  n = entries
 * written. */
int cg_last_kernel_times(cg_ctx* ctx, float* ms, int n);
/* Expansion phase timing: 2 (default) = a HIP event between every phase;
 * 1 = events around k_write_cf only ([3]; [0..2], [4], [5] read -1).  Events
 * recorded between kernels leave the GPU idle for several us each, so
 * throughput measurements use 1.  (No reference counterpart: instrumentation.) */
int cg_set_phase_timing(cg_ctx* ctx, int level);

/* Order-sensitive checksum of a device array on the ctx's device
 * (instrumentation for integrity and parity checks; no reference
 * counterpart): sum over i < n of mix(first_index + i, v[i] + add) mod 2^64,
 * v = int64 (elem_bytes 8) or int32 (elem_bytes 4), mix = a 64-bit finaliser.
 * Checksums of consecutive ranges add up, so a shard's output (first_index =
 * its global base) can be compared with its range of another result. */
int cg_checksum_device(cg_ctx* ctx, const void* d_ptr, int64_t n, int elem_bytes,
                       int64_t first_index, int64_t add, uint64_t* out);
/* Integrity helpers for benchmarks and tests (no reference counterpart):
 * fill `bytes` of a device buffer with one byte value (e.g. poison an output
 * before timed runs), and count the int64/int32 elements equal to `value`
 * (e.g. poison a later run left unwritten). */
int cg_fill_device(cg_ctx* ctx, void* d_ptr, int64_t bytes, int byte_value);
int cg_count_value_device(cg_ctx* ctx, const void* d_ptr, int64_t n, int elem_bytes, int64_t value,
                          int64_t* count);
/* The store ceiling of this device (instrumentation; no reference
 * counterpart): the rate at which `bytes` (a multiple of 16) of the device
 * buffer d_ptr can be written, measured on the ctx stream with HIP events as
 * the mean over `reps` launches after one warm-up, for three fills:
 *   ms[0]  k_fill_stream, 16 B per lane nontemporal stores, a grid-stride
 *          loop over the whole buffer at full occupancy (one launch);
 *   ms[1]  the same with plain stores;
 *   ms[2]  hipMemsetAsync of the same bytes.
 * The output-bound kernels' roofline fractions are also reported against the
 * fastest of the three.  The buffer's contents are overwritten. */
int cg_fill_rate_device(cg_ctx* ctx, void* d_ptr, int64_t bytes, int reps, float* ms /* [3] */);

/* --------------------------------------------- rule -> node resolution --- */
/* Integer-interned jobs/groups (host interns string IDs; see cg_jobset_*).
 * Resolution modes:
 *   CG_EXCLUDE_NONE       reference scheduling semantics, Job.Cmds/IsRunOn
 *                         (job.go:591-630): ExcludeNodeIDs has no effect (the
 *                         inner-loop `continue`, job.go:598-602); Pause => none.
 *   CG_EXCLUDE_RULE       per-rule exclusion N_r \ E_r; Pause => none.
 *   CG_EXCLUDE_CUMULATIVE web/job.go:222-257 GetJobNodes: N_r \ U_{q<=r} E_q
 *                         over the job's rules in order; Pause => none. */
#define CG_EXCLUDE_NONE 0
#define CG_EXCLUDE_RULE 1
#define CG_EXCLUDE_CUMULATIVE 2
typedef struct {
  int32_t n_nodes, n_groups, n_rules, n_jobs;
  const int64_t* group_off;     /* [G+1] group -> node CSR (Group.NodeIDs, group.go:17-22) */
  const int32_t* group_nodes;
  const uint8_t* group_exists;  /* [G] 0 = gid referenced but absent from the groups map */
  const int32_t* rule_job;      /* [R] owning job; a job's rules are contiguous, in order */
  const int64_t* nid_off;       /* [R+1] JobRule.NodeIDs */
  const int32_t* nids;
  const int64_t* gid_off;       /* [R+1] JobRule.GroupIDs */
  const int32_t* gids;
  const int64_t* ex_off;        /* [R+1] JobRule.ExcludeNodeIDs */
  const int32_t* ex;
  const uint8_t* job_pause;     /* [J] Job.Pause */
  /* [R] or NULL: the rule's Cmd key (job.go:130-132 Cmd.GetID() = Job.ID +
   * Rule.ID), interned to any int32 such that two rules OF THE SAME JOB have
   * equal values exactly when their Rule.IDs are equal.  Job.Cmds keeps one
   * Cmd per key -- `cmds[cmd.GetID()] = cmd` (job.go:604-609): the LAST
   * included rule of the job with that key -- and the node's Cron replaces an
   * entry by ID (node/node.go:209-211, node/cron/cron.go:131-135).  So in
   * every mode the pair (r, n) is dropped when a later rule of r's job with
   * the same key is also scheduled on n (under the same mode: RULE and
   * CUMULATIVE test the later rule with their own exclusion).  Keys are only
   * compared within a job: equal Job.ID+Rule.ID strings of DIFFERENT jobs
   * ("a"+"bc", "ab"+"c") replace each other in the reference in the random
   * order of GetJobs' map, so both are kept here.  NULL: every rule is its
   * own key (the caller guarantees distinct Rule.IDs within a job).
   * cg_jobset_rules fills it from the Rule.IDs. */
  const int32_t* rule_key;
} cg_rules_in;

/* Per-node fire lists: for every node n, the (time, rule) events of the rules
 * scheduled on n (per `mode`), rule-major in ascending rule index, times
 * ascending within a rule.  Output CSR: node_off[N+1], time[], rule[].
 * Replaces every node's Node.loadJobs -> addJob -> Job.Cmds filter
 * (node/node.go:121-158) plus its Cron entries' Next loop. */
typedef struct {
  int64_t* node_off;  /* [N+1] caller-allocated (may be NULL) */
  int64_t* time;      /* [cap] */
  int32_t* rule;      /* [cap] */
  int64_t cap;
  int64_t n_events;   /* out */
  int64_t nnz;        /* out: sum over rules of |nodes(rule)| */
} cg_node_csr;
int cg_expand_per_node(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0,
                       int64_t t1, const cg_rules_in* rules, int mode, cg_node_csr* out);
/* device-resident variant (bench / multi-GPU); results stay in ctx memory */
int cg_expand_per_node_device(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0,
                              int64_t t1, const cg_rules_in* rules, int mode,
                              int64_t* n_events, int64_t* nnz);
/* device pointers of the last per-node result */
int cg_node_result_device(cg_ctx* ctx, const int64_t** d_node_off, const int64_t** d_time,
                          const int32_t** d_rule, int64_t* n_events);
/* Reorder every node's list of the last per-node result by (time, rule), in
 * device memory: the order the node's scheduler keeps its entries in
 * (Cron.run's sort.Sort(byTime), node/cron/cron.go:64-79,220; equal times in
 * ascending rule order, one of the orders that unstable sort may give).
 * Later cg_node_result_* calls see the ordered lists; the node offsets are
 * unchanged.  Time of the pass: cg_last_kernel_times [12]. */
int cg_node_result_order_by_time(cg_ctx* ctx);
/* Order in which the per-node calls (cg_expand_per_node*, synchronous and
 * pipelined) write every node's list:
 *   CG_NODE_ORDER_RULE  rule-major (rules ascending, times ascending within a
 *                       rule) -- the default, Job.Cmds' evaluation order
 *   CG_NODE_ORDER_TIME  (time, rule): the byTime order a node's Cron keeps
 *                       (cron.go:64-79,220): the call runs the time-order
 *                       pass of cg_node_result_order_by_time itself, after
 *                       the writer (the pipelined calls enqueue it behind
 *                       each window's writer, windows of at most 4096 s; a
 *                       longer pipelined window is refused with CG_EINVAL)
 * cg_node_result_order_by_time on a result already in time order does
 * nothing. */
#define CG_NODE_ORDER_RULE 0
#define CG_NODE_ORDER_TIME 1
int cg_set_node_order(cg_ctx* ctx, int order);
/* copy the last per-node result to host buffers (node_off [N+1]; time/rule
 * [n_events], cap = their capacity); any pointer may be NULL */
int cg_node_result_copy(cg_ctx* ctx, int64_t* node_off, int64_t* time, int32_t* rule, int64_t cap);
/* copy events [first, first+count) of the last per-node result (one node's
 * list is [node_off[n], node_off[n+1])) -- what a single node's scheduler
 * fetches; either pointer may be NULL */
int cg_node_result_copy_range(cg_ctx* ctx, int64_t first, int64_t count, int64_t* time,
                              int32_t* rule);
/* Integrity check for pipelined windows (instrumentation; no reference
 * counterpart): enqueues on the ctx's stream, right behind the last enqueued
 * per-node window (or the last synchronous result), order-sensitive checksums
 * of the lists of the k nodes d_nodes[] (device int32): d_out[2i] = sum_j
 * mix(j, time[j]), d_out[2i+1] = sum_j mix(j, rule[j]) over node d_nodes[i]'s
 * list, j node-relative, mix as cg_checksum_device (device uint64 [2k]).  A
 * window past the output capacity gives zeros.  Lets a caller check windows
 * whose result a later window overwrites. */
int cg_node_checksum_enqueue(cg_ctx* ctx, const int32_t* d_nodes, int32_t k, uint64_t* d_out);
/* per-node event counts of the last per-node result, copied to a DEVICE
 * buffer of N int64 (e.g. a torch tensor for an RCCL allgather) */
int cg_node_counts_to_device(cg_ctx* ctx, int64_t* d_counts);
/* Multi-GPU per-node gather, placement step (north_star: RCCL "gathers the
 * final per-node CSR"; the node lists node/node.go:121-158 builds from
 * Job.Cmds over every job in job-ID order).  One rank's slice of the
 * per-node CSR -- d_src_node_off[N+1] (from 0), d_src_time / d_src_rule
 * (rule indices local to the rank's job-ID range) -- is copied on the ctx's
 * device so that node n's slice starts at d_dst_start[n] (= the node's global
 * offset plus the slices of the ranks before this one, from the all-gathered
 * per-node counts) in d_dst_time / d_dst_rule, rule indices plus rule_add
 * (the range's first global rule).  All pointers are device memory of the
 * ctx's device; the call returns after the copy (stream synchronised). */
int cg_node_csr_place(cg_ctx* ctx, int32_t n_nodes, const int64_t* d_src_node_off, const int64_t* d_src_time,
                      const int32_t* d_src_rule, int32_t rule_add, const int64_t* d_dst_start,
                      int64_t* d_dst_time, int32_t* d_dst_rule);
/* Multi-GPU per-node gather, merge step for TIME-ORDERED slices (the byTime
 * order every node's Cron keeps, node/cron/cron.go:64-79,220): after each
 * rank's (time, rule)-ordered slice has been placed (cg_node_csr_place), node
 * n's list in d_time / d_rule holds `world` runs in rank (= job-ID) order, run
 * g = [run_bounds[n*(world+1)+g], run_bounds[n*(world+1)+g+1]) (HOST array of
 * n_nodes*(world+1) positions, ascending).  Every node's runs are merged in
 * place into (time, rule) order -- equal times by global rule index, which
 * for job-ID-range shards is rank order -- the list one scheduler over all
 * jobs would hold.  Works through a scratch copy of node groups of at most
 * budget_bytes / 12 events (a larger node alone; never more than the events
 * being merged); world <= 64.  Returns after the merge (stream synchronised). */
int cg_node_csr_merge_ranks(cg_ctx* ctx, int32_t n_nodes, int32_t world, const int64_t* run_bounds,
                            int64_t* d_time, int32_t* d_rule, int64_t budget_bytes);

/* Device-resident rule sets: a cg_rules_in validated and copied into HBM once
 * (as specs are by cg_specs_upload), then used by any number of per-node
 * expansions on the same ctx without re-upload.  Same resolution as
 * cg_expand_per_node_device (job.go:591-630 / web/job.go:222-257). */
typedef struct cg_rules cg_rules;
int cg_rules_upload(cg_ctx* ctx, const cg_rules_in* rules, cg_rules** out);
void cg_rules_free(cg_rules* rules);
int cg_expand_per_node_rules_device(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z,
                                    int64_t t0, int64_t t1, const cg_rules* rules, int mode,
                                    int64_t* n_events, int64_t* nnz);
/* Pipelined per-node windows for a node scheduler's tick loop
 * (node/node.go:121-158 filtering every job, node/cron/cron.go:210-275 firing
 * them, window after window): enqueues window (t0, t1] and returns.  Window
 * k+1's rule-major expansion, rule infos, segment records and node offsets
 * run on the ctx's second stream while window k's per-node writer streams.
 * Needs an earlier cg_expand_per_node_rules_device on the same rule set and
 * exclude mode (the rule->node join, its transpose and the band width are
 * reused) whose rule-major and per-node results were at least as large as
 * every window's: a window that would exceed them writes nothing and
 * cg_expand_per_node_wait returns CG_ECAPACITY.  Every window writes the same
 * per-node output: after the wait only the LAST window's result is readable
 * (cg_node_result_*), and a returned error may belong to any window since the
 * previous wait.  The per-node result accessors refuse (CG_EINVAL) while
 * windows are pending; a synchronous call drains them and discards their
 * results and errors.  The call refuses (CG_EINVAL) while pipelined
 * rule-major calls (cg_expand_device_async) are pending: wait for them first
 * (a per-node window replaces the readable rule-major result).  cg_last_kernel_times [8] = the mean per-node writer
 * time of the waited windows. */
int cg_expand_per_node_rules_device_async(cg_ctx* ctx, const cg_specs* specs, const cg_zone* z, int64_t t0,
                                          int64_t t1, const cg_rules* rules, int mode);
/* *n_events: the last window's node events (its result is then readable);
 * *n_events_all (may be NULL): the node events of every window waited for. */
int cg_expand_per_node_wait(cg_ctx* ctx, int64_t* n_events, int64_t* n_events_all);

/* ------------------------------------------- multi-GPU (RCCL over xGMI) --- */
/* One process (or thread) per MI355X, each with its own cg_ctx; rules shard
 * by contiguous job-ID ranges with no data-path collective (every cronsun
 * node filters every job itself, node/node.go:121-141; here a rank evaluates
 * one range of jobs for every node).  The only exchanges (north_star) are the
 * all-gather of per-node event counts / offsets and the gather of the final
 * per-node CSR.  RCCL is loaded at run time (see below); CG_ENODEV if absent.
 *
 *   cg_comm_unique_id   ncclGetUniqueId: rank 0 makes the id, the caller
 *                       hands it to every rank (any channel)
 *   cg_comm_init        ncclCommInitRank on the ctx's device (collective)
 *   cg_comm_allgather_i64  all[g*n + i] = rank g's mine[i] (host buffers;
 *                       event totals -> global rule-major offsets, per-block
 *                       weights of the event-balanced cut)
 *   cg_comm_node_offsets   all-gather of the per-node event counts of every
 *                       rank's last per-node result (N int64 per rank):
 *                       node_start[n] = node_base[n] + the counts of the
 *                       ranks before this one (where this rank's slice of
 *                       node n lands in the job-ID-ordered global list),
 *                       node_base[N+1] the global node offsets (host; either
 *                       may be NULL)
 *   cg_comm_gather_node_csr  every rank's last per-node result gathered on
 *                       `root` into the caller's DEVICE buffers
 *                       d_node_off [N+1], d_time / d_rule [cap] (root only;
 *                       ignored elsewhere): node n's global list is the ranks'
 *                       slices in rank (= job-ID) order, rule indices made
 *                       global by each rank's rule_base (its range's first
 *                       global rule).  When every rank's result is in (time,
 *                       rule) order (CG_NODE_ORDER_TIME), root merges each
 *                       node's slices into one (time, rule)-ordered list
 *                       (cg_node_csr_merge_ranks), the byTime list of one
 *                       scheduler over every job; ranks mixing the two orders
 *                       are refused, and so are time-ordered results of more
 *                       than 64 ranks or whose rule_base does not ascend with
 *                       the rank among the ranks holding events (the merge
 *                       breaks time ties by rank), on every rank before any
 *                       transfer.  The payload moves in chunks of whole
 *                       node ranges (a node larger than the budget in parts)
 *                       whose peer bytes (12 B per event) stay within
 *                       budget_bytes (the smallest any rank passes; at least
 *                       24 B per rank), so root's staging is bounded by it;
 *                       grouped ncclSend/ncclRecv per chunk, placed on root by
 *                       a kernel (root's staging, also the merge's scratch:
 *                       at most the budget, or the largest node when a time-
 *                       ordered node exceeds it).  Every rank returns the same
 *                       status: CG_ECAPACITY when the total exceeds root's
 *                       cap, CG_EINVAL when a rank has no readable result, the
 *                       node counts or list orders differ, and root's
 *                       allocation failure on every rank.  A transfer that
 *                       fails after all ranks agreed aborts the communicator
 *                       (later calls fail with CG_EHIP).  *n_events = the
 *                       global total.
 *   cg_comm_gather_plan the gather's chunk plan, host only (no device, no
 *                       communicator): counts [world * n_nodes] per-node event
 *                       counts of every rank; chunks[4i..4i+3] = {n0, n1, j,
 *                       k}: nodes [n0, n1) whole (k == 1), or part j of k of
 *                       node n0, rank g's part being its events [c*j/k,
 *                       c*(j+1)/k) of that node.  *n_chunks always set;
 *                       CG_ECAPACITY when it exceeds cap.
 * Collective calls must be made by every rank of the comm, in the same order.
 * RCCL is loaded by full path with local symbol scope, one copy per process:
 * one already mapped, else the librccl.so beside the HIP runtime the library
 * runs on, else /opt/rocm/lib; when a different RCCL is mapped later the
 * cg_comm calls fail with CG_EINVAL naming both. */
typedef struct cg_comm cg_comm;
#define CG_COMM_ID_BYTES 128
int cg_comm_unique_id(uint8_t id[CG_COMM_ID_BYTES]);
int cg_comm_init(cg_ctx* ctx, int world, int rank, const uint8_t id[CG_COMM_ID_BYTES], cg_comm** out);
void cg_comm_free(cg_comm* comm);
int cg_comm_allgather_i64(cg_comm* comm, const int64_t* mine, size_t n, int64_t* all);
int cg_comm_node_offsets(cg_comm* comm, int64_t* node_start, int64_t* node_base);
int cg_comm_gather_node_csr(cg_comm* comm, int root, int64_t rule_base, int64_t budget_bytes,
                            int64_t* d_node_off, int64_t* d_time, int32_t* d_rule, int64_t cap,
                            int64_t* n_events);
int cg_comm_gather_plan(const int64_t* counts, int32_t world, int32_t n_nodes, int32_t root,
                        int64_t budget_bytes, int64_t* chunks, int64_t cap, int64_t* n_chunks);

/* rule -> node CSR only (GPU join), host output */
int cg_rule_nodes(cg_ctx* ctx, const cg_rules_in* rules, int mode, int64_t* rn_off /*[R+1]*/,
                  int32_t* rn_nodes, int64_t cap, int64_t* nnz);

/* ----------------------------------- string-keyed job model (host) --- */
/* Host interning of cronsun's string IDs (Job/JobRule/Group, job.go:38-84,
 * group.go:17-22) into cg_rules_in.  Job IDs, rule IDs, group IDs and node
 * IDs are arbitrary byte strings (NUL-terminated here). */
int cg_jobset_new(cg_jobset** out);
void cg_jobset_free(cg_jobset* js);
int cg_jobset_add_group(cg_jobset* js, const char* gid, const char* const* nids, size_t n);
int cg_jobset_add_job(cg_jobset* js, const char* job_id, int pause);
/* appends a rule to the last added job */
int cg_jobset_add_rule(cg_jobset* js, const char* rule_id, const char* const* gids, size_t ng,
                       const char* const* nids, size_t nn, const char* const* ex, size_t ne);
/* freeze and expose the interned arrays (valid until the jobset is freed) */
int cg_jobset_rules(cg_jobset* js, cg_rules_in* out);
/* node index of a node ID (-1 if unknown) / node ID of an index */
int32_t cg_jobset_node_index(const cg_jobset* js, const char* nid);
const char* cg_jobset_node_id(const cg_jobset* js, int32_t idx);
/* Job.Cmds(nid, groups) keys (job.go:591-614): writes the rule indices of
 * the job's Cmds on node nid -- after the map's last-writer-wins dedup of
 * Job.ID+Rule.ID -- and returns their count (host reference semantics). */
int32_t cg_jobset_cmds(const cg_jobset* js, int32_t job, const char* nid, int32_t* rules_out,
                       int32_t cap);
/* Job.IsRunOn(nid, groups) (job.go:616-630) */
int cg_jobset_is_run_on(const cg_jobset* js, int32_t job, const char* nid);
/* Job.GetJobNodes (web/job.go:222-257): node indices in first-seen order */
int32_t cg_jobset_job_nodes(const cg_jobset* js, int32_t job, int32_t* nodes_out, int32_t cap);

/* ------------------------------------------ bulk ingestion (etcd JSON) --- */
/* GetGroups("") / GetJobs() (group.go:39-63, job.go:339-365) over the raw
 * etcd values: docs[i] is the JSON value of one key under /cronsun/group/
 * (groups) or /cronsun/cmd/ (jobs), in key order.  Each value goes through
 * json.Unmarshal into Group / Job (Go 1.7-1.8 encoding/json semantics, see
 * cg_ingest.cpp), Job.Valid (every rule's Timer through cron.Parse) and
 * alone(); the last valid value of an ID wins.  Decoding runs on nthreads
 * host threads.  status[i] (optional) gets one of: */
#define CG_INGEST_OK 0          /* added to the jobset */
#define CG_INGEST_UNMARSHAL 1   /* json.Unmarshal error: skipped (job.go:353-356) */
#define CG_INGEST_INVALID 2     /* Job.Valid error (ErrNilRule, parse error): skipped */
#define CG_INGEST_PANIC 3       /* a null rule: the reference panics in JobRule.Valid */
#define CG_INGEST_REPLACED 4    /* a later value with the same ID replaced it */
#define CG_INGEST_UNSUPPORTED 5 /* an ID containing NUL (not representable here) */
int cg_jobset_ingest_groups(cg_jobset* js, const char* const* docs, const size_t* lens, size_t n,
                            int nthreads, int32_t* status);
int cg_jobset_ingest_jobs(cg_jobset* js, const char* const* docs, const size_t* lens, size_t n,
                          int nthreads, int32_t* status);
/* JobRule.Schedule per rule (rule order of cg_jobset_rules); returns the rule
 * count (writes at most cap).  CG_EINVAL if a rule was added without a timer. */
int cg_jobset_schedules(const cg_jobset* js, cg_schedule* out, size_t cap);
/* Job.Kind, Job.AvgTime (ms) and Job.Parallels (after alone()) per job;
 * returns the job count (writes at most cap; any pointer may be NULL) */
int cg_jobset_job_meta(const cg_jobset* js, int32_t* kind, int64_t* avg_time_ms,
                       int64_t* parallels, size_t cap);
const char* cg_jobset_job_id(const cg_jobset* js, int32_t job);
const char* cg_jobset_group_id(const cg_jobset* js, int32_t group);
const char* cg_jobset_rule_id(const cg_jobset* js, int32_t rule);

#ifdef __cplusplus
}
#endif
#endif /* CRONSUN_GPU_H */
