/*
 * cron_oracle.h -- CPU restatement of cronsun's scheduling hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (cronsun_amd/, include/)
 * links, loads or calls this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg do, and only as the checker / CPU baseline.
 *
 * What it restates (reference = /root/reference, qlchan/cronsun):
 *   node/cron/spec.go:55-158         SpecSchedule.Next + dayMatches
 *   node/cron/parser.go:78-377       Parser.Parse, getField/getRange/getBits, descriptors
 *   node/cron/constantdelay.go:14-27 Every / ConstantDelaySchedule.Next
 *   job.go:274-288, 591-630          JobRule.included, Job.Cmds, Job.IsRunOn
 *   group.go:111-119                 Group.Included
 *   web/job.go:222-257               Job.GetJobNodes (cumulative excludes)
 *   job.go:194-233                   Cmd.lockTtl
 *   node/cron/cron.go:64-79,210-244  byTime + the Cron.run wake loop
 * plus the Go standard library `time` semantics the reference relies on but
 * which are not under /root/reference (third-party boundary, Go >= 1.15
 * semantics with TZif footer support): Location.lookup, tzset (POSIX TZ
 * footer), Date (normalisation + zone adjust), AddDate, Add, Truncate,
 * accessors, ParseDuration, strconv.Atoi.
 *
 * Parity pins: every known-answer case in node/cron/spec_test.go (74),
 * constantdelay_test.go (14) and parser_test.go (45) is transcribed as data
 * in tests/golden/kats.json and checked against this oracle by
 * tests/test_oracle_kats.py.
 *
 * Times are int64 unix seconds (+ int32 nanoseconds where Go keeps them).
 * Go's zero time.Time{} is represented by OR_ZERO_TIME = -62135596800.
 */
#ifndef CRON_ORACLE_H
#define CRON_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_ZERO_TIME (-62135596800LL)
/* returned where the reference's Next never terminates (see or_spec_next) */
#define OR_NO_PROGRESS (INT64_MIN + 1)

/* ---- Go *time.Location restatement ---- */
typedef struct or_loc or_loc;

/* LoadLocationFromTZData(name, data).  Returns 0 on success. */
int or_loc_from_tzif(const uint8_t *data, size_t len, or_loc **out);
/* time.FixedZone("", offset) */
int or_loc_fixed(int32_t offset, or_loc **out);
/* time.UTC (a Location with no zones) */
int or_loc_utc(or_loc **out);
void or_loc_free(or_loc *l);
/* Location.lookup(sec): offset, and the [start,end) Go reports. */
int32_t or_lookup(const or_loc *l, int64_t sec, int64_t *start, int64_t *end);

/* Civil fields of an instant in a location (Go accessors). */
typedef struct {
    int64_t year;
    int month, day, hour, minute, second, weekday, yday;
} or_fields;
void or_fields_of(int64_t usec, const or_loc *l, or_fields *f);
/* time.Date(y, mo, d, h, mi, s, 0, loc).Unix() */
int64_t or_date(int64_t y, int64_t mo, int64_t d, int64_t h, int64_t mi,
                int64_t s, const or_loc *l);

/* ---- node/cron schedules ---- */
#define OR_STAR_BIT (1ULL << 63)
typedef struct {
    uint64_t second, minute, hour, dom, month, dow;
} or_spec;

typedef struct {
    int kind;           /* 0 = *SpecSchedule, 1 = ConstantDelaySchedule */
    or_spec spec;
    int64_t delay_ns;   /* ConstantDelaySchedule.Delay (time.Duration) */
} or_sched;

/* SpecSchedule.Next(t) for t = (usec, nsec) in loc.  spec.go:55-145 */
int64_t or_spec_next(const or_spec *s, int64_t usec, int32_t nsec,
                     const or_loc *l);
/* Every(d).Delay  constantdelay.go:14-21 */
int64_t or_every(int64_t d_ns);
/* ConstantDelaySchedule.Next(t): returns unix seconds; result nsec is
 * always 0 (Delay is whole seconds).  constantdelay.go:25-27 */
int64_t or_const_next(int64_t delay_ns, int64_t usec, int32_t nsec);
int64_t or_sched_next(const or_sched *s, int64_t usec, int32_t nsec,
                      const or_loc *l);

/* ---- node/cron/parser.go ---- */
#define OR_OPT_SECOND 1
#define OR_OPT_MINUTE 2
#define OR_OPT_HOUR 4
#define OR_OPT_DOM 8
#define OR_OPT_MONTH 16
#define OR_OPT_DOW 32
#define OR_OPT_DOWOPTIONAL 64
#define OR_OPT_DESCRIPTOR 128
#define OR_OPT_DEFAULT (1 | 2 | 4 | 8 | 16 | 64 | 128)
#define OR_OPT_STANDARD (2 | 4 | 8 | 16 | 32 | 128)

/* Parser{options}.Parse(spec).  Returns 0 on success; on error returns -1
 * and writes Go's error text to err (NUL-terminated, truncated to errcap). */
int or_parse(int options, const char *spec, size_t len, or_sched *out,
             char *err, size_t errcap);
/* getRange / getField / getBits / all, exposed for the parser KATs. */
int or_get_range(const char *expr, size_t len, unsigned min, unsigned max,
                 uint64_t *bits, char *err, size_t errcap);
int or_get_field(const char *expr, size_t len, unsigned min, unsigned max,
                 uint64_t *bits, char *err, size_t errcap);
uint64_t or_get_bits(unsigned min, unsigned max, unsigned step);
/* time.ParseDuration; returns 0 on success. */
int or_parse_duration(const char *s, size_t len, int64_t *out, char *err,
                      size_t errcap);

/* ---- expansion loop (build-defined batch form of cron.go:212-215) ----
 * t = T0; loop { t = Next(t); if t.IsZero() || t > T1 break; emit t }
 * Returns the number of events (writes at most cap of them), or -1 when the
 * reference loop never terminates: Next never returns (OR_NO_PROGRESS) or
 * returns a time <= its input, after which the loop cycles. */
int64_t or_expand(const or_sched *s, int64_t t0, int64_t t1, const or_loc *l,
                  int64_t *out, int64_t cap);
/* Batch over R rules with nthreads POSIX threads.  offsets[R+1] is filled;
 * times may be NULL (count only).  Returns total events, or -1 if any rule
 * hit OR_NO_PROGRESS (its count is then 0). */
int64_t or_expand_batch(const or_sched *s, size_t R, int64_t t0, int64_t t1,
                        const or_loc *l, int nthreads, int64_t *offsets,
                        int64_t *times);

/* ---- rule -> node resolution (job.go / group.go / web/job.go) ----
 * Integer-interned form: nodes 0..N-1, groups 0..G-1, rules 0..R-1.
 * group_exists[g] == 0 models a gid with no entry in the groups map. */
typedef struct {
    int32_t n_nodes, n_groups, n_rules, n_jobs;
    const int64_t *group_off;  /* [G+1] */
    const int32_t *group_nodes;
    const uint8_t *group_exists;
    const int32_t *rule_job;   /* [R] job of each rule; rules of a job are contiguous, in order */
    const int64_t *nid_off;    /* [R+1] */
    const int32_t *nids;
    const int64_t *gid_off;    /* [R+1] */
    const int32_t *gids;
    const int64_t *ex_off;     /* [R+1] */
    const int32_t *ex;
    const uint8_t *job_pause;  /* [J] */
    const int32_t *rule_key;   /* [R] or NULL: Cmd key (Job.ID+Rule.ID, job.go:130-132),
                                  equal within a job exactly when the Rule.IDs are */
} or_jobset;

/* mode 0: reference scheduling path, Job.Cmds (excludes are a no-op,
 *         job.go:598-602; Pause => nothing).
 * mode 1: per-rule exclude (N_r \ E_r), Pause honoured.
 * mode 2: cumulative exclude as web/job.go:222-257 (N_r \ U_{j<=r} E_j within
 *         the job), Pause honoured.
 * In every mode a rule is dropped on n when a later rule of its job with the
 * same rule_key is scheduled on n too: Job.Cmds' map keeps the last included
 * rule per Cmd.GetID() (job.go:604-609).
 * Returns 1 if rule r is scheduled on node n. */
int or_rule_on_node(const or_jobset *js, int mode, int32_t r, int32_t n);
/* Job.IsRunOn(nid, groups)  job.go:616-630 (ignores Pause). */
int or_job_is_run_on(const or_jobset *js, int32_t job, int32_t n);
/* Job.GetJobNodes node list (web/job.go:222-257, first-seen order).
 * Returns the count; writes at most cap node ids. */
int32_t or_job_nodes(const or_jobset *js, int32_t job, int32_t *out,
                     int32_t cap);
/* Each requested node's own filter over every rule (node/node.go:121-158 ->
 * Job.Cmds): off[k+1] offsets and out[] = the rules scheduled on nodes[i]
 * (per mode, ascending), nthreads host threads.  out may be NULL (counts
 * only).  Returns the total. */
int64_t or_node_rules_batch(const or_jobset *js, int mode, const int32_t *nodes, size_t k,
                            int nthreads, int64_t *off, int32_t *out);

/* Cron.run (node/cron/cron.go:210-275), one wake at a time.  An entry is a
 * schedule + Next + Prev + id (the caller's handle). */
typedef struct {
    const or_sched *s;
    int64_t next, prev;
    int32_t id;
} or_entry;
/* run() start: entry.Next = entry.Schedule.Next(now) (cron.go:212-215) */
void or_cron_start(or_entry *e, size_t n, int64_t now, const or_loc *l);
/* sort.Sort(byTime) (cron.go:64-79, 220) in place; returns entries[0].Next,
 * or OR_ZERO_TIME when there are no entries or it is zero (cron.go:223-230) */
int64_t or_cron_effective(or_entry *e, size_t n);
/* the timer fired at `now` (cron.go:234-244): walk the sorted entries while
 * Next == effective, Prev = Next, Next = Schedule.Next(now); writes the ids
 * run, returns how many */
int64_t or_cron_fire(or_entry *e, size_t n, int64_t effective, int64_t now,
                     const or_loc *l, int32_t *due_ids);

/* Cmd.lockTtl() (job.go:194-233) with time.Now() = (now, now_nsec), the
 * rule's schedule in loc, Job.Kind, Job.AvgTime (ms) and conf LockTtl.
 * OR_NO_PROGRESS where a Next call never returns. */
#define OR_KIND_COMMON 0
#define OR_KIND_ALONE 1
#define OR_KIND_INTERVAL 2
int64_t or_lock_ttl(const or_sched *s, int64_t now, int32_t now_nsec,
                    const or_loc *l, int kind, int64_t avg_time,
                    int64_t lock_ttl);

#ifdef __cplusplus
}
#endif
#endif
