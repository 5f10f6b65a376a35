/*
 * abi_c.c -- the C-ABI (include/cronsun_gpu.h) driven from plain C11, in the
 * call order of the cgo stub node/cron/gpu/gpu.go: parse -> zone -> upload ->
 * next_batch -> expand (with the CG_ECAPACITY re-query) -> jobset ->
 * per-node -> lockTtl -> dispatcher.  Test infrastructure:
 * tests/test_abi_c.py compiles it with `gcc -std=c11 -pedantic -Werror` and
 * compares what it prints with the oracle.
 *
 *   abi_c <zoneinfo dir> check        the call sequence; "K key values..." lines
 *   abi_c <zoneinfo dir> bench FILE   FILE: one spec per line; 20 timed
 *                                     cg_expand_device calls over 24 h (UTC)
 *
 * Without a gfx950 device cg_init fails with CG_ENODEV; the host-side calls
 * (parser, zones, jobset) still run and the program prints "NODEV".
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/cronsun_gpu.h"

#define T0 1767571200LL /* 2026-01-05T00:00:00Z */
#define CHECK(x)                                                                  \
  do {                                                                            \
    int rc_ = (x);                                                                \
    if (rc_ != CG_OK) {                                                           \
      fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_,      \
              cg_last_error());                                                   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

static const char* kSpecs[] = {
    "0 */5 * * * *",    "0 30 9 * * 1-5",      "0 0 12 1,15 * Mon", "@daily",
    "@every 90s",       "*/10 * * * * *",      "0 0 0 30 Feb ?",    "15/35 20-35/15 1/2 */2 * *",
    "0 30 2 * * *",     "0 0 0 29 Feb ?",      "@hourly",           "59 59 23 * * Sun"};
#define NSPEC ((int)(sizeof kSpecs / sizeof kSpecs[0]))

static unsigned char* read_file(const char* path, size_t* len) {
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  fseek(f, 0, SEEK_END);
  long n = ftell(f);
  fseek(f, 0, SEEK_SET);
  unsigned char* b = (unsigned char*)malloc(n > 0 ? (size_t)n : 1);
  *len = fread(b, 1, (size_t)(n > 0 ? n : 0), f);
  fclose(f);
  return b;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int bench(const char* path) {
  size_t len = 0;
  char* text = (char*)read_file(path, &len);
  if (!text) return 2;
  size_t n = 0, cap = 1 << 20;
  const char** specs = (const char**)malloc(cap * sizeof *specs);
  size_t* lens = (size_t*)malloc(cap * sizeof *lens);
  for (char* p = text; p < text + len;) {
    char* e = memchr(p, '\n', (size_t)(text + len - p));
    if (!e) e = text + len;
    if (n == cap) {
      cap *= 2;
      specs = (const char**)realloc(specs, cap * sizeof *specs);
      lens = (size_t*)realloc(lens, cap * sizeof *lens);
    }
    specs[n] = p;
    lens[n] = (size_t)(e - p);
    n++;
    p = e + 1;
  }
  cg_schedule* s = (cg_schedule*)malloc(n * sizeof *s);
  int32_t* st = (int32_t*)malloc(n * sizeof *st);
  double tp = now_s();
  CHECK(cg_parse_batch(CG_PARSE_DEFAULT, specs, lens, n, s, st, 16));
  tp = now_s() - tp;
  for (size_t i = 0; i < n; i++)
    if (st[i] != CG_OK) return 3;
  cg_ctx* ctx;
  CHECK(cg_init(0, &ctx));
  cg_zone* utc;
  CHECK(cg_zone_utc(&utc));
  cg_specs* sp;
  CHECK(cg_specs_upload_schedules(ctx, s, n, &sp));
  CHECK(cg_set_phase_timing(ctx, 1));
  int64_t E = 0;
  for (int w = 0; w < 5; w++) CHECK(cg_expand_device(ctx, sp, utc, T0, T0 + 86400, &E));
  double t = now_s();
  const int steps = 20;
  float writer = 0.f;
  for (int k = 0; k < steps; k++) {
    CHECK(cg_expand_device(ctx, sp, utc, T0, T0 + 86400, &E));
    float ms[12];
    cg_last_kernel_times(ctx, ms, 12);
    writer += ms[3];
  }
  t = now_s() - t;
  printf("B rules %zu events %lld parse_s %.4f ms_per_step %.4f writer_ms %.4f events_per_s %.4e\n", n,
         (long long)E, tp, t / steps * 1e3, writer / steps, (double)E * steps / t);
  cg_specs_free(sp);
  cg_zone_free(utc);
  cg_destroy(ctx);
  free(s);
  free(st);
  free(specs);
  free(lens);
  free(text);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  if (strcmp(argv[2], "bench") == 0) return argc > 3 ? bench(argv[3]) : 2;
  if (cg_abi_version() != CG_ABI_VERSION) return 4;

  /* cron.Parse (parser.go:181-183) */
  cg_schedule sched[NSPEC];
  char err[256];
  for (int i = 0; i < NSPEC; i++)
    CHECK(cg_parse(CG_PARSE_DEFAULT, kSpecs[i], strlen(kSpecs[i]), &sched[i], err, sizeof err));
  if (cg_parse(CG_PARSE_DEFAULT, "* * *", 5, &sched[0], err, sizeof err) != CG_EPARSE) return 5;
  printf("P parse_error %s\n", err);
  CHECK(cg_parse(CG_PARSE_DEFAULT, kSpecs[0], strlen(kSpecs[0]), &sched[0], err, sizeof err));

  /* zones: LoadLocationFromTZData */
  char path[1024];
  snprintf(path, sizeof path, "%s/America/New_York", argv[1]);
  size_t zlen = 0;
  unsigned char* tzif = read_file(path, &zlen);
  if (!tzif) return 6;
  cg_zone* ny;
  CHECK(cg_zone_from_tzif(tzif, zlen, &ny));
  free(tzif);
  int32_t off = 0;
  CHECK(cg_zone_offset(ny, 1772953200, &off));
  printf("Z offset_after_spring_forward %d\n", off);

  /* jobs and groups (job.go:38-84, group.go:17-22) interned on the host */
  cg_jobset* js;
  CHECK(cg_jobset_new(&js));
  const char* g1[] = {"n1", "n2", "n3"};
  const char* g2[] = {"n3", "n4"};
  CHECK(cg_jobset_add_group(js, "g1", g1, 3));
  CHECK(cg_jobset_add_group(js, "g2", g2, 2));
  for (int i = 0; i < NSPEC; i++) {
    char id[16];
    snprintf(id, sizeof id, "job%d", i);
    CHECK(cg_jobset_add_job(js, id, i == 7));
    const char* gids[] = {i % 2 ? "g1" : "g2"};
    const char* nids[] = {"n5"};
    const char* ex[] = {"n3"};
    CHECK(cg_jobset_add_rule(js, "r", gids, 1, nids, (size_t)(i % 3 == 0), ex, (size_t)(i % 4 == 0)));
  }
  cg_rules_in rules;
  CHECK(cg_jobset_rules(js, &rules));
  printf("J rules %d nodes %d groups %d jobs %d\n", rules.n_rules, rules.n_nodes, rules.n_groups,
         rules.n_jobs);

  cg_ctx* ctx = NULL;
  int rc = cg_init(0, &ctx);
  if (rc == CG_ENODEV) {
    printf("NODEV %s\n", cg_last_error());
    cg_jobset_free(js);
    cg_zone_free(ny);
    return 0;
  }
  CHECK(rc);

  /* upload -> Schedule.Next for every rule (cron.go:212-215) */
  cg_specs* sp;
  CHECK(cg_specs_upload_schedules(ctx, sched, NSPEC, &sp));
  int64_t tin[NSPEC], tout[NSPEC];
  for (int i = 0; i < NSPEC; i++) tin[i] = 1772953200LL - 3600 + 977 * i;
  CHECK(cg_next_batch(ctx, sp, ny, tin, tout));
  printf("N");
  for (int i = 0; i < NSPEC; i++) printf(" %lld", (long long)tout[i]);
  printf("\n");

  /* the Next loop over (t0, t1], sized by CG_ECAPACITY */
  const int64_t t0 = 1772953200LL - 12 * 3600, t1 = t0 + 2 * 86400;
  int64_t offsets[NSPEC + 1];
  int64_t small[4];
  cg_csr csr = {offsets, small, 4, 0};
  rc = cg_expand(ctx, sp, ny, t0, t1, &csr);
  if (rc != CG_ECAPACITY) return 7;
  int64_t* times = (int64_t*)malloc((size_t)csr.n_events * sizeof *times);
  csr.times = times;
  csr.times_cap = csr.n_events;
  CHECK(cg_expand(ctx, sp, ny, t0, t1, &csr));
  printf("E %lld", (long long)csr.n_events);
  for (int i = 0; i <= NSPEC; i++) printf(" %lld", (long long)offsets[i]);
  printf("\n");
  printf("T");
  for (int64_t k = 0; k < csr.n_events; k++) printf(" %lld", (long long)times[k]);
  printf("\n");
  free(times);

  /* every node's Job.Cmds filter + its Next loop (node.go:121-158) */
  int64_t node_off[64];
  cg_node_csr nc;
  memset(&nc, 0, sizeof nc);
  nc.node_off = node_off;
  CHECK(cg_expand_per_node(ctx, sp, ny, t0, t1, &rules, CG_EXCLUDE_NONE, &nc));
  int64_t* nt = (int64_t*)malloc((size_t)(nc.n_events + 1) * sizeof *nt);
  int32_t* nr = (int32_t*)malloc((size_t)(nc.n_events + 1) * sizeof *nr);
  CHECK(cg_node_result_copy(ctx, NULL, nt, nr, nc.n_events));
  printf("M %lld %lld", (long long)nc.n_events, (long long)nc.nnz);
  for (int n = 0; n <= rules.n_nodes; n++) printf(" %lld", (long long)node_off[n]);
  printf("\n");
  for (int n = 0; n < rules.n_nodes; n++) {
    printf("L %s", cg_jobset_node_id(js, n));
    for (int64_t k = node_off[n]; k < node_off[n + 1]; k++) printf(" %d:%lld", nr[k], (long long)nt[k]);
    printf("\n");
  }
  /* the same lists in the node scheduler's byTime order (cron.go:64-79) */
  CHECK(cg_node_result_order_by_time(ctx));
  CHECK(cg_node_result_copy(ctx, NULL, nt, nr, nc.n_events));
  for (int n = 0; n < rules.n_nodes; n++) {
    printf("O %s", cg_jobset_node_id(js, n));
    for (int64_t k = node_off[n]; k < node_off[n + 1]; k++) printf(" %d:%lld", nr[k], (long long)nt[k]);
    printf("\n");
  }
  /* ... and written in that order by the per-node call itself (the cgo
     stub's ExpandPerNode with byTime) */
  CHECK(cg_set_node_order(ctx, CG_NODE_ORDER_TIME));
  CHECK(cg_expand_per_node(ctx, sp, ny, t0, t1, &rules, CG_EXCLUDE_NONE, &nc));
  CHECK(cg_node_result_copy(ctx, NULL, nt, nr, nc.n_events));
  CHECK(cg_set_node_order(ctx, CG_NODE_ORDER_RULE));
  for (int n = 0; n < rules.n_nodes; n++) {
    printf("Q %s", cg_jobset_node_id(js, n));
    for (int64_t k = node_off[n]; k < node_off[n + 1]; k++) printf(" %d:%lld", nr[k], (long long)nt[k]);
    printf("\n");
  }
  free(nt);
  free(nr);

  /* Cmd.lockTtl (job.go:194-233) */
  int32_t kind[NSPEC];
  int64_t avg[NSPEC], ttl[NSPEC];
  for (int i = 0; i < NSPEC; i++) {
    kind[i] = i % 3;
    avg[i] = 1000 * (int64_t)i - 2500;
  }
  CHECK(cg_lock_ttl_batch(ctx, sp, ny, tin, kind, avg, 300, ttl));
  printf("K");
  for (int i = 0; i < NSPEC; i++) printf(" %lld", (long long)ttl[i]);
  printf("\n");

  /* Cron.run: start, three wakes, one replace, one removal (cron.go:210-275) */
  cg_dispatcher* d;
  CHECK(cg_dispatcher_new(ctx, sp, ny, t0, &d));
  for (int w = 0; w < 3; w++) {
    int64_t eff, n_due, next_eff;
    CHECK(cg_dispatcher_effective(d, &eff));
    CHECK(cg_dispatcher_fire(d, eff, &n_due, &next_eff));
    int32_t due[NSPEC];
    CHECK(cg_dispatcher_due(d, 0, n_due, due));
    printf("W %lld", (long long)eff);
    for (int64_t k = 0; k < n_due; k++) printf(" %d", due[k]);
    printf("\n");
    if (w == 0) {
      int64_t slot = 2;
      CHECK(cg_dispatcher_set(d, &slot, &sched[4], 1, eff));
      slot = 5;
      CHECK(cg_dispatcher_remove(d, &slot, 1));
    }
  }
  cg_dispatcher_free(d);
  cg_specs_free(sp);
  cg_jobset_free(js);
  cg_zone_free(ny);
  cg_destroy(ctx);
  printf("OK\n");
  return 0;
}
