// Host-side check of the batch Cmd.lockTtl algorithm (the k_lock_ttl body:
// next_exact twice on the zone table cg_lock_ttl_batch builds, then
// lock_ttl_of) against the oracle's or_lock_ttl (job.go:194-233 restated with
// Go's saturating Sub).  Test infrastructure; the GPU test checks the kernel.
#include <climits>
#include <random>

#include "host_common.h"

using namespace cg;

static const char* atoms[6][12] = {
    {"*", "0", "5", "*/7", "15/35", "10-40/3", "7,30,45", "59", "0/15", "3-3", "*/1", "58-59"},
    {"*", "0", "30", "*/5", "20-35/15", "1,31,59", "5-7/2", "*/59", "10-12", "0", "0", "59"},
    {"*", "0", "9", "23", "*/2", "1/2", "9-17", "22,23,0", "2", "1", "3", "0-23/5"},
    {"*", "?", "1", "15", "31", "29", "30", "1,15", "*/2", "9-20", "28-31", "5/7"},
    {"*", "?", "1", "2", "Feb", "Jan,Jul", "Apr-Oct", "*/3", "Mar", "Nov", "Dec", "*"},
    {"*", "?", "0", "1-5", "Mon", "Sun", "mon/2", "Sat,Sun", "*/2", "3", "fri-sat", "*"}};

int main(int argc, char** argv) {
  const char* zone = argc > 1 ? argv[1] : "UTC";
  int n = argc > 2 ? atoi(argv[2]) : 3000;
  ZoneRules zr;
  or_loc* ol = nullptr;
  load_zone(zone, &zr, &ol);
  std::mt19937_64 rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 99);
  const int64_t lo = 946684800, hi = 2208988800, kDay = 86400;
  // the table cg_lock_ttl_batch builds (cg_api.cpp)
  ZoneTable tab = build_table(zr, CG_ZERO_TIME - 64 * kDay, hi + (12 * 366 + 64) * kDay);
  ZoneView zv{tab.when.data(), tab.off.data(), int32_t(tab.when.size())};
  ZoneTable near = build_table(zr, lo, hi);
  const int64_t avgs[] = {0, 999, 1000, 1500, 3500, 12000, -1, -999, -1000, -2500, 3600000,
                          INT64_MIN, INT64_MAX, INT64_MIN + 999, -9223372036854775LL};
  const int64_t ttls[] = {300, 2, 1, 0, -5, 10, 86400, INT64_MAX, INT64_MIN};
  int bad = 0, zero = 0, noprog = 0;
  for (int i = 0; i < n; i++) {
    std::string spec;
    if (rng() % 8 == 0) spec = "@every " + std::to_string(1 + rng() % 7200) + "s";
    else for (int f = 0; f < 6; f++) { if (f) spec += " "; spec += atoms[f][rng() % 12]; }
    or_sched s;
    char err[256];
    if (or_parse(OR_OPT_DEFAULT, spec.c_str(), spec.size(), &s, err, sizeof err)) continue;
    int64_t now = lo + int64_t(rng() % uint64_t(hi - lo));
    if (near.when.size() > 1 && rng() % 3 == 0)
      now = near.when[1 + rng() % (near.when.size() - 1)] + int64_t(rng() % (2 * kDay)) - kDay;
    const int kind = int(rng() % 4) == 3 ? 7 : int(rng() % 3);
    const int64_t avg = rng() % 3 ? int64_t(rng() % 20000) - 5000 : avgs[rng() % 15];
    const int64_t L = ttls[rng() % 9];
    DSpec d = pack(s);
    int64_t prev, nxt;
    if (d.kind == KIND_EVERY) { prev = now + int64_t(d.sec); nxt = prev + int64_t(d.sec); }
    else {
      prev = next_exact(d, zv, now, INT64_MAX);
      nxt = prev == CG_NO_PROGRESS ? prev : next_exact(d, zv, prev, INT64_MAX);
    }
    int64_t got = lock_ttl_of(prev, nxt, kind, avg, L);
    int64_t exp = or_lock_ttl(&s, now, 0, ol, kind, avg, L);
    zero += exp == 0;
    noprog += exp == OR_NO_PROGRESS;
    if (got != exp && bad++ < 10)
      printf("MISMATCH %s [%s] now=%lld kind=%d avg=%lld L=%lld: %lld vs %lld\n", zone,
             spec.c_str(), (long long)now, kind, (long long)avg, (long long)L, (long long)got,
             (long long)exp);
  }
  printf("%s: %d mismatches (%d zero, %d no-progress)\n", zone, bad, zero, noprog);
  return bad ? 1 : 0;
}
