// Host-side check of the expansion algorithm (cg_expand.h: count_rule +
// closed-form iteration + WALK re-walk, exactly what k_count/k_write_cf/
// k_write_walk run) against the oracle's literal Next loop.  Test
// infrastructure; the GPU tests check the kernels themselves.
#include <algorithm>
#include <cstdlib>
#include <random>

#include "../../cronsun_amd/csrc/cg_expand.h"
#include "host_common.h"

using namespace cg;

static const char* atoms[6][16] = {
    {"*/7", "0", "5", "*/20", "15/35", "10-40/3", "7,30,45", "59", "0/15", "3-3", "0", "58-59", "0", "0", "30", "*/30"},
    {"*", "0", "30", "*/5", "20-35/15", "1,31,59", "5-7/2", "*/59", "10-12", "0", "0", "59", "45", "15", "0,30", "*/15"},
    {"*", "0", "9", "23", "*/2", "1/2", "9-17", "22,23,0", "2", "1", "3", "0-23/5", "0", "1", "0,1", "23"},
    {"*", "?", "1", "15", "31", "29", "30", "1,15", "*/2", "9-20", "28-31", "5/7", "8", "*", "?", "1-7"},
    {"*", "?", "1", "2", "Feb", "Jan,Jul", "Apr-Oct", "*/3", "Mar", "Nov", "Dec", "*", "*", "*", "Oct", "Sep-Dec"},
    {"*", "?", "0", "1-5", "Mon", "Sun", "mon/2", "Sat,Sun", "*/2", "3", "fri-sat", "*", "*", "0", "6", "?"}};

// long-horizon mode: sparse specs (at most one fire per matching hour) so that
// multi-year horizons stay cheap for the oracle's literal loop
static const char* long_atoms[6][8] = {
    {"0", "30", "15", "0", "0", "45", "0", "7"},
    {"0", "30", "0,30", "15", "0", "59", "0", "1"},
    {"*", "0", "9", "*/6", "12", "2", "1", "23"},
    {"*", "?", "1", "15", "29", "31", "28-31", "1,15"},
    {"*", "Feb", "Jan,Jul", "*/3", "Mar", "Nov", "*", "Feb"},
    {"*", "?", "Mon", "Sun", "1-5", "?", "*", "Sat"}};
static const char* long_specials[] = {"@yearly", "@monthly", "@weekly", "@daily", "0 0 0 29 Feb ?",
                                      "59 59 23 28,29 Feb ?", "0 0 12 29 Feb Mon", "0 30 2 * * *",
                                      "0 30 1 * * Sun", "0 0 0 31 * ?", "0 0 0 30 Feb ?"};

int main(int argc, char** argv) {
  const char* zone = argc > 1 ? argv[1] : "UTC";
  int nspec = argc > 2 ? atoi(argv[2]) : 400;
  const bool long_mode = argc > 4 && std::string(argv[4]) == "long";
  // near mode: T0 at many offsets around transitions of 2011-2027 (just before,
  // on, inside the overlap, hours and days after), 30-hour horizons
  const bool near_mode = argc > 4 && std::string(argv[4]) == "near";
  ZoneRules zr;
  or_loc* ol = nullptr;
  load_zone(zone, &zr, &ol);
  std::mt19937_64 rng(argc > 3 ? strtoull(argv[3], nullptr, 10) : 777);
  std::vector<or_sched> scheds;
  std::vector<std::string> names;
  size_t nspecial = 0;
  while ((int)scheds.size() < nspec) {
    std::string spec;
    if (long_mode && nspecial < sizeof long_specials / sizeof long_specials[0])
      spec = long_specials[nspecial++];
    else if (long_mode && rng() % 10 == 0)
      spec = "@every " + std::to_string(3600 + rng() % (3 * 86400)) + "s";
    else if (long_mode)
      for (int f = 0; f < 6; f++) { if (f) spec += " "; spec += long_atoms[f][rng() % 8]; }
    else if (rng() % 10 == 0) spec = "@every " + std::to_string(1 + rng() % 7200) + "s";
    else for (int f = 0; f < 6; f++) { if (f) spec += " "; spec += atoms[f][rng() % 16]; }
    or_sched s;
    char err[256];
    if (or_parse(OR_OPT_DEFAULT, spec.c_str(), spec.size(), &s, err, sizeof err)) continue;
    scheds.push_back(s);
    names.push_back(spec);
  }
  // horizons: around each zone transition in 2025-2027 and plain ones
  ZoneTable tt = build_table(zr, 1735689600, 1830297600);
  std::vector<std::pair<int64_t, int64_t>> hz = {{1767571200, 1767571200 + 86400},
                                                 {1767571200 - 77, 1767571200 + 40 * 86400}};
  for (size_t i = 1; i < tt.when.size() && i < 5; i++) {
    hz.push_back({tt.when[i] - 43217, tt.when[i] + 43200});
    hz.push_back({tt.when[i] - 3 * 86400, tt.when[i] + 4 * 86400});
  }
  if (near_mode) {
    hz.clear();
    ZoneTable nt = build_table(zr, 1293840000, 1830297600);
    const size_t n = nt.when.size() > 1 ? nt.when.size() - 1 : 0;
    const int64_t offs[] = {-7201, -3600, -2, -1, 0, 1, 2, 1799, 3599, 3600, 3601, 5400, 18000,
                            18001, 72000, 90000, 3 * 86400, 35 * 86400 + 7};
    std::vector<size_t> pick;
    for (size_t k = 0; k < 6 && k < n; k++) pick.push_back(1 + (n > 6 ? k * (n - 1) / 5 : k));
    size_t big = 0;  // and the largest jump (Pacific/Apia's skipped 2011-12-30)
    for (size_t i = 1; i <= n; i++)
      if (!big || std::abs(nt.off[i] - nt.off[i - 1]) > std::abs(nt.off[big] - nt.off[big - 1])) big = i;
    if (big && std::find(pick.begin(), pick.end(), big) == pick.end()) pick.push_back(big);
    for (size_t i : pick)
      for (int64_t o : offs) hz.push_back({nt.when[i] + o, nt.when[i] + o + 30 * 3600});
  }
  // clean mode: every transition of 2011-2027 that the plan treats as clean
  // (no WALK window, no exact walk from T0): horizons of 30 h from T0 at
  // offsets around it, and 24 h from T0 = tau + k days (k = 1..39, the days a
  // walk from T0 could reset back across it)
  const bool clean_mode = argc > 4 && std::string(argv[4]) == "clean";
  int clean_plans = 0;
  if (clean_mode) {
    hz.clear();
    ZoneTable nt = build_table(zr, 1293840000, 1830297600);
    const int64_t offs[] = {-86400, -7201, -3601, -3600, -3599, -2, -1, 0, 1, 2, 1799, 3599, 3600, 3601, 7199, 7200};
    for (size_t i = 1; i < nt.when.size(); i++) {
      if (!clean_transition(nt, i)) continue;
      for (int64_t o : offs) hz.push_back({nt.when[i] + o, nt.when[i] + o + 30 * 3600});
      for (int k = 1; k < 40; k += (i % 3) + 1) hz.push_back({nt.when[i] + k * 86400 + 3 * k * 877, nt.when[i] + k * 86400 + 3 * k * 877 + 86400});
    }
  }
  if (long_mode)  // three years from 2026; 2095-06-01 .. 2106-06-01 (Feb 29 gap over 2100)
    hz = {{1767571200 - 77, 1767571200 + 1096 * 86400}, {3957984000, 3957984000 + 4018 * 86400}};
  int bad = 0;
  long long total = 0;
  for (auto [t0, t1] : hz) {
    Plan plan = build_plan(zr, t0, t1);
    ZoneView zv{plan.table.when.data(), plan.table.off.data(), int32_t(plan.table.when.size())};
    int G = int(plan.segs.size());
    if (clean_mode && plan.flags == 0) clean_plans++;
    for (size_t r = 0; r < scheds.size(); r++) {
      DSpec d = pack(scheds[r]);
      std::vector<int64_t> anc(G);
      std::vector<int32_t> cnt(G);
      std::vector<uint32_t> dm(G);
      std::vector<int64_t> got;
      bool ok = G == 0 || count_rule(d, zv, plan.segs.data(), G, plan.dtab.data(), t0, t1, plan.flags, anc.data(), cnt.data(), dm.data());
      if (G > 0 && plan.flags == 0) {  // the kernel's no-walk specialisation must agree exactly
        std::vector<int64_t> anc2(G);
        std::vector<int32_t> cnt2(G);
        std::vector<uint32_t> dm2(G);
        const bool ok2 = count_rule<false>(d, zv, plan.segs.data(), G, plan.dtab.data(), t0, t1, plan.flags,
                                           anc2.data(), cnt2.data(), dm2.data());
        if (ok2 != ok || anc2 != anc || cnt2 != cnt || dm2 != dm) {
          if (bad++ < 10) printf("NOWALK mismatch %s\n", names[r].c_str());
        }
      }
      for (int s = 0; s < G && ok; s++) {
        const Segment& sg = plan.segs[s];
        if (d.kind == KIND_EVERY) {
          for (int k = 0; k < cnt[s]; k++) got.push_back(anc[s] + int64_t(k + 1) * int64_t(d.sec));
        } else if (!run_is_walked(sg, dm[s])) {
          CFRule c = cf_rule(d);
          // mimic the writer: seek at a random start, then step
          int k0 = cnt[s] ? int(rng() % cnt[s]) : 0;
          std::vector<int64_t> part(cnt[s]);
          for (int k = 0; k < k0; k++) part[k] = cf_value(sg, cf_seek(c, sg, dm[s], anc[s], k));
          if (cnt[s]) {
            CFIter it = cf_seek(c, sg, dm[s], anc[s], k0);
            for (int k = k0; k < cnt[s]; k++) {
              if (k > k0) cf_next(c, dm[s], it);
              part[k] = cf_value(sg, it);
            }
          }
          got.insert(got.end(), part.begin(), part.end());
        } else {
          int64_t t = anc[s];
          for (int k = 0; k < cnt[s]; k++) { t = next_exact(d, zv, t, t1); got.push_back(t); }
        }
      }
      int64_t n = or_expand(&scheds[r], t0, t1, ol, nullptr, 0);
      if (n < 0) { if (ok) { if (bad++ < 10) printf("NOPROGRESS mismatch %s (%lld,%lld] got %zu fires, G=%d\n", names[r].c_str(), (long long)t0, (long long)t1, got.size(), G); } continue; }
      std::vector<int64_t> exp(n);
      or_expand(&scheds[r], t0, t1, ol, exp.data(), n);
      total += n;
      if (got != exp && bad++ < 10) {
        size_t i = 0;
        while (i < got.size() && i < exp.size() && got[i] == exp[i]) i++;
        printf("MISMATCH %s [%s] (%lld,%lld] n=%zu/%zu first diff idx %zu: %lld vs %lld (G=%d)\n", zone,
               names[r].c_str(), (long long)t0, (long long)t1, got.size(), exp.size(), i,
               (long long)(i < got.size() ? got[i] : -1), (long long)(i < exp.size() ? exp[i] : -1), G);
      }
    }
  }
  if (clean_mode) printf("%s: %d of %zu horizons planned without any exact walk\n", zone, clean_plans, hz.size());
  printf("%s: %d mismatches, %lld events checked\n", zone, bad, total);
  return bad ? 1 : 0;
}
