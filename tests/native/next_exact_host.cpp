// Host-side check of cg_time.h's next_exact (the device Next walk, compiled
// for the CPU) against the oracle's literal restatement.  Test infrastructure.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../cronsun_amd/csrc/cg_time.h"
#include "../../cronsun_amd/csrc/cg_zone.h"
#include "../../oracle/cron_oracle.h"

using namespace cg;

static std::vector<uint8_t> slurp(const char* p) {
  FILE* f = fopen(p, "rb");
  if (!f) { perror(p); exit(2); }
  std::vector<uint8_t> d;
  uint8_t b[4096];
  size_t n;
  while ((n = fread(b, 1, sizeof b, f)) > 0) d.insert(d.end(), b, b + n);
  fclose(f);
  return d;
}

static const char* atoms[6][12] = {
    {"*", "0", "5", "*/7", "15/35", "10-40/3", "7,30,45", "59", "0/15", "3-3", "*/1", "58-59"},
    {"*", "0", "30", "*/5", "20-35/15", "1,31,59", "5-7/2", "*/59", "10-12", "0", "0", "59"},
    {"*", "0", "9", "23", "*/2", "1/2", "9-17", "22,23,0", "2", "1", "3", "0-23/5"},
    {"*", "?", "1", "15", "31", "29", "30", "1,15", "*/2", "9-20", "28-31", "5/7"},
    {"*", "?", "1", "2", "Feb", "Jan,Jul", "Apr-Oct", "*/3", "Mar", "Nov", "Dec", "*"},
    {"*", "?", "0", "1-5", "Mon", "Sun", "mon/2", "Sat,Sun", "*/2", "3", "fri-sat", "*"}};

int main(int argc, char** argv) {
  const char* zone = argc > 1 ? argv[1] : "UTC";
  int n = argc > 2 ? atoi(argv[2]) : 20000;
  std::string base = "tests/golden/zoneinfo/";
  ZoneRules zr;
  or_loc* ol = nullptr;
  if (!strcmp(zone, "UTC")) {
    zr = zone_utc();
    or_loc_utc(&ol);
  } else {
    auto d = slurp((base + zone).c_str());
    std::string e;
    if (!zone_from_tzif(d.data(), d.size(), &zr, &e)) { printf("bad zone %s\n", e.c_str()); return 2; }
    or_loc_from_tzif(d.data(), d.size(), &ol);
  }
  std::mt19937_64 rng(12345);
  int64_t lo = 946684800, hi = 2208988800;
  ZoneTable tab = build_table(zr, lo - 64 * 86400LL, hi + (6 * 366 + 64) * 86400LL);
  ZoneView zv{tab.when.data(), tab.off.data(), int32_t(tab.when.size())};
  int bad = 0;
  for (int i = 0; i < n; i++) {
    std::string spec;
    int nf = (rng() % 5 == 0) ? 5 : 6;
    for (int f = 0; f < nf; f++) { if (f) spec += " "; spec += atoms[f][rng() % 12]; }
    or_sched s;
    char err[256];
    if (or_parse(OR_OPT_DEFAULT, spec.c_str(), spec.size(), &s, err, sizeof err)) continue;
    int64_t t = lo + int64_t(rng() % uint64_t(hi - lo));
    if (tab.when.size() > 1 && rng() % 3 == 0) {
      int64_t w = tab.when[1 + rng() % (tab.when.size() - 1)];
      if (w > lo && w < hi) t = w + int64_t(rng() % 172800) - 86400;
    }
    DSpec d{};
    d.sec = s.spec.second & 0x0FFFFFFFFFFFFFFFull;
    d.min = s.spec.minute & 0x0FFFFFFFFFFFFFFFull;
    d.hour = uint32_t(s.spec.hour & 0xFFFFFF);
    d.dom = uint32_t(s.spec.dom & 0xFFFFFFFEu) | uint32_t(s.spec.dom >> 63);
    d.mondow = uint32_t(s.spec.month & 0x1FFE) | (uint32_t(s.spec.dow & 0x7F) << 16) |
               (uint32_t(s.spec.dow >> 63) << 23);
    int64_t got = next_exact(d, zv, t, INT64_MAX);
    int64_t exp = or_spec_next(&s.spec, t, 0, ol);
    if (got != exp && bad++ < 10) printf("MISMATCH %s [%s] t=%lld got=%lld exp=%lld\n", zone, spec.c_str(), (long long)t, (long long)got, (long long)exp);
  }
  printf("%s: %d/%d mismatches\n", zone, bad, n);
  return bad ? 1 : 0;
}
