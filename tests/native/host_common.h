// Shared scaffolding of the host-side checks (test infrastructure): TZif
// loading into both the product's ZoneRules and the oracle's Location, and
// packing an oracle schedule into the product's 32-byte DSpec.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../cronsun_amd/csrc/cg_time.h"
#include "../../cronsun_amd/csrc/cg_zone.h"
#include "../../oracle/cron_oracle.h"

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

// zone name -> (product rules, oracle location); tests/golden/zoneinfo/<name>
static void load_zone(const char* zone, cg::ZoneRules* zr, or_loc** ol) {
  if (!strcmp(zone, "UTC")) { *zr = cg::zone_utc(); or_loc_utc(ol); return; }
  auto d = slurp((std::string("tests/golden/zoneinfo/") + zone).c_str());
  std::string e;
  cg::zone_from_tzif(d.data(), d.size(), zr, &e);
  or_loc_from_tzif(d.data(), d.size(), ol);
}

static cg::DSpec pack(const or_sched& s) {
  cg::DSpec d{};
  if (s.kind == 1) { d.kind = cg::KIND_EVERY; d.sec = uint64_t(s.delay_ns / 1000000000LL); return d; }
  d.sec = s.spec.second & 0x0FFFFFFFFFFFFFFFull;
  d.min = s.spec.minute & 0x0FFFFFFFFFFFFFFFull;
  d.hour = uint32_t(s.spec.hour & 0xFFFFFF);
  d.dom = uint32_t(s.spec.dom & 0xFFFFFFFEu) | uint32_t(s.spec.dom >> 63);
  d.mondow = uint32_t(s.spec.month & 0x1FFE) | (uint32_t(s.spec.dow & 0x7F) << 16) |
             (uint32_t(s.spec.dow >> 63) << 23);
  return d;
}
