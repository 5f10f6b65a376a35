// cg_zone.h -- host-side zone rules (Go *time.Location restated) and the
// per-batch breakpoint table / segment plan shipped to the device.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace cg {

// A Location as Go's time package models it (zoneinfo.go): zones, transitions
// and the optional POSIX TZ footer ("extend") applied after the last
// transition.  has_zones == false is time.UTC.
struct ZoneRules {
  bool has_zones = false;
  std::vector<int32_t> zone_off;
  std::vector<uint8_t> zone_dst;
  std::vector<int64_t> tx_when;
  std::vector<uint8_t> tx_index;
  std::string extend;
  std::string name;

  // Location.lookup(sec): offset, with Go's reported [start, end).
  int32_t lookup(int64_t sec, int64_t* start, int64_t* end) const;
  int32_t offset(int64_t sec) const {
    int64_t s, e;
    return lookup(sec, &s, &e);
  }
  // Instants in (lo, hi] where lookup() may change value: transitions,
  // footer rule instants and footer year boundaries.
  void breakpoints(int64_t lo, int64_t hi, std::vector<int64_t>* out) const;
};

// LoadLocationFromTZData.  Returns false on malformed data.
bool zone_from_tzif(const uint8_t* data, size_t len, ZoneRules* out, std::string* err);
ZoneRules zone_fixed(int32_t offset);  // time.FixedZone
ZoneRules zone_utc();                  // time.UTC

// Flat offset table covering [lo, hi]: when[0] = INT64_MIN, strictly
// increasing, consecutive offsets differ.
struct ZoneTable {
  std::vector<int64_t> when;
  std::vector<int32_t> off;
  int32_t max_abs_off = 0;
};
ZoneTable build_table(const ZoneRules& z, int64_t lo, int64_t hi);

// Expansion plan for (T0, T1]: closed-form (CF) spans of one offset, on which
// every Date call of the Go walk returns its fixed-offset instant, and WALK
// spans around zone transitions (at least the transition instant itself, plus
// the overlap Go resolves to the other pass) where Next is emulated step by
// step.  margin = A: transitions closer than 2A share one WALK span.
struct Segment {
  int64_t a, b;    // (a, b] in UTC seconds
  int64_t base;    // UTC instant of local midnight of day0 (CF only)
  int64_t day0;    // first local day number (CF only)
  int32_t off;     // constant offset (CF only)
  int32_t kind;    // 0 = CF, 1 = WALK
  int32_t ndays;   // local days spanned (CF only, <= 31)
  int32_t dt_off;  // offset into the day table (CF only)
};
constexpr uint32_t kPlanT0Walk = 1;     // Next(T0) by the exact walk
constexpr uint32_t kPlanFinalWalk = 2;  // the Next past T1 walked to its end
constexpr uint32_t kPlanWalkSegs = 4;   // the plan has WALK segments
struct Plan {
  std::vector<Segment> segs;
  std::vector<uint32_t> dtab;  // per CF local day: month | dom << 4 | dow << 9
  ZoneTable table;
  int64_t margin = 0;
  uint32_t flags = 0;  // kPlanT0Walk | kPlanFinalWalk | kPlanWalkSegs
};
Plan build_plan(const ZoneRules& z, int64_t t0, int64_t t1);
// breakpoint i (>= 1) of t is a clean transition: no WALK window, no exact
// walk from T0 after it (cg_zone.cpp)
bool clean_transition(const ZoneTable& t, size_t i);

}  // namespace cg
