// cg_zone.cpp -- Go time.Location semantics on the host, and the per-batch
// breakpoint table + expansion plan the kernels consume.
//
// Go's Location.lookup (time/zoneinfo.go) is: the offset of the last
// transition at or before sec (the "first zone" rule before any transition),
// and -- for instants at or after the last transition -- the POSIX TZ footer
// evaluated per UTC year by tzset.  The reference's tests pin this footer
// behaviour: the America/New_York DST vectors in node/cron/spec_test.go:112-148
// fall after the last explicit transition of a slim 2026a TZif.
#include "cg_zone.h"

#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "cg_time.h"

namespace cg {

static const int64_t kAlpha = INT64_MIN;
static const int64_t kOmega = INT64_MAX;

namespace {

uint32_t rd32(const uint8_t* p) {
  return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
}

// ---- POSIX TZ footer (Go's tzset / tzsetName / tzsetOffset / tzsetRule) ----
struct Rule {
  int kind = 0;  // 0 julian (Jn), 1 day-of-year (n), 2 month-week-day (Mm.w.d)
  int day = 0, week = 0, mon = 0, time = 7200;
};

struct Footer {
  bool ok = false;
  bool has_dst = false;
  int std_off = 0, dst_off = 0;
  Rule start, end;
};

bool ft_name(const char*& s) {
  if (!*s) return false;
  if (*s != '<') {
    int i = 0;
    for (; s[i]; i++) {
      char c = s[i];
      if ((c >= '0' && c <= '9') || c == ',' || c == '-' || c == '+') {
        if (i < 3) return false;
        s += i;
        return true;
      }
    }
    if (i < 3) return false;
    s += i;
    return true;
  }
  const char* close = std::strchr(s, '>');
  if (!close) return false;
  s = close + 1;
  return true;
}

bool ft_num(const char*& s, int lo, int hi, int* out) {
  if (!*s) return false;
  int v = 0, i = 0;
  for (; s[i] >= '0' && s[i] <= '9'; i++) {
    v = v * 10 + (s[i] - '0');
    if (v > hi) return false;
  }
  if (i == 0 && s[0]) return false;
  if (v < lo) return false;
  s += i;
  *out = v;
  return true;
}

bool ft_offset(const char*& s, int* out) {
  if (!*s) return false;
  bool neg = false;
  if (*s == '+') s++;
  else if (*s == '-') { s++; neg = true; }
  int h, m = 0, sec = 0;
  if (!ft_num(s, 0, 24 * 7, &h)) return false;
  int off = h * 3600;
  if (*s == ':') {
    s++;
    if (!ft_num(s, 0, 59, &m)) return false;
    off += m * 60;
    if (*s == ':') {
      s++;
      if (!ft_num(s, 0, 59, &sec)) return false;
      off += sec;
    }
  }
  *out = neg ? -off : off;
  return true;
}

bool ft_rule(const char*& s, Rule* r) {
  if (!*s) return false;
  if (*s == 'J') {
    s++;
    r->kind = 0;
    if (!ft_num(s, 1, 365, &r->day)) return false;
  } else if (*s == 'M') {
    s++;
    r->kind = 2;
    if (!ft_num(s, 1, 12, &r->mon) || *s != '.') return false;
    s++;
    if (!ft_num(s, 1, 5, &r->week) || *s != '.') return false;
    s++;
    if (!ft_num(s, 0, 6, &r->day)) return false;
  } else {
    r->kind = 1;
    if (!ft_num(s, 0, 365, &r->day)) return false;
  }
  r->time = 7200;
  if (*s == '/') {
    s++;
    if (!ft_offset(s, &r->time)) return false;
  }
  return true;
}

Footer parse_footer(const std::string& ext) {
  Footer f;
  const char* s = ext.c_str();
  if (!ft_name(s) || !ft_offset(s, &f.std_off)) return f;
  f.std_off = -f.std_off;
  if (*s == 0 || *s == ',') {
    f.ok = true;
    return f;
  }
  if (!ft_name(s)) return f;
  if (*s == 0 || *s == ',') {
    f.dst_off = f.std_off + 3600;
  } else {
    if (!ft_offset(s, &f.dst_off)) return f;
    f.dst_off = -f.dst_off;
  }
  const char* r = *s ? s : ",M3.2.0,M11.1.0";
  if (*r != ',' && *r != ';') return f;
  r++;
  if (!ft_rule(r, &f.start) || *r != ',') return f;
  r++;
  if (!ft_rule(r, &f.end) || *r != 0) return f;
  f.ok = true;
  f.has_dst = true;
  return f;
}

const int kDaysBefore[13] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334, 365};

// seconds after the start of `year` (UTC) at which rule r takes effect
int64_t rule_time(int32_t year, const Rule& r, int off) {
  int64_t s = 0;
  if (r.kind == 0) {
    s = int64_t(r.day - 1) * 86400;
    if (is_leap(year) && r.day >= 60) s += 86400;
  } else if (r.kind == 1) {
    s = int64_t(r.day) * 86400;
  } else {
    // day of week of the first of the month, then the r.week-th r.day
    int64_t first = days_from_civil(year, r.mon, 1);
    int dow = weekday_of_day(first);
    int d = r.day - dow;
    if (d < 0) d += 7;
    int dim = days_in_month(year, r.mon);
    for (int i = 1; i < r.week; i++) {
      if (d + 7 >= dim) break;
      d += 7;
    }
    d += kDaysBefore[r.mon - 1];
    if (is_leap(year) && r.mon > 2) d++;
    s = int64_t(d) * 86400;
  }
  return s + r.time - off;
}

struct YearRule {
  int64_t abs;          // unix time of Jan 1 00:00 UTC
  int64_t start, end;   // seconds into the year (after the southern flip)
  int32_t std_off, dst_off;
};

YearRule year_rule(const Footer& f, int32_t year) {
  YearRule y;
  y.abs = days_from_civil(year, 1, 1) * 86400;
  y.start = rule_time(year, f.start, f.std_off);
  y.end = rule_time(year, f.end, f.dst_off);
  y.std_off = f.std_off;
  y.dst_off = f.dst_off;
  if (y.end < y.start) {
    std::swap(y.start, y.end);
    std::swap(y.std_off, y.dst_off);
  }
  return y;
}

// tzset(extend, lastTxSec, sec)
int32_t footer_lookup(const Footer& f, int64_t last_tx, int64_t sec, int64_t* start, int64_t* end) {
  if (!f.has_dst) {
    *start = last_tx;
    *end = kOmega;
    return f.std_off;
  }
  int64_t day = floordiv64(sec, 86400);
  int32_t year = civil_from_days(day).y;
  YearRule y = year_rule(f, year);
  int64_t ysec = (day - days_from_civil(year, 1, 1)) * 86400 + sec % 86400;  // Go's truncating %
  if (ysec < y.start) {
    *start = y.abs;
    *end = y.start + y.abs;
    return y.std_off;
  }
  if (ysec >= y.end) {
    *start = y.end + y.abs;
    *end = y.abs + 365 * 86400;
    return y.std_off;
  }
  *start = y.start + y.abs;
  *end = y.end + y.abs;
  return y.dst_off;
}

}  // namespace

int32_t ZoneRules::lookup(int64_t sec, int64_t* start, int64_t* end) const {
  if (!has_zones) {
    *start = kAlpha;
    *end = kOmega;
    return 0;
  }
  const size_t ntx = tx_when.size();
  if (ntx == 0 || sec < tx_when[0]) {
    // lookupFirstZone
    size_t zi = 0;
    bool used = false;
    for (uint8_t i : tx_index) used |= (i == 0);
    if (used) {
      bool found = false;
      if (ntx > 0 && zone_dst[tx_index[0]]) {
        for (int k = int(tx_index[0]) - 1; k >= 0; k--)
          if (!zone_dst[k]) { zi = size_t(k); found = true; break; }
      }
      if (!found) {
        for (size_t k = 0; k < zone_off.size(); k++)
          if (!zone_dst[k]) { zi = k; found = true; break; }
      }
      if (!found) zi = 0;
    }
    *start = kAlpha;
    *end = ntx > 0 ? tx_when[0] : kOmega;
    return zone_off[zi];
  }
  // largest transition at or before sec
  size_t lo = size_t(std::upper_bound(tx_when.begin(), tx_when.end(), sec) - tx_when.begin()) - 1;
  *start = tx_when[lo];
  *end = lo + 1 < ntx ? tx_when[lo + 1] : kOmega;
  int32_t off = zone_off[tx_index[lo]];
  if (lo == ntx - 1 && !extend.empty()) {
    Footer f = parse_footer(extend);
    if (f.ok) return footer_lookup(f, *start, sec, start, end);
  }
  return off;
}

void ZoneRules::breakpoints(int64_t lo, int64_t hi, std::vector<int64_t>* out) const {
  if (!has_zones) return;
  for (int64_t w : tx_when)
    if (w > lo && w <= hi) out->push_back(w);
  if (extend.empty() || tx_when.empty()) return;
  Footer f = parse_footer(extend);
  if (!f.ok || !f.has_dst) return;
  int64_t from = std::max(lo, tx_when.back());
  if (from > hi) return;
  int32_t y0 = civil_from_days(floordiv64(from, 86400)).y - 1;
  int32_t y1 = civil_from_days(floordiv64(hi, 86400)).y + 1;
  for (int32_t y = y0; y <= y1; y++) {
    YearRule r = year_rule(f, y);
    int64_t pts[3] = {r.abs, r.abs + r.start, r.abs + r.end};
    for (int64_t p : pts)
      if (p > lo && p <= hi) out->push_back(p);
  }
}

bool zone_from_tzif(const uint8_t* d, size_t len, ZoneRules* out, std::string* err) {
  auto fail = [&](const char* m) {
    if (err) *err = m;
    return false;
  };
  if (len < 44 || std::memcmp(d, "TZif", 4) != 0) return fail("not a TZif file");
  int version = d[4] == 0 ? 1 : d[4] - '0';
  size_t p = 20;
  uint32_t n[6];
  for (int i = 0; i < 6; i++) n[i] = rd32(d + p + 4 * i);
  p += 24;
  enum { UTCLOCAL, STDWALL, LEAP, TIME, ZONE, CHAR };
  bool is64 = false;
  if (version > 1) {
    p += size_t(n[TIME]) * 5 + size_t(n[ZONE]) * 6 + n[CHAR] + size_t(n[LEAP]) * 8 + n[STDWALL] +
         n[UTCLOCAL];
    if (p + 44 > len || std::memcmp(d + p, "TZif", 4) != 0) return fail("bad TZif v2 header");
    p += 20;
    for (int i = 0; i < 6; i++) n[i] = rd32(d + p + 4 * i);
    p += 24;
    is64 = true;
  }
  size_t tsz = is64 ? 8 : 4;
  size_t body = size_t(n[TIME]) * (tsz + 1) + size_t(n[ZONE]) * 6 + n[CHAR] +
                size_t(n[LEAP]) * (tsz + 4) + n[STDWALL] + n[UTCLOCAL];
  if (p + body > len) return fail("truncated TZif");
  if (n[ZONE] == 0 || n[ZONE] > 255) return fail("bad zone count");
  ZoneRules z;
  z.has_zones = true;
  const uint8_t* tt = d + p;
  const uint8_t* ti = tt + size_t(n[TIME]) * tsz;
  const uint8_t* zd = ti + n[TIME];
  for (uint32_t i = 0; i < n[ZONE]; i++) {
    z.zone_off.push_back(int32_t(rd32(zd + 6 * i)));
    z.zone_dst.push_back(zd[6 * i + 4] != 0);
  }
  for (uint32_t i = 0; i < n[TIME]; i++) {
    int64_t w = is64 ? int64_t((uint64_t(rd32(tt + 8 * i)) << 32) | rd32(tt + 8 * i + 4))
                     : int64_t(int32_t(rd32(tt + 4 * i)));
    if (ti[i] >= n[ZONE]) return fail("bad zone index");
    z.tx_when.push_back(w);
    z.tx_index.push_back(ti[i]);
  }
  if (z.tx_when.empty()) {  // fake transition covering all time
    z.tx_when.push_back(kAlpha);
    z.tx_index.push_back(0);
  }
  const uint8_t* rest = d + p + body;
  size_t rl = len - size_t(rest - d);
  if (version > 1 && rl > 2 && rest[0] == '\n' && rest[rl - 1] == '\n')
    z.extend.assign(reinterpret_cast<const char*>(rest + 1), rl - 2);
  *out = std::move(z);
  return true;
}

ZoneRules zone_fixed(int32_t offset) {
  ZoneRules z;
  z.has_zones = true;
  z.zone_off = {offset};
  z.zone_dst = {0};
  z.tx_when = {kAlpha};
  z.tx_index = {0};
  return z;
}

ZoneRules zone_utc() { return ZoneRules(); }

ZoneTable build_table(const ZoneRules& z, int64_t lo, int64_t hi) {
  std::vector<int64_t> pts;
  z.breakpoints(lo, hi, &pts);
  std::sort(pts.begin(), pts.end());
  pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
  ZoneTable t;
  t.when.push_back(INT64_MIN);
  t.off.push_back(z.offset(lo));
  for (int64_t p : pts) {
    int32_t o = z.offset(p);
    if (o == t.off.back()) continue;
    t.when.push_back(p);
    t.off.push_back(o);
  }
  for (int32_t o : t.off) t.max_abs_off = std::max(t.max_abs_off, o < 0 ? -o : o);
  return t;
}

// Is breakpoint i of table t a "clean" transition -- one the Go walk crosses
// exactly as the closed form in the local time of each instant does, so it
// needs no WALK window and no exact walk from T0 (clean
// transitions)?  Conditions: a one-hour shift (d = o2 - o1 = +-3600) between
// whole-minute offsets, at a local hour start, whose skipped or repeated local
// hour lies at least one hour away from local midnight on both sides, with no
// other breakpoint within three days.  Then (1) every Date call of the walk
// (midnights, month starts, hour starts) either resolves to its own instant or
// is an hour-level reset inside a mismatching hour whose other pass mismatches
// too; (2) the hour, minute and second walks step across tau without missing a
// wrap (no midnight nearby, minutes continuous); (3) Truncate(Minute) is wall
// truncation.  America/New_York's, Europe's and Australia's DST changes are
// clean; Havana's (midnight), Lord_Howe's (30 min), Chatham's (02:45) and
// Apia's (a day) are not.
static int64_t floormod_i64(int64_t a, int64_t b) { return a - floordiv64(a, b) * b; }

bool clean_transition(const ZoneTable& t, size_t i) {
  const int64_t kDay = 86400;
  const int64_t tau = t.when[i];
  const int64_t o1 = t.off[i - 1], o2 = t.off[i], d = o2 - o1;
  if (d != 3600 && d != -3600) return false;
  if (o1 % 60 != 0 || o2 % 60 != 0) return false;
  if (floormod_i64(tau + o1, 3600) != 0) return false;
  const int64_t lo = std::min(tau + o1, tau + o2);  // the skipped / repeated local hour [lo, lo + 3600)
  const int64_t sod = floormod_i64(lo, kDay);
  if (sod < 3600 || sod + 3600 > kDay - 3600) return false;
  if (i > 1 && tau - t.when[i - 1] < 3 * kDay) return false;
  if (i + 1 < t.when.size() && t.when[i + 1] - tau < 3 * kDay) return false;
  return true;
}

Plan build_plan(const ZoneRules& z, int64_t t0, int64_t t1) {
  Plan plan;
  const int64_t kDay = 86400;
  // the table reaches six years past T1: the reference's last Next (the one
  // past T1) may walk up to five years on (spec.go:70-76)
  plan.table = build_table(z, t0 - 64 * kDay, t1 + (6 * 366 + 64) * kDay);
  if (t1 <= t0) return plan;
  std::vector<char> clean(plan.table.when.size(), 0);
  for (size_t i = 1; i < plan.table.when.size(); i++) clean[i] = clean_transition(plan.table, i);
  for (size_t i = 1; i < plan.table.when.size(); i++) {
    const int64_t tau = plan.table.when[i];
    // the walk from T0 may reset back across a transition of the last 40 days
    // (harmless across a clean one: its resets land on midnights, month
    // starts and hour starts Date resolves exactly, or inside a mismatching hour)
    if (tau > t0 - 40 * kDay && tau <= t0 && !clean[i]) plan.flags |= kPlanT0Walk;
    // a skipped local day (e.g. Pacific/Apia 2011-12-30): AddDate(0,0,1) can
    // stall there, so the last Next must be walked to its end
    if (tau > t0 && plan.table.off[i] - plan.table.off[i - 1] >= kDay) plan.flags |= kPlanFinalWalk;
  }
  // WALK windows.  Between two consecutive fires e < u the Go
  // walk visits only instants in [e + 1, u]; it reads fields there (exact when
  // the offset is the segment's) and calls Date for civil times whose
  // fixed-offset instant X lies there.  With a single transition tau (o1 ->
  // o2, d = o2 - o1) within A = max|off| + max|d| of X, Date(X + o(X)) = X
  // except on the overlap of a backward transition (d < 0): after tau,
  // [tau, tau + min(-o2, -d)) when o2 < 0 (Go resolves those civil times to
  // the first pass); before tau, [tau - min(o1, -d), tau) when o1 > 0.  So a CF
  // segment may run up to tau - 1 and resume after that bad set: the window
  // around tau is (tau - 1 - before, tau + after], and the walk that crosses it
  // (from the last fire before) is the exact walk.  Transitions closer than
  // 2A share one window (a CF instant must see at most one of them).
  // The overlap's bad set matters only where it holds a local hour start (see
  // below): America/New_York's 01:00-02:00 second pass holds none past tau
  // itself, Pacific/Chatham's 02:45-03:45 first pass holds 03:00.
  int32_t max_d = 0;
  for (size_t i = 2; i < plan.table.when.size(); i++)
    max_d = std::max(max_d, std::abs(plan.table.off[i] - plan.table.off[i - 1]));
  const int64_t A = int64_t(plan.table.max_abs_off) + max_d;
  plan.margin = A;
  std::vector<std::pair<int64_t, int64_t>> win;  // (lo, hi] WALK windows
  int64_t prev_tau = INT64_MIN;
  std::vector<int64_t> cuts;  // clean transitions: a CF span is only cut there, (.., tau - 1] | (tau - 1, ..]
  for (size_t i = 1; i < plan.table.when.size(); i++) {
    const int64_t tau = plan.table.when[i];
    if (clean[i]) {
      if (tau - 1 > t0 && tau - 1 < t1) cuts.push_back(tau - 1);
      continue;
    }
    const int64_t o1 = plan.table.off[i - 1], o2 = plan.table.off[i], d = o2 - o1;
    int64_t before = (d < 0 && o1 > 0) ? std::min(o1, -d) : 0;
    int64_t after = (d < 0 && o2 < 0) ? std::min(-o2, -d) : 0;
    // Between two fires of a segment, Go's walk calls Date only for local
    // hour starts (its resets land on the instant after the previous fire,
    // which starts the unit that changed; AddDate steps go from midnights to
    // midnights or month starts).  A bad set with no local hour start on the
    // segment's side of the +-2 s margin is never reached: no window for it.
    auto hour_start_at_or_after = [](int64_t x, int64_t o) {  // first instant >= x with local h:00:00
      return floordiv64(x + o + 3599, 3600) * 3600 - o;
    };
    if (after > 0 && hour_start_at_or_after(tau + 3, o2) >= tau + after) after = 0;
    if (before > 0 && floordiv64(tau - 3 + o1, 3600) * 3600 - o1 < tau - before) before = 0;
    int64_t lo = tau - 1 - before - 2, hi = tau + after + 2;  // +-2 s: no off-by-one risk
    if (prev_tau != INT64_MIN && tau - prev_tau <= 2 * A + 8) lo = std::min(lo, prev_tau);  // one window
    prev_tau = tau;
    lo = std::max(lo, t0);
    hi = std::min(hi, t1);
    if (hi <= lo) continue;
    if (!win.empty() && lo <= win.back().second) win.back().second = std::max(win.back().second, hi);
    else win.push_back({lo, hi});
  }
  auto add_cf = [&](int64_t a, int64_t b) {
    const int64_t kChunk = 30 * kDay;
    for (int64_t x = a, xe; x < b; x = xe) {
      xe = std::min(b, x + kChunk);
      for (int64_t cut : cuts)
        if (cut > x && cut < xe) { xe = cut; break; }  // cuts ascend
      Segment s;
      s.a = x;
      s.b = xe;
      s.kind = 0;
      s.off = plan.table.off[0];
      ZoneView zv{plan.table.when.data(), plan.table.off.data(), int32_t(plan.table.when.size())};
      s.off = zone_offset(zv, s.a + 1);
      s.day0 = floordiv64(s.a + 1 + s.off, kDay);
      int64_t last = floordiv64(s.b + s.off, kDay);
      s.ndays = int32_t(last - s.day0 + 1);
      s.base = s.day0 * kDay - s.off;
      s.dt_off = int32_t(plan.dtab.size());
      for (int64_t dd = s.day0; dd <= last; dd++) {
        Civil c = civil_from_days(dd);
        plan.dtab.push_back(uint32_t(c.m) | (uint32_t(c.d) << 4) | (uint32_t(weekday_of_day(dd)) << 9));
      }
      plan.segs.push_back(s);
    }
  };
  int64_t cur = t0;
  for (auto& w : win) {
    if (w.first > cur) add_cf(cur, w.first);
    Segment s{};
    s.a = w.first;
    s.b = w.second;
    s.kind = 1;
    plan.segs.push_back(s);
    cur = w.second;
  }
  if (cur < t1) add_cf(cur, t1);
  for (const Segment& sg : plan.segs)
    if (sg.kind != 0) plan.flags |= kPlanWalkSegs;
  return plan;
}

}  // namespace cg
