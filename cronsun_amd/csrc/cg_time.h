// cg_time.h -- Go `time` arithmetic used by node/cron's Next, as inline
// host+device functions over a flat zone-offset table.
//
// The reference evaluates SpecSchedule.Next (node/cron/spec.go:55-145) with
// Go's time.Time accessors, time.Date, AddDate, Add and Truncate.  Here a
// Location is reduced, per batch, to a sorted table of (utc_instant, offset)
// breakpoints built on the host from the TZif data + POSIX footer
// (cg_zone.cpp), which reproduces Location.lookup's offset function over the
// batch's time range.  With off(u) the offset in force at UTC instant u:
//
//   fields(t)   = civil(t + off(t))                      (Year/Month/Day/...)
//   Date(L)     = L - off(L - off(L))                    (time.Date, L = local
//                 seconds; equals Go's lookup/re-lookup rule, zoneinfo.go)
//   AddDate     = Date(fields + delta)                   (keeps wall clock)
//   Add(d)      = t + d                                  (absolute)
//   Truncate(m) = t - floormod(t, 60)                    (absolute, since year 1)
#pragma once
#include <stdint.h>

#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define CG_HD __host__ __device__ __forceinline__
#else
#define CG_HD static inline
#endif

#define CG_ZERO_TIME (-62135596800LL)  // Go time.Time{}.Unix()
#define CG_BEYOND INT64_MAX            // "next fire is past the bound"
// Go's Next never returns: AddDate(0,0,1) does not advance across a skipped
// local day (e.g. Pacific/Apia 2011-12-30), so spec.go:96-106 spins forever.
#define CG_NO_PROGRESS (INT64_MIN + 1)
#define CG_SECS_PER_DAY 86400LL

namespace cg {

CG_HD int64_t floordiv64(int64_t a, int64_t b) {
  int64_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
  return q;
}

CG_HD int32_t floordiv32(int32_t a, int32_t b) {
  int32_t q = a / b;
  if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
  return q;
}

// days since 1970-01-01 of y-m-d (m 1..12); Hinnant's algorithm.
CG_HD int64_t days_from_civil(int64_t y, int32_t m, int32_t d) {
  y -= m <= 2;
  int64_t era = floordiv64(y, 400);
  int32_t yoe = (int32_t)(y - era * 400);
  int32_t mp = (m + 9) % 12;
  int32_t doy = (153 * mp + 2) / 5 + d - 1;
  int32_t doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
  return era * 146097 + doe - 719468;
}

struct Civil {
  int32_t y, m, d;
};

// civil date of a unix day number (|z| small enough for int32 years).
CG_HD Civil civil_from_days(int64_t z64) {
  z64 += 719468;
  int64_t era = floordiv64(z64, 146097);
  int32_t doe = (int32_t)(z64 - era * 146097);
  int32_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  int32_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  int32_t mp = (5 * doy + 2) / 153;
  int32_t d = doy - (153 * mp + 2) / 5 + 1;
  int32_t m = mp < 10 ? mp + 3 : mp - 9;
  Civil c;
  c.y = (int32_t)(yoe + era * 400) + (m <= 2);
  c.m = m;
  c.d = d;
  return c;
}

CG_HD bool is_leap(int32_t y) { return y % 4 == 0 && (y % 100 != 0 || y % 400 == 0); }

CG_HD int32_t days_in_month(int32_t y, int32_t m) {
  if (m == 2) return is_leap(y) ? 29 : 28;
  return (m == 4 || m == 6 || m == 9 || m == 11) ? 30 : 31;
}

// weekday of a unix day number (Sunday = 0); 1970-01-01 was a Thursday.
CG_HD int32_t weekday_of_day(int64_t day) {
  int32_t w = (int32_t)(day % 7);
  w = (w + 4) % 7;
  if (w < 0) w += 7;
  return w;
}

// ---- zone table: sorted breakpoints, when[0] == INT64_MIN ----
struct ZoneView {
  const int64_t* when;
  const int32_t* off;
  int32_t n;
};

// offset in force at instant u, plus the next breakpoint after u
CG_HD int32_t zone_lookup(const ZoneView& z, int64_t u, int64_t* next_change) {
  int32_t lo = 0, hi = z.n;  // invariant: when[lo] <= u < when[hi] (when[n] = +inf)
  while (hi - lo > 1) {
    int32_t mid = (lo + hi) >> 1;
    if (z.when[mid] <= u) lo = mid;
    else hi = mid;
  }
  if (next_change) *next_change = hi < z.n ? z.when[hi] : INT64_MAX;
  return z.off[lo];
}

CG_HD int32_t zone_offset(const ZoneView& z, int64_t u) { return zone_lookup(z, u, nullptr); }

// time.Date(y, mo, d, h, mi, s, 0, loc) with Go's normalisation; returns unix
// seconds.  Month overflow carries into the year; the other fields are linear.
CG_HD int64_t go_date(const ZoneView& z, int64_t y, int64_t mo, int64_t d, int64_t h,
                      int64_t mi, int64_t s) {
  int64_t m0 = mo - 1;
  int64_t carry = floordiv64(m0, 12);
  y += carry;
  m0 -= carry * 12;
  int64_t local = days_from_civil(y, (int32_t)(m0 + 1), 1) * CG_SECS_PER_DAY +
                  (d - 1) * CG_SECS_PER_DAY + h * 3600 + mi * 60 + s;
  int32_t o1 = zone_offset(z, local);
  int32_t o2 = zone_offset(z, local - o1);
  return local - o2;
}

struct Fields {
  int64_t day;      // local unix day number
  int32_t tod;      // local second of day
  int32_t y, mo, d, h, mi, s, wd;
  int32_t off;      // offset in force
  int64_t next_change;  // next zone breakpoint after t
};

CG_HD Fields go_fields(const ZoneView& z, int64_t t) {
  Fields f;
  f.off = zone_lookup(z, t, &f.next_change);
  int64_t local = t + f.off;
  f.day = floordiv64(local, CG_SECS_PER_DAY);
  f.tod = (int32_t)(local - f.day * CG_SECS_PER_DAY);
  Civil c = civil_from_days(f.day);
  f.y = c.y;
  f.mo = c.m;
  f.d = c.d;
  f.h = f.tod / 3600;
  f.mi = (f.tod / 60) % 60;
  f.s = f.tod % 60;
  f.wd = weekday_of_day(f.day);
  return f;
}

// ---- packed spec (32 B per rule in HBM) ----
// sec/min: 60-bit masks.  hour: bits 0..23.  dom: bits 1..31, bit 0 = dom
// star.  mondow: month bits 1..12, dow bits 16..22, dow star bit 23.
// kind 1 (@every): sec holds the delay in whole seconds.
struct alignas(16) DSpec {
  uint64_t sec;
  uint64_t min;
  uint32_t hour;
  uint32_t dom;
  uint32_t mondow;
  uint32_t kind;
};

enum { KIND_SPEC = 0, KIND_EVERY = 1 };

CG_HD bool dom_star(const DSpec& s) { return s.dom & 1u; }
CG_HD bool dow_star(const DSpec& s) { return (s.mondow >> 23) & 1u; }
CG_HD bool month_ok(const DSpec& s, int32_t mo) { return (s.mondow >> mo) & 1u; }

// dayMatches, node/cron/spec.go:149-158
CG_HD bool day_matches(const DSpec& s, int32_t dom, int32_t dow) {
  bool dm = (s.dom >> dom) & 1u;
  bool wm = (s.mondow >> (16 + dow)) & 1u;
  if (dom_star(s) || dow_star(s)) return dm && wm;
  return dm || wm;
}

// lowest set bit of m strictly above position p (p may be -1); 64 if none
CG_HD int32_t next_bit64(uint64_t m, int32_t p) {
  uint64_t r = (p >= 63) ? 0 : (m & (~0ULL << (p + 1)));
  return r ? __builtin_ctzll(r) : 64;
}
CG_HD int32_t next_bit32(uint32_t m, int32_t p) {
  uint32_t r = (p >= 31) ? 0u : (m & (~0u << (p + 1)));
  return r ? __builtin_ctz(r) : 32;
}

// SpecSchedule.Next(t) -- node/cron/spec.go:55-145, literally, with each
// field walk advanced in one jump when no zone breakpoint lies inside the
// jumped span (within a constant-offset span an absolute +k*unit step moves the
// local field by exactly k units, so the intermediate loop iterations are
// no-ops).  Returns CG_ZERO_TIME for "no time within five years" and
// CG_BEYOND as soon as the (monotone) walk passes `bound`.
CG_HD int64_t next_exact(const DSpec& sp, const ZoneView& z, int64_t t, int64_t bound) {
  t += 1;  // t.Add(1s - nsec): inputs are whole seconds
  if (t > bound) return CG_BEYOND;
  // Masks that can never match make Go walk to the five-year limit and return
  // the zero time; answer that directly.
  {
    bool dom_any = (sp.dom & 0xFFFFFFFEu) != 0, dow_any = (sp.mondow & 0x7F0000u) != 0;
    bool day_any = (dom_star(sp) || dow_star(sp)) ? (dom_any && dow_any) : (dom_any || dow_any);
    if ((sp.sec & 0x0FFFFFFFFFFFFFFFull) == 0 || (sp.min & 0x0FFFFFFFFFFFFFFFull) == 0 ||
        (sp.hour & 0xFFFFFFu) == 0 || (sp.mondow & 0x1FFEu) == 0 || !day_any)
      return CG_ZERO_TIME;
  }
  bool added = false;
  Fields f = go_fields(z, t);
  const int32_t year_limit = f.y + 5;
  const uint32_t hourm = sp.hour;
  for (int guard = 0; guard < (1 << 22); guard++) {
    // WRAP:
    f = go_fields(z, t);
    if (f.y > year_limit) return CG_ZERO_TIME;
    bool wrapped = false;
    // month walk (spec.go:80-93)
    while (!month_ok(sp, f.mo)) {
      if (!added) {
        added = true;
        t = go_date(z, f.y, f.mo, 1, 0, 0, 0);
        f = go_fields(z, t);
      }
      t = go_date(z, f.y, f.mo + 1, f.d, f.h, f.mi, f.s);  // AddDate(0,1,0)
      f = go_fields(z, t);
      if (t > bound) return CG_BEYOND;
      if (f.mo == 1) { wrapped = true; break; }
    }
    if (wrapped) continue;
    // day walk (spec.go:96-106)
    while (!day_matches(sp, f.d, f.wd)) {
      if (!added) {
        added = true;
        t = go_date(z, f.y, f.mo, f.d, 0, 0, 0);
        f = go_fields(z, t);
      }
      // jump to the next matching day of this month, or to day 1 of the next
      int32_t dim = days_in_month(f.y, f.mo);
      int32_t k = dim - f.d + 1;  // steps until the day-1 wrap
      for (int32_t j = 1; j <= dim - f.d; j++) {
        if (day_matches(sp, f.d + j, (f.wd + j) % 7)) { k = j; break; }
      }
      // Date(L + j days) == t + j days for every step j <= k when the offset
      // is constant on [t - 2d, t + (k + 2)d] (Date looks up L and L - off(L)).
      int64_t nc;
      int32_t olo = zone_lookup(z, t - 2 * CG_SECS_PER_DAY, &nc);
      bool flat = olo == f.off && nc > t + (int64_t)(k + 2) * CG_SECS_PER_DAY;
      if (k > 1 && flat) {
        t += (int64_t)k * CG_SECS_PER_DAY;
      } else {
        int64_t prev = t;
        t = go_date(z, f.y, f.mo, f.d + 1, f.h, f.mi, f.s);  // AddDate(0,0,1)
        if (t <= prev) return CG_NO_PROGRESS;  // the reference loops forever here
      }
      f = go_fields(z, t);
      if (t > bound) return CG_BEYOND;
      if (f.d == 1) { wrapped = true; break; }
    }
    if (wrapped) continue;
    // hour walk (spec.go:108-118)
    while (!((hourm >> f.h) & 1u)) {
      if (!added) {
        added = true;
        t = go_date(z, f.y, f.mo, f.d, f.h, 0, 0);
        f = go_fields(z, t);
      }
      int32_t nh = next_bit32(hourm & 0xFFFFFFu, f.h);
      int32_t k = (nh < 24 ? nh : 24) - f.h;
      if (k > 1 && t + (int64_t)k * 3600 < f.next_change) t += (int64_t)k * 3600;
      else t += 3600;
      f = go_fields(z, t);
      if (t > bound) return CG_BEYOND;
      if (f.h == 0) { wrapped = true; break; }
    }
    if (wrapped) continue;
    // minute walk (spec.go:120-130)
    while (!((sp.min >> f.mi) & 1ull)) {
      if (!added) {
        added = true;
        t -= t - floordiv64(t, 60) * 60;  // Truncate(time.Minute)
        f = go_fields(z, t);
      }
      int32_t nm = next_bit64(sp.min & 0x0FFFFFFFFFFFFFFFull, f.mi);
      int32_t k = (nm < 60 ? nm : 60) - f.mi;
      if (k > 1 && t + (int64_t)k * 60 < f.next_change) t += (int64_t)k * 60;
      else t += 60;
      f = go_fields(z, t);
      if (t > bound) return CG_BEYOND;
      if (f.mi == 0) { wrapped = true; break; }
    }
    if (wrapped) continue;
    // second walk (spec.go:132-142)
    while (!((sp.sec >> f.s) & 1ull)) {
      added = true;  // Truncate(time.Second) is a no-op on whole seconds
      int32_t ns = next_bit64(sp.sec & 0x0FFFFFFFFFFFFFFFull, f.s);
      int32_t k = (ns < 60 ? ns : 60) - f.s;
      if (k > 1 && t + (int64_t)k < f.next_change) t += k;
      else t += 1;
      f = go_fields(z, t);
      if (t > bound) return CG_BEYOND;
      if (f.s == 0) { wrapped = true; break; }
    }
    if (wrapped) continue;
    return t;
  }
  return CG_ZERO_TIME;  // unreachable for valid tables (guard)
}

// ---- closed form inside a constant-offset span ----
// combos of (hour, minute, second) at or before second-of-day `tod`
CG_HD uint32_t tod_rank(uint32_t H, uint64_t M, uint64_t S, uint32_t nM, uint32_t nS,
                        int32_t tod) {
  if (tod < 0) return 0;
  int32_t h = tod / 3600, m = (tod / 60) % 60, s = tod % 60;
  uint32_t r = (uint32_t)__builtin_popcount(H & ((1u << h) - 1u)) * nM * nS;
  if ((H >> h) & 1u) {
    r += (uint32_t)__builtin_popcountll(M & ((1ull << m) - 1ull)) * nS;
    if ((M >> m) & 1ull) r += (uint32_t)__builtin_popcountll(S & ((2ull << s) - 1ull));
  }
  return r;
}

// position of the i-th (0-based) set bit of m; m must have > i bits set
CG_HD int32_t select64(uint64_t m, uint32_t i) {
  int32_t pos = 0;
  uint32_t c = (uint32_t)__builtin_popcount((uint32_t)m);
  if (i >= c) { i -= c; m >>= 32; pos = 32; }
  c = (uint32_t)__builtin_popcount((uint32_t)(m & 0xFFFFu));
  if (i >= c) { i -= c; m >>= 16; pos += 16; }
  c = (uint32_t)__builtin_popcount((uint32_t)(m & 0xFFu));
  if (i >= c) { i -= c; m >>= 8; pos += 8; }
  c = (uint32_t)__builtin_popcount((uint32_t)(m & 0xFu));
  if (i >= c) { i -= c; m >>= 4; pos += 4; }
  c = (uint32_t)__builtin_popcount((uint32_t)(m & 0x3u));
  if (i >= c) { i -= c; m >>= 2; pos += 2; }
  c = (uint32_t)(m & 1u);
  if (i >= c) { pos += 1; }
  return pos;
}

// ---- Cmd.lockTtl (job.go:194-233) ----
// Job kinds, job.go:30-34.
enum { JOB_COMMON = 0, JOB_ALONE = 1, JOB_INTERVAL = 2 };
// Maximum time.Duration in whole seconds: Sub saturates at +-(2^63-1) ns, and
// Duration / Second truncates toward zero (time.go Sub, job.go:197).
#define CG_SUB_SAT_SECS 9223372036LL

// The lease TTL from prev = Next(now) and nxt = Next(prev) (whole seconds),
// the job's Kind and AvgTime (ms) and conf.Config.LockTtl.  Go's int64
// arithmetic wraps, so the adds run in uint64.  CG_NO_PROGRESS where either
// Next never returns (the reference then never returns either).
CG_HD int64_t lock_ttl_of(int64_t prev, int64_t nxt, int32_t kind, int64_t avg_ms,
                          int64_t lock_ttl) {
  if (prev == CG_NO_PROGRESS || nxt == CG_NO_PROGRESS) return CG_NO_PROGRESS;
  const int64_t d = nxt - prev;  // both within [ZERO_TIME, 2^45]
  int64_t ttl = d > CG_SUB_SAT_SECS ? CG_SUB_SAT_SECS : (d < -CG_SUB_SAT_SECS ? -CG_SUB_SAT_SECS : d);
  if (ttl == 0) return 0;
  if (kind == JOB_INTERVAL) {  // job.go:202-211
    ttl -= 2;
    if (ttl > lock_ttl) ttl = lock_ttl;
    if (ttl < 1) ttl = 1;
    return ttl;
  }
  // job.go:213-216.  Both operands are int64 (1e3 is an untyped constant), so
  // AvgTime/1e3 - cost*1e3 is cost - 1000*cost: the round-up fires only for a
  // negative cost.
  int64_t cost = avg_ms / 1000;
  if (int64_t(uint64_t(cost) - uint64_t(cost) * 1000u) > 0) cost = int64_t(uint64_t(cost) + 1u);
  if (ttl >= cost) ttl = int64_t(uint64_t(ttl) - uint64_t(cost));  // job.go:219-221
  if (ttl > lock_ttl) ttl = lock_ttl;
  if (ttl < 2) ttl = 2;  // job.go:227-230
  return ttl;
}

}  // namespace cg
