// cg_expand.h -- per-rule expansion logic shared by the kernels (and by the
// host-side algorithm check in tests/native): the closed form inside a
// constant-offset CF segment, and the per-rule run planner of k_count.
//
// Expansion of one rule over (T0, T1] is the reference loop
//   t = T0; loop { t = Next(t); if t.IsZero() || t > T1 break; emit t }
// (cron.go:212-215 batched).  Per plan segment the engine records a run:
//   CF   segment: first fire f = Next(previous fire) by the exact walk, then
//                 the closed form: every later matching local time in the
//                 segment (DESIGN.md §3 proves these coincide with Next).
//   WALK segment: fires produced one by one by the exact walk.
#pragma once
#include "cg_time.h"
#include "cg_zone.h"

namespace cg {

struct CFRule {
  uint64_t M, S;
  uint32_t H, nM, nS, nMS, C;
  int32_t s0, m0, h0;  // lowest set bit of S, M, H
};

CG_HD CFRule cf_rule(const DSpec& sp) {
  CFRule c;
  c.H = sp.hour & 0xFFFFFFu;
  c.M = sp.min & 0x0FFFFFFFFFFFFFFFull;
  c.S = sp.sec & 0x0FFFFFFFFFFFFFFFull;
  c.nM = (uint32_t)__builtin_popcountll(c.M);
  c.nS = (uint32_t)__builtin_popcountll(c.S);
  c.nMS = c.nM * c.nS;
  c.C = (uint32_t)__builtin_popcount(c.H) * c.nMS;
  c.s0 = c.S ? __builtin_ctzll(c.S) : 0;
  c.m0 = c.M ? __builtin_ctzll(c.M) : 0;
  c.h0 = c.H ? __builtin_ctz(c.H) : 0;
  return c;
}

CG_HD uint32_t cf_rank(const CFRule& c, int32_t tod) {
  return tod_rank(c.H, c.M, c.S, c.nM, c.nS, tod);
}

// matching local days of a CF segment (Month bit + dayMatches), bit j = day0 + j
CG_HD uint32_t seg_daymask(const DSpec& sp, const Segment& sg, const uint32_t* dtab) {
  uint32_t m = 0;
  for (int j = 0; j < sg.ndays; j++) {
    uint32_t e = dtab[sg.dt_off + j];
    int mo = e & 15, dom = (e >> 4) & 31, dow = (e >> 9) & 7;
    if (month_ok(sp, mo) && day_matches(sp, dom, dow)) m |= 1u << j;
  }
  return m;
}

// # of matching instants in (uf, ue], both inside CF segment sg
CG_HD int64_t cf_count(const CFRule& c, const Segment& sg, uint32_t dmask, int64_t uf,
                       int64_t ue) {
  if (c.C == 0 || ue <= uf) return 0;
  int32_t rf = (int32_t)(uf - sg.base), re = (int32_t)(ue - sg.base);
  int32_t jf = rf / 86400, tf = rf - jf * 86400;
  int32_t je = re / 86400, te = re - je * 86400;
  uint64_t dm = dmask;
  if (jf == je) return ((dm >> jf) & 1) ? (int64_t)cf_rank(c, te) - (int64_t)cf_rank(c, tf) : 0;
  int64_t n = 0;
  if ((dm >> jf) & 1) n += (int64_t)c.C - (int64_t)cf_rank(c, tf);
  uint64_t mid = dm & ~((2ull << jf) - 1ull) & ((1ull << je) - 1ull);
  n += (int64_t)c.C * __builtin_popcountll(mid);
  if ((dm >> je) & 1) n += cf_rank(c, te);
  return n;
}

struct CFIter {
  int32_t day, h, m, s;
};

// iterator state of the anchor fire itself (k = 0): plain decode, no rank/select
CG_HD CFIter cf_decode(const Segment& sg, int64_t uf) {
  uint32_t rf = (uint32_t)(uf - sg.base);
  uint32_t day = rf / 86400u, tod = rf - day * 86400u;
  CFIter it;
  it.day = (int32_t)day;
  it.h = (int32_t)(tod / 3600u);
  uint32_t r = tod - (uint32_t)it.h * 3600u;
  it.m = (int32_t)(r / 60u);
  it.s = (int32_t)(r - (uint32_t)it.m * 60u);
  return it;
}

// iterator state of the k-th (k >= 0) fire counted from the anchor fire uf
// (32-bit: a segment holds at most 31 days x 86400 combinations)
CG_HD CFIter cf_seek(const CFRule& c, const Segment& sg, uint32_t dmask, int64_t uf, int64_t k) {
  if (k == 0) return cf_decode(sg, uf);
  uint32_t rf = (uint32_t)(uf - sg.base);
  uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  uint32_t idx = cf_rank(c, (int32_t)tf) - 1u + (uint32_t)k;
  CFIter it;
  it.day = (int32_t)jf;
  if (idx >= c.C) {
    idx -= c.C;
    uint32_t dskip = idx / c.C;
    idx -= dskip * c.C;
    uint64_t above = (uint64_t)dmask & ~((2ull << jf) - 1ull);
    it.day = select64(above, dskip);
  }
  uint32_t hi = idx / c.nMS;
  uint32_t rem = idx - hi * c.nMS;
  uint32_t mi = rem / c.nS;
  uint32_t si = rem - mi * c.nS;
  it.h = select64(c.H, hi);
  it.m = select64(c.M, mi);
  it.s = select64(c.S, si);
  return it;
}

// next matching (day, h, m, s), branch-free: the carries are selects, so lanes
// of a wave at different phases of the same (or another) rule do not diverge
CG_HD void cf_next(const CFRule& c, uint32_t dmask, CFIter& it) {
  uint64_t rs = c.S & (~0ull << (it.s + 1));   // it.s <= 59
  uint64_t rm = c.M & (~0ull << (it.m + 1));   // it.m <= 59
  uint32_t rh = c.H & (~0u << (it.h + 1));      // it.h <= 23
  uint32_t rd = (it.day >= 31) ? 0u : (dmask & (~0u << (it.day + 1)));
  int32_t s1 = rs ? __builtin_ctzll(rs) : 64;
  int32_t m1 = rm ? __builtin_ctzll(rm) : 64;
  int32_t h1 = rh ? __builtin_ctz(rh) : 32;
  int32_t d1 = rd ? __builtin_ctz(rd) : 32;
  bool os = s1 >= 64;
  bool om = os && m1 >= 64;
  bool oh = om && h1 >= 32;
  it.s = os ? c.s0 : s1;
  it.m = os ? (om ? c.m0 : m1) : it.m;
  it.h = om ? (oh ? c.h0 : h1) : it.h;
  it.day = oh ? d1 : it.day;
}

CG_HD int64_t cf_value(const Segment& sg, const CFIter& it) {
  return sg.base + (int64_t)(uint32_t)(it.day * 86400 + it.h * 3600 + it.m * 60 + it.s);
}

// First matching local time after instant u inside CF segment sg (day mask
// dmask), or INT64_MAX when none of the segment's days has one.  Within a
// constant-offset span Go's Next is the fixed-offset walk, which returns
// exactly this, so a run's first fire needs no walk when the
// walk from its start would stay inside the span.
CG_HD int64_t cf_first_after(const CFRule& c, const Segment& sg, uint32_t dmask, int64_t u) {
  if (c.C == 0) return INT64_MAX;
  const int64_t rf = u - sg.base;
  int32_t j = 0, tod = -1;  // u's local day in the segment and second of day
  if (rf >= 0) {
    if (rf >= 32 * 86400LL) return INT64_MAX;
    j = (int32_t)(rf / 86400);
    tod = (int32_t)(rf - (int64_t)j * 86400);
  }
  uint32_t r = 0;  // rank of the first combination after tod
  if (!((dmask >> j) & 1u) || (r = cf_rank(c, tod)) >= c.C) {
    const uint32_t above = j >= 31 ? 0u : (dmask & (~0u << (j + 1)));
    if (!above) return INT64_MAX;
    j = __builtin_ctz(above);
    r = 0;
  }
  const uint32_t hi = r / c.nMS, rem = r - hi * c.nMS;
  const uint32_t mi = rem / c.nS, si = rem - mi * c.nS;
  return sg.base + (int64_t)j * 86400 + (int64_t)select64(c.H, hi) * 3600 +
         (int64_t)select64(c.M, mi) * 60 + select64(c.S, si);
}

// Run records of one rule over the plan's G segments (k_count's body).
// Writes anchor/count/dmask at stride 1 from the given pointers.  Returns
// false where the reference loop never terminates: Next never returns
// (CG_NO_PROGRESS) or returns a time <= its input (it then cycles forever,
// e.g. Pacific/Chatham's 45-minute fall-back).
//
// A CF segment's run switches to the closed form only at a fire whose fields
// all match in the segment's offset (premise (i)).  The walk can
// emit fires that do not (America/Havana: the hour walk misses the wrap when
// local midnight does not exist, so the day is never re-checked); such a
// segment is walked fire by fire instead and flagged with kRunWalked in its
// daymask word.
constexpr uint32_t kRunWalked = 0x80000000u;

CG_HD bool cf_full_match(const DSpec& sp, const CFRule& c, const Segment& sg,
                         const uint32_t* dtab, int64_t u) {
  int32_t r = (int32_t)(u - sg.base);
  int32_t j = r / 86400, tod = r - j * 86400;
  uint32_t e = dtab[sg.dt_off + j];
  int mo = e & 15, dom = (e >> 4) & 31, dow = (e >> 9) & 7;
  if (!month_ok(sp, mo) || !day_matches(sp, dom, dow)) return false;
  int32_t h = tod / 3600, m = (tod / 60) % 60, s = tod % 60;
  return ((c.H >> h) & 1u) && ((c.M >> m) & 1ull) && ((c.S >> s) & 1ull);
}

// Next's five-year limit (spec.go:70-76): the walk from t returns the zero time
// instead of a match e whose local year is past Year(t + 1s) + 5 (it reaches a
// WRAP in that year first).  Only a gap of more than five years can trip it
// (e.g. Feb 29 across 2100), so the exact test runs only for such gaps.
CG_HD bool past_year_limit(const ZoneView& z, int64_t t, int64_t e, int32_t e_off) {
  if (e - t < 1800 * CG_SECS_PER_DAY) return false;
  const int64_t u = t + 1;
  const int32_t y0 = civil_from_days(floordiv64(u + zone_offset(z, u), CG_SECS_PER_DAY)).y;
  const int32_t ye = civil_from_days(floordiv64(e + e_off, CG_SECS_PER_DAY)).y;
  return ye > y0 + 5;
}

// kWalk = false: a plan with no WALK segment and no flags (e.g. UTC, or a
// zone far from its transitions): every run is closed form, no exact walk is
// reachable, and the kernel drops next_exact (and its registers).
template <bool kWalk = true>
CG_HD bool count_rule(const DSpec& sp, const ZoneView& z, const Segment* segs, int G,
                      const uint32_t* dtab, int64_t t0, int64_t t1, uint32_t flags,
                      int64_t* anchor_out, int32_t* count_out, uint32_t* dmask_out) {
  if (sp.kind == KIND_EVERY) {
    // ConstantDelaySchedule: T0 + k*D for k >= 1 (constantdelay.go:25-27),
    // one run per segment (k with T0 + kD in (a, b]; anchor = the time one
    // period before its first fire), so no run outgrows int32 on long horizons
    const int64_t D = (int64_t)sp.sec;
    for (int s = 0; s < G; s++) {
      const int64_t ka = (segs[s].a - t0) / D, kb = ((segs[s].b < t1 ? segs[s].b : t1) - t0) / D;
      anchor_out[s] = t0 + ka * D;
      count_out[s] = (int32_t)(kb > ka ? kb - ka : 0);
      dmask_out[s] = 0;
    }
    return true;
  }
  const CFRule c = cf_rule(sp);
  int64_t pos = t0;             // last fire so far (or T0)
  int64_t pending = INT64_MIN;  // Next(pos) if already computed
  bool done = false, ok = true;
  // The walk from T0 (not a fire) may first reset back to the start of T0's
  // month, day or hour; with a zone transition in the 40 days before T0 that
  // reset can land across it, so Next(T0) then comes from the exact walk.
  const bool t0_walk = (flags & kPlanT0Walk) != 0;
  // A skipped local day ahead (kPlanFinalWalk): the reference's last Next,
  // the one past T1, may never return; it is walked to its end.
  const bool final_walk = (flags & kPlanFinalWalk) != 0;
  bool final_known = false;  // that last Next has been walked to its end
  for (int s = 0; s < G; s++) {
    const Segment& sg = segs[s];
    int64_t anchor = 0, cnt = 0;
    uint32_t dm = 0;
    if (!done && sg.kind == 0 && pending == INT64_MIN && !(t0_walk && pos == t0)) {
      // Next(pos) in closed form: pos is T0 (no transition in the 40 days
      // before it) or the last fire of a CF segment before this one in the
      // same span, so the walk from pos stays in the span until its result
      const int64_t b = sg.b < t1 ? sg.b : t1;
      dm = seg_daymask(sp, sg, dtab);
      const int64_t e = cf_first_after(c, sg, dm, pos > sg.a ? pos : sg.a);
      if (e <= b && past_year_limit(z, pos, e, sg.off)) {
        dm = 0;  // Next(pos) is the zero time: the reference loop stops here
        done = true;
        final_known = true;
      } else if (e <= b) {
        cnt = 1 + cf_count(c, sg, dm, e, b);
        anchor = e;
        // the run's last fire starts the next segment's search (not needed
        // after the last segment: one closed-form seek saved per rule)
        if (s + 1 < G || final_walk) pos = cnt > 1 ? cf_value(sg, cf_seek(c, sg, dm, e, cnt - 1)) : e;
      } else {
        dm = 0;  // no fire in this segment; the next one searches from its start
      }
    } else if (!done) {
      const int64_t b = sg.b < t1 ? sg.b : t1;
      int64_t e = CG_BEYOND;
      if constexpr (kWalk) e = pending != INT64_MIN ? pending : next_exact(sp, z, pos, t1);
      pending = INT64_MIN;
      if (e <= pos && e != CG_ZERO_TIME) e = CG_NO_PROGRESS;  // backwards: the loop cycles
      if (sg.kind == 0 && e != CG_NO_PROGRESS && e != CG_ZERO_TIME && e != CG_BEYOND &&
          e <= b && cf_full_match(sp, c, sg, dtab, e)) {
        dm = seg_daymask(sp, sg, dtab);
        cnt = 1 + cf_count(c, sg, dm, e, b);
        anchor = e;
        // the run's last fire starts the next segment's search (not needed
        // after the last segment: one closed-form seek saved per rule)
        if (s + 1 < G || final_walk) pos = cnt > 1 ? cf_value(sg, cf_seek(c, sg, dm, e, cnt - 1)) : e;
      } else {
        // walked run: a WALK segment, or a CF segment entered by a fire the
        // closed form cannot continue from
        anchor = pos;
        if (sg.kind == 0) dm = kRunWalked;
        for (;;) {
          if (e <= pos && e != CG_ZERO_TIME) e = CG_NO_PROGRESS;
          if (e == CG_NO_PROGRESS) { done = true; ok = false; break; }
          if (e == CG_ZERO_TIME || e == CG_BEYOND) { done = true; final_known = e == CG_ZERO_TIME; break; }
          if (e > b) { pending = e; break; }
          cnt++;
          pos = e;
          if constexpr (kWalk) e = next_exact(sp, z, pos, t1);
        }
        if (cnt == 0) dm = 0;
      }
    }
    anchor_out[s] = anchor;
    count_out[s] = (int32_t)cnt;
    dmask_out[s] = dm;
  }
  if (kWalk && final_walk && ok && !final_known) {
    const int64_t e = next_exact(sp, z, pos, INT64_MAX);
    if (e == CG_NO_PROGRESS || (e <= pos && e != CG_ZERO_TIME)) ok = false;
  }
  return ok;
}

// does run (segment kind, daymask word) hold walked fires?
CG_HD bool run_is_walked(const Segment& sg, uint32_t dmask) {
  return sg.kind != 0 || (dmask & kRunWalked) != 0;
}

}  // namespace cg
