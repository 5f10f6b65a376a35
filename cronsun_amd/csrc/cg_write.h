// cg_write.h -- device helpers of the closed-form writer (k_write_cf in
// cg_kernels.hip; the diagnostic library's experimental writers in
// cg_diag.hip reuse them): the per-wave run window, the aligned 64-fire block
// protocol (drive / Pending) and the fire generators of a closed-form run
// (mixed-radix digits, lane rank tables, per-lane seeks, @every progressions).
// Everything here follows cg_expand.h's enumeration (cf_seek / cf_next), i.e.
// the reference's Next loop inside a constant-offset span.
#pragma once
#include <hip/hip_runtime.h>

#include "cg_expand.h"
#include "cg_kernels.h"

namespace cg {
namespace {

// one run of a wave's 64-run window (lane i holds run jw + i), staged in LDS
// (48 B; the run offset stays in a VGPR of lane i, the plan segment index
// rides in the spec's kind word: kind | seg << 8)
struct WinRun {
  int64_t anchor;  // run_anchor[j]
  DSpec sp;        // specs[j / G]
  int32_t count;   // run_count[j]
  uint32_t dmask;  // run_dmask[j]
};
__device__ __forceinline__ bool win_every(const WinRun& w) { return (w.sp.kind & 0xFFu) == KIND_EVERY; }
__device__ __forceinline__ int win_seg(const WinRun& w) { return int(w.sp.kind >> 8); }

__device__ __forceinline__ int32_t rl32(int32_t v, int i) { return __builtin_amdgcn_readlane(v, i); }
__device__ __forceinline__ int64_t rl64(int64_t v, int i) {
  const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), i));
  const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(v) >> 32)), i));
  return int64_t((uint64_t(hi) << 32) | lo);
}

// Lane k of the result holds unit * (position of the k-th set bit of m), for
// k < popcount(m): each lane pushes its own position to the lane of its rank
// (set bits to 0..n-1, clear bits to n..63 -- a permutation), ds_permute_b32.
// All 64 lanes must be active.
__device__ __forceinline__ int32_t rank_table(uint64_t m, int32_t unit) {
  const int lane = threadIdx.x & 63;
  const bool set = (m >> lane) & 1ull;
  const int32_t below = __popcll(m & ((1ull << lane) - 1ull));
  const int32_t n = __popcll(m);
  const int32_t dst = set ? below : n + (lane - below);
  return __builtin_amdgcn_ds_permute(dst << 2, lane * unit);
}
// entry idx of a rank table (ds_bpermute_b32; idx is taken mod 64)
__device__ __forceinline__ int32_t rank_at(int32_t table, uint32_t idx) {
  return __builtin_amdgcn_ds_bpermute(int(idx << 2), table);
}
// floor(x / n) for x < 2^16, n >= 1, with inv = 1/n (the +0.5 keeps the
// product at least 0.5/n away from an integer, far above the f32 error)
__device__ __forceinline__ uint32_t small_div(uint32_t x, float inv) {
  return uint32_t((float(x) + 0.5f) * inv);
}
// floor(x / n) for x < 2^24, n >= 1, inv = 1/n: the f32 quotient is off by at
// most one, fixed by one remainder test each way (cheaper than a u32 divide)
__device__ __forceinline__ uint32_t fdiv(uint32_t x, uint32_t n, float inv) {
  uint32_t q = uint32_t(float(x) * inv);
  const int32_t r = int32_t(x) - int32_t(q * n);
  q = r < 0 ? q - 1u : (r >= int32_t(n) ? q + 1u : q);
  return q;
}

// Output store: one lane's fire (every store instruction of the writer covers
// one whole 512-B block); nontemporal: the fires are not read back by this
// kernel (same-box A/B, profiles/r03_ab_writer_nt.json: equal or ~1 % faster
// than plain stores on configs 2 and 4).
#ifndef CG_WRITE_NT
#define CG_WRITE_NT 1
#endif
__device__ __forceinline__ void put(int64_t* p, int64_t v) {
  if (CG_WRITE_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// cf_seek (cg_expand.h) with the three variable divisions done by fdiv
// (quotients < 2^24); same result, fewer instructions.
__device__ __forceinline__ CFIter cf_seek_fast(const CFRule& c, const Segment& sg, uint32_t dmask,
                                               int64_t uf, int64_t k) {
  if (k == 0) return cf_decode(sg, uf);
  const uint32_t rf = uint32_t(uf - sg.base);
  const uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  uint32_t idx = cf_rank(c, int32_t(tf)) - 1u + uint32_t(k);
  CFIter it;
  it.day = int32_t(jf);
  if (idx >= c.C) {
    idx -= c.C;
    const uint32_t dskip = fdiv(idx, c.C, 1.0f / float(c.C));
    idx -= dskip * c.C;
    const uint64_t above = uint64_t(dmask) & ~((2ull << jf) - 1ull);
    it.day = select64(above, dskip);
  }
  const uint32_t hi = fdiv(idx, c.nMS, 1.0f / float(c.nMS));
  const uint32_t rem = idx - hi * c.nMS;
  const uint32_t mi = fdiv(rem, c.nS, 1.0f / float(c.nS));
  const uint32_t si = rem - mi * c.nS;
  it.h = select64(c.H, hi);
  it.m = select64(c.M, mi);
  it.s = select64(c.S, si);
  return it;
}

// Does mask m (n set bits) hold an arithmetic progression p0 + r*step?
// (rank r -> position is then linear; n <= 1 counts, with step 0)
__device__ __forceinline__ bool ap_level(uint64_t m, uint32_t n, int32_t* p0, int32_t* step) {
  *p0 = m ? __builtin_ctzll(m) : 0;
  *step = 0;
  if (n <= 1) return true;
  const uint64_t rest = m >> *p0;  // bit 0 set
  const int32_t st = __builtin_ctzll(rest >> 1) + 1;
  *step = st;
  // {0, st, 2st, ...} up to the top bit  <=>  ((rest << st) | 1) below the top == rest
  const int32_t top = 63 - __builtin_clzll(rest);
  const uint64_t low = top >= 63 ? ~0ull : ((2ull << top) - 1ull);
  return (((rest << st) | 1ull) & low) == rest;
}

// The aligned 64-fire block holding a run boundary, assembled across runs:
// each run fills its lanes, and the run that completes the block stores it
// with one whole 512 B store (no partially written cache line reaches HBM).
struct Pending {
  int64_t blk;  // block start, or -1 (wave-uniform)
  int64_t val;  // this lane's fire in it
};

// Position offset of this lane's first fire of a piece starting at p0: lane l
// covers p0 + x, x = (floor64(p0) + l - p0) mod 64 -- lanes before p0 in the
// head block belong to earlier runs and start one block later.
__device__ __forceinline__ uint32_t lane_offset(int64_t p0) {
  const int lane = threadIdx.x & 63;
  const int32_t x = int32_t((p0 & ~int64_t(63)) + lane - p0);
  return uint32_t(x < 0 ? x + 64 : x);
}

#ifndef CG_WRITE_BATCH
#define CG_WRITE_BATCH 8
#endif
constexpr int kBatch = CG_WRITE_BATCH;  // blocks computed before their stores are issued
// 64-bit ds_bpermute (lane src's value; src taken mod 64)
__device__ __forceinline__ int64_t bperm64_w(int64_t v, int src) {
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(v)));
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, int(uint32_t(uint64_t(v) >> 32)));
  return int64_t((uint64_t(uint32_t(hi)) << 32) | uint32_t(lo));
}

// Runs the piece [p0, p1) through the block protocol: value() is this lane's
// current fire, step() advances it by 64 fires.  Full blocks are stored as
// computed (8 values first, then 8 stores: a wave held back by a full memory
// pipe has no arithmetic queued behind the store); the head block merges the
// pending fires of earlier runs; a partial tail block becomes pending.
// GAP: a walked run -- its fires come from k_write_walk, so only the shared
// blocks are written (placeholders there), never its own full blocks.
template <bool GAP, class Val, class Step>
__device__ __forceinline__ void drive(Val&& value, Step&& step, int64_t p0, int64_t p1,
                                      Pending& pd, int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63;
  const int64_t b0 = p0 & ~int64_t(63);
  const bool mine0 = b0 + lane >= p0;
  {
    int64_t v = GAP ? 0 : value();
    if (!mine0) v = pd.val;
    if (b0 + 64 > p1) {  // the run ends inside its head block
      pd.blk = b0;
      pd.val = v;
      return;
    }
    put(times + b0 + lane, v);
    pd.blk = -1;
    if (!GAP && mine0) step();
  }
  int64_t b = b0 + 64;
  if (GAP) {
    b += (p1 - b) & ~int64_t(63);
  } else {
    for (; b + kBatch * 64 <= p1; b += kBatch * 64) {
      int64_t vv[kBatch];
#pragma unroll
      for (int u = 0; u < kBatch; u++) {
        vv[u] = value();
        step();
      }
#pragma unroll
      for (int u = 0; u < kBatch; u++) asm volatile("" : "+v"(vv[u]));
#pragma unroll
      for (int u = 0; u < kBatch; u++) put(times + b + 64 * u + lane, vv[u]);
    }
    for (; b + 64 <= p1; b += 64) {
      put(times + b + lane, value());
      step();
    }
  }
  if (b < p1) {
    pd.blk = b;
    pd.val = GAP ? 0 : value();
  }
}

// Fires [p0, p1) of closed-form run w (run start roff), wave-cooperatively.
// A fire's index g = rank(anchor) - 1 + (p - roff) counts (day, hour, minute,
// second) combinations from the anchor's local day, so it is carried as
// mixed-radix digits (matching-day rank, hour/minute/second ranks; radices -,
// nH, nM, nS) and stepped by the constant 64.  Same enumeration as
// cf_seek/cf_next.  Rank -> seconds, cheapest form first:
//   linear   every level an arithmetic progression and the sequence has one
//            stride (e.g. */10 s with every minute/hour/day): t += 64*stride;
//   affine   every level an arithmetic progression: t = C0 + sum r_i * w_i;
//   tables   otherwise: per-level lane tables read with ds_bpermute.
__device__ void coop_cf(const WinRun& w, int64_t roff, const Segment& sg, int64_t p0, int64_t p1,
                        Pending& pd, int64_t* __restrict__ times) {
  const CFRule c = cf_rule(w.sp);
  const uint32_t nS = c.nS, nM = c.nM, nH = uint32_t(__builtin_popcount(c.H));
  const uint32_t rf = uint32_t(w.anchor - sg.base);
  const uint32_t jf = rf / 86400u, tf = rf - jf * 86400u;
  const uint32_t dmask = w.dmask >> jf;  // matching days from the anchor's (bit 0)
  const float iS = 1.0f / float(nS), iM = 1.0f / float(nM), iH = 1.0f / float(nH);
  // g < 31 * 86400 < 2^24
  uint32_t g = cf_rank(c, int32_t(tf)) - 1u + uint32_t(p0 - roff);
  uint32_t d = fdiv(g, c.C, 1.0f / float(c.C));
  g -= d * c.C;
  uint32_t h = fdiv(g, c.nMS, 1.0f / float(c.nMS));
  g -= h * c.nMS;
  uint32_t m = fdiv(g, nS, iS);
  uint32_t s = g - m * nS;
  // + this lane's offset (< 128)
  uint32_t q;
  s += lane_offset(p0);
  q = small_div(s, iS);
  s -= q * nS;
  m += q;
  q = small_div(m, iM);
  m -= q * nM;
  h += q;
  q = small_div(h, iH);
  h -= q * nH;
  d += q;
  // digits of 64
  uint32_t a = small_div(64, iS);
  const uint32_t a0 = 64 - a * nS;
  uint32_t a_ = small_div(a, iM);
  const uint32_t a1 = a - a_ * nM;
  a = small_div(a_, iH);
  const uint32_t a2 = a_ - a * nH;
  const uint32_t a3 = a;
  auto step = [&]() {
    s += a0;
    const uint32_t cs = s >= nS;
    s -= cs ? nS : 0u;
    m += a1 + cs;
    const uint32_t cm = m >= nM;
    m -= cm ? nM : 0u;
    h += a2 + cm;
    const uint32_t ch = h >= nH;
    h -= ch ? nH : 0u;
    d += a3 + ch;
  };
  int32_t s0, ss, m0, ms, h0, hs, d0, ds;
  const uint32_t nD = uint32_t(__builtin_popcount(dmask));
  const bool apS = ap_level(c.S, nS, &s0, &ss), apM = ap_level(c.M, nM, &m0, &ms);
  const bool apH = ap_level(c.H, nH, &h0, &hs), apD = ap_level(dmask, nD, &d0, &ds);
  if (apS && apM && apH && apD) {
    const int64_t C0 = sg.base + s0 + 60 * m0 + 3600 * h0 + 86400 * int32_t(jf);  // d0 == 0
    const uint32_t ws = uint32_t(ss), wm = 60u * uint32_t(ms), wh = 3600u * uint32_t(hs),
                   wd = 86400u * uint32_t(ds);
    auto value = [&]() -> int64_t {
      // every product < 2^24 x 2^24 operands: v_mul_u32_u24 (full rate)
      return C0 + int64_t(__umul24(s, ws) + __umul24(m, wm) + __umul24(h, wh) + __umul24(d, wd));
    };
    // one stride: the lowest level with > 1 value wraps evenly into the next
    // unit, and every level above it takes every value (days: consecutive)
    const bool days_full = nD <= 1 || ds == 1;
    int32_t stride = 0;
    if (nS > 1) {
      if (uint32_t(ss) * nS == 60 && s0 < ss && nM == 60 && nH == 24 && days_full) stride = ss;
    } else if (nM > 1) {
      if (uint32_t(ms) * nM == 60 && m0 < ms && nH == 24 && days_full) stride = 60 * ms;
    } else if (nH > 1) {
      if (uint32_t(hs) * nH == 24 && h0 < hs && days_full) stride = 3600 * hs;
    } else {
      stride = 86400 * ds;
    }
    if (stride > 0) {
      int64_t v = value();
      const int64_t st = 64 * int64_t(stride);
      drive<false>([&]() { return v; }, [&]() { v += st; }, p0, p1, pd, times);
    } else {
      drive<false>(value, step, p0, p1, pd, times);
    }
    return;
  }
  const int32_t ts = rank_table(c.S, 1);
  const int32_t tm = rank_table(c.M, 60);
  const int32_t th = rank_table(c.H, 3600);
  const int32_t td = rank_table(uint64_t(dmask), 86400) + int32_t(jf) * 86400;
  const int64_t base = sg.base;
  auto value = [&]() -> int64_t {  // all lanes active: the table reads are cross-lane
    return base + int64_t(rank_at(td, d) + rank_at(th, h) + rank_at(tm, m) + rank_at(ts, s));
  };
  drive<false>(value, step, p0, p1, pd, times);
}

// Fires [p0, p1) of a short closed-form run: each lane seeks its own fire
// (the anchor itself, its successor, or cf_seek).
__device__ void tiny_cf(const WinRun& w, int64_t roff, const Segment& sg, int64_t p0, int64_t p1,
                        Pending& pd, int64_t* __restrict__ times) {
  int32_t k = int32_t(p0 - roff) + int32_t(lane_offset(p0));
  const CFRule c = cf_rule(w.sp);
  auto value = [&]() -> int64_t {
    if (k == 0) return w.anchor;
    if (int64_t(k) >= p1 - roff) return 0;  // not this run's (a later run's lane)
    if (k == 1) {
      CFIter it = cf_decode(sg, w.anchor);
      cf_next(c, w.dmask, it);
      return cf_value(sg, it);
    }
    return cf_value(sg, cf_seek_fast(c, sg, w.dmask, w.anchor, k));
  };
  drive<false>(value, [&]() { k += 64; }, p0, p1, pd, times);
}

// Fires [p0, p1) of @every run w: anchor + (k + 1) * D (constantdelay.go:25-27)
__device__ void coop_every(const WinRun& w, int64_t roff, int64_t p0, int64_t p1, Pending& pd,
                           int64_t* __restrict__ times) {
  const int64_t D = int64_t(w.sp.sec);
  int64_t t = w.anchor + (p0 - roff + int64_t(lane_offset(p0)) + 1) * D;
  const int64_t st = 64 * D;
  drive<false>([&]() { return t; }, [&]() { t += st; }, p0, p1, pd, times);
}

// Fire k (>= 0) of window run w, for one lane (the per-lane form of
// coop_every / tiny_cf): @every anchor + (k + 1) D (constantdelay.go:25-27),
// a walked run's placeholder 0 (k_write_walk writes it), else the k-th
// closed-form fire from the anchor.
__device__ __forceinline__ int64_t run_fire(const WinRun& w, const Segment& sg, int64_t k) {
  if (win_every(w)) return w.anchor + (k + 1) * int64_t(w.sp.sec);
  if (run_is_walked(sg, w.dmask)) return 0;
  if (k == 0) return w.anchor;
  const CFRule c = cf_rule(w.sp);
  if (k == 1) {
    CFIter it = cf_decode(sg, w.anchor);
    cf_next(c, w.dmask, it);
    return cf_value(sg, it);
  }
  return cf_value(sg, cf_seek_fast(c, sg, w.dmask, w.anchor, k));
}

}  // namespace
}  // namespace cg
