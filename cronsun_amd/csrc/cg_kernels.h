// cg_kernels.h -- launch wrappers for the gfx950 kernels (cg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cg_time.h"
#include "cg_zone.h"

namespace cg {

// Per-batch plan as the kernels see it (device pointers).
struct PlanArgs {
  const int64_t* zwhen;
  const int32_t* zoff;
  const Segment* segs;
  const uint32_t* dtab;
  int32_t zn, G, nd;
  int32_t dtab_global;  // 1: the day table is read from HBM (too large to stage in LDS)
  uint32_t flags;       // Plan::flags (kPlanT0Walk | kPlanFinalWalk)
  int64_t t0, t1;
};

// Plan limits: segments (k_write_cf keeps all of them in LDS beside its 12 KB
// run windows) and the LDS the zone table + segments (+ day table) may use.
constexpr int kMaxSegments = 1024;
constexpr size_t kPlanLdsBytes = 60 * 1024;

// closed-form writer: 4 waves per block; waves take output slices by ticket
// 2-wave blocks, 6 per CU (12 waves per CU, as 3 blocks of 4): 1-2 % faster
// than 4-wave blocks on two boxes (profiles/r04_ab_writer_layout.txt; 8-wave
// blocks, 1-wave blocks, 1024-event slices, plain stores, 4/16-block store
// batches and 16/64 ticket groups were slower or equal)
#ifndef CG_WRITE_WAVES
#define CG_WRITE_WAVES 2
#endif
constexpr int kWriteWaves = CG_WRITE_WAVES;
// 3 blocks per CU (12 waves): fewer concurrent write streams store faster
// (same-box A/B on config 2, profiles/r04_ab_writer_bpc.txt: k_write_cf
// 1.005-1.008 ms at 3 vs 1.041-1.042 at 4 and 1.081-1.088 at 2; a window
// prefetched one slice ahead was slower at 4 (spills) and at 3 -- the wait at
// its commit drains the previous slice's stores anyway)
#ifndef CG_WRITE_BPC
#define CG_WRITE_BPC (12 / CG_WRITE_WAVES)
#endif
constexpr int kWriteBlocksPerCU = CG_WRITE_BPC;  // persistent grid: blocks of 4 waves per CU
// writer slice tickets: one u32 counter per group of blocks, 128 B apart
#ifndef CG_TICKET_GROUPS
#define CG_TICKET_GROUPS 32
#endif
constexpr int kTicketGroups = CG_TICKET_GROUPS;
constexpr int kTicketStride = 32;                                  // u32 words
constexpr int kTicketWords = kTicketGroups * kTicketStride / 2;    // int64 words
// Events per writer slice, chosen per call from the output capacity (host and
// kernels derive it from the same cap): 2048 (a 16-KB write front per wave)
// below 2^31 events, 16384 above (fewer slices, tickets and map entries).
// A/B on one box (profiles/r02_ab_slices.json): config 2 (0.67 G events)
// 0.99-1.01 ms at 2048 vs 1.10 ms at 16384; config 4 (18.2 G) 25.9 ms vs 24.2.
#ifndef CG_SUPER_SHIFT_SMALL
#define CG_SUPER_SHIFT_SMALL 11
#endif
#ifndef CG_SUPER_SHIFT_LARGE
#define CG_SUPER_SHIFT_LARGE 14
#endif
static_assert(CG_SUPER_SHIFT_SMALL >= 6 && CG_SUPER_SHIFT_LARGE >= 6, "slices are whole 64-event blocks");
__host__ __device__ inline int super_shift(int64_t cap) {
  return cap >= (int64_t(1) << 31) ? CG_SUPER_SHIFT_LARGE : CG_SUPER_SHIFT_SMALL;
}
// Short windows.  Fewer than kUSlices position slices (E < 2^(shift + 14):
// a tick loop's next minute or hour) leave most writer waves idle, and a
// slice then stretches over thousands of runs, most of them empty (a 1-min
// window of 1M rules: 338 k fires in 1M runs).  The writer's slices are then
// cut in cost space instead: run j costs its fires + 1, u_j = run_off[j] + j,
// slice c starts at the position of u = c * 2^s rounded down to a 64-event
// block (k_chunk_map_u), with s the smallest shift (>= 6) giving at most
// kUSlices slices.  Host and kernels decide the mode from E on the device.
constexpr int64_t kUSlices = 16384;
__host__ __device__ inline bool u_mode(int64_t E, int64_t cap) { return (E >> super_shift(cap)) < kUSlices; }
__host__ __device__ inline int u_shift(int64_t U) {
  int s = 6;
  while ((U >> s) >= kUSlices) s++;
  return s;
}
// slice-map entries for an output capacity: the map, 2 sentinels, the ticket
// counters, 8 debug words, then the cost-space map ({first position, first
// run} per slice and one past the last)
__host__ __device__ inline int64_t u_map_base(int64_t cap) {
  return (cap >> super_shift(cap)) + 2 + kTicketWords + 8;
}
inline int64_t slice_map_words(int64_t cap) { return u_map_base(cap) + 2 * (kUSlices + 2); }


size_t plan_lds_bytes(const PlanArgs& p);

// *out += order-sensitive checksum of n elements (int64 or int32) of v,
// positions first.., values + add (cg_checksum_device)
void launch_checksum(const void* v, int64_t n, int elem_bytes, int64_t first, int64_t add,
                     unsigned long long* out, hipStream_t st);

// *out += count of elements (int64 or int32) of v equal to x (cg_count_value_device)
// streaming fill of n16 16-B words (store-ceiling probe of cg_fill_rate_device):
// nt = 1 nontemporal stores, 0 plain
void launch_fill_stream(void* p, int64_t n16, int nt, hipStream_t st);

void launch_count_eq(const void* v, int64_t n, int elem_bytes, int64_t x, unsigned long long* out,
                     hipStream_t st);

void launch_next_batch(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* t_in,
                       int64_t* t_out, hipStream_t st);
// GPU-resident dispatcher (cg_dispatch.cpp): one block per kDispatchTile entries
constexpr int kDispatchTile = 4096;
struct DispatchState {
  unsigned long long min_key;  // byTime minimum of Next (sign-flipped; ~0 = none)
  unsigned long long n_due;    // entries fired by the last wake
  unsigned long long stuck;    // first entry whose Next never returns (~0 = none)
  unsigned long long pad;
};
void launch_dispatch_scan(const int64_t* next, int64_t n, int64_t effective,
                          unsigned long long* due_bits, uint32_t* tile_cnt,
                          unsigned long long* tile_min, hipStream_t s);
void launch_dispatch_advance(const DSpec* specs, const int32_t* due, int64_t n, const PlanArgs& p,
                             int64_t now, int64_t* next, int64_t* prev, DispatchState* st,
                             hipStream_t s);
void launch_dispatch_compact(const unsigned long long* due_bits, const uint32_t* tile_cnt,
                             const unsigned long long* tile_min, int64_t n, int32_t* due,
                             DispatchState* st, hipStream_t s);
void launch_dispatch_place(DSpec* specs, const int64_t* idx, const DSpec* src, int64_t first,
                           int64_t k, const PlanArgs& p, int64_t now, int64_t* next, int64_t* prev,
                           DispatchState* st, hipStream_t s);
void launch_dispatch_clear(const int64_t* idx, int64_t first, int64_t k, int64_t* next, int64_t* prev,
                           hipStream_t s);
void launch_dispatch_min(const int64_t* next, int64_t n, DispatchState* st, hipStream_t s);
void launch_lock_ttl(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* now,
                     const int32_t* kind, const int64_t* avg_ms, int64_t lock_ttl, int64_t* ttl,
                     hipStream_t st);

// stuck_rule: atomicMin of the first rule whose reference Next never returns
void launch_count(const DSpec* specs, int64_t R, const PlanArgs& p, int64_t* run_anchor,
                  int32_t* run_count, uint32_t* run_dmask, unsigned long long* stuck_rule,
                  hipStream_t st);

// exclusive scan of n int32 counts into out[0..n] (out[n] = total)
size_t scan_temp_bytes(int64_t n);
void launch_scan(const int32_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st);
// the same over int64 counts
void launch_scan64(const int64_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st);
// expansion scan (R*G > 0 run counts): also writes the per-rule offsets
// (offsets[r] = run_off[r*G]), res = {E, stuck rule} and re-arms *stuck;
// with chunk_run (else null) also the writer's slice map for capacity cap
// (as launch_chunk_map)
void launch_scan_runs(const int32_t* run_count, int64_t* run_off, int64_t R, int32_t G, void* temp,
                      int64_t* offsets, int64_t* res, unsigned long long* stuck,
                      int64_t* chunk_run, int64_t cap, hipStream_t st);

// chunk_run needs slice_map_words(cap) entries (slice map, the
// writer's slice tickets, 8 diagnostic counters); both read E = run_off[nruns]
// on the device (no host sync) and do nothing when E > cap
void launch_chunk_map(const int64_t* run_off, int64_t nruns, int64_t cap, int64_t* chunk_run,
                      hipStream_t st);
// the cost-space slice map of a short window (u_mode; nothing otherwise);
// launched by launch_scan_runs (with chunk_run) and launch_chunk_map
void launch_chunk_map_u(const int64_t* run_off, int64_t nruns, int64_t cap, int64_t* chunk_run,
                        hipStream_t st);
void launch_write_cf(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor,
                     const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                     int64_t nruns, int64_t* chunk_run, int64_t cap, int64_t* times,
                     int n_blocks, hipStream_t st);

void launch_write_walk(const DSpec* specs, int64_t R, const PlanArgs& p, const int64_t* run_anchor,
                       const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                       int64_t cap, int64_t* times, hipStream_t st);

#ifdef CG_DIAG
// diagnostic library only (cg_diag.hip): launches a probe or an experimental
// writer in place of k_write_cf when CG_WRITE_PROBE / CG_WRITE_VARIANT ask for
// one (returns true), else nothing
bool launch_write_diag(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor, const int32_t* run_count,
                       const uint32_t* run_dmask, const int64_t* run_off, int64_t nruns, int64_t* chunk_run,
                       int64_t cap, int64_t* times, int n_blocks, size_t lds, hipStream_t st);
#endif


}  // namespace cg
