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
  int32_t zn, G, nd, pad;
  int64_t t0, t1;
};

constexpr int kWriteThreads = 256;
constexpr int kWritePerThread = 8;
constexpr int kWriteChunk = kWriteThreads * kWritePerThread;  // events per write block

size_t plan_lds_bytes(const PlanArgs& p);

void launch_next_batch(const DSpec* specs, int64_t n, const PlanArgs& p, const int64_t* t_in,
                       int64_t* t_out, hipStream_t st);

// stuck_rule: atomicMin of the first rule whose reference Next never returns
void launch_count(const DSpec* specs, int64_t R, const PlanArgs& p, int64_t* run_anchor,
                  int32_t* run_count, uint32_t* run_dmask, unsigned long long* stuck_rule,
                  hipStream_t st);

// exclusive scan of n int32 counts into out[0..n] (out[n] = total)
size_t scan_temp_bytes(int64_t n);
void launch_scan(const int32_t* in, int64_t* out, int64_t n, void* temp, hipStream_t st);

void launch_block_map(const int64_t* run_off, int64_t nruns, int64_t nblocks, int64_t* block_run,
                      hipStream_t st);

void launch_write_cf(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor,
                     const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                     int64_t nruns, const int64_t* block_run, int64_t nblocks, int64_t E,
                     int64_t* times, hipStream_t st);

void launch_write_walk(const DSpec* specs, int64_t R, const PlanArgs& p, const int64_t* run_anchor,
                       const int32_t* run_count, const uint32_t* run_dmask, const int64_t* run_off,
                       int64_t* times, hipStream_t st);

void launch_rule_offsets(const int64_t* run_off, int64_t R, int32_t G, int64_t* offsets,
                         hipStream_t st);

}  // namespace cg
