// cg_diag.hip -- diagnostic library only (`make diag`, CG_DIAG): kernels that
// stand in for the production writer to measure it, never part of
// libcronsun_gpu.so.  cg_build_info() reports CG_BUILD_DIAG for a library that
// holds them and bench.py refuses to print a headline from it.
//   CG_WRITE_PROBE=1..7  k_fill_probe: plain fills of the writer's output in
//                        its own grid and slices (store-ceiling probes)
//   CG_WRITE_PROBE=5     hipMemsetAsync of the output capacity
//   CG_WRITE_VARIANT=255 k_write_lw, the loader/writer split (DESIGN.md §5:
//                        correct, slower); 256 = the same with wait counters
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "cg_kernels.h"
#include "cg_write.h"

namespace cg {
namespace {

// ---- k_write_lw: the closed-form writer with its loads split off ----------
// On gfx9 a wave's vector loads and stores retire in issue order (one vmcnt),
// so every load a writer wave waits for -- its slice ticket, the slice's run
// window -- also waits for every store it issued before: in k_write_cf each
// slice drains the wave's store queue one to three times.  Here each block
// has kLwWriters writer waves that issue no vector loads and one loader wave
// that issues them all: it takes the tickets, reads the slice map and copies
// each slice's 64-run windows (run offsets, anchors, counts, day masks and
// the runs' rule specs) into one LDS slot per writer with global->LDS DMA
// (no registers; one wait for every writer's copies).  A writer turns its
// slot into its own window (as k_write_cf's) and hands the slot back at once,
// so the next window is copied while it writes.  Writers wait on LDS flags
// only (lgkmcnt): their stores stream without drains.  Every wait is
// bounded: a wave that waits ~2 s (the other side gone) sets an error word
// and leaves, so the grid always drains.
#ifndef CG_LW_WRITERS
#define CG_LW_WRITERS 7
#endif
constexpr int kLwWriters = CG_LW_WRITERS;
#ifndef CG_LW_WPE
#define CG_LW_WPE 4  // waves per SIMD the register allocation must allow
#endif
constexpr uint32_t kLwSpin = 1u << 25;  // polls of ~64 clocks each before giving up

struct LwSlot {  // one window, as copied: structure of arrays
  int64_t off[64];     // run_off
  int64_t anchor[64];  // run_anchor
  int32_t count[64];   // run_count
  uint32_t dmask[64];  // run_dmask
  DSpec spec[65];      // specs of rules jw / G .. (jw + 63) / G
  int64_t c, jw, jend;  // slice (-1: no more slices for this writer), first run, runs end
  int32_t k, nw;        // window k of the slice's nw windows
  int32_t seg0;         // jw % G (the first run's segment; spec[0] is rule jw / G)
};

__device__ __forceinline__ uint32_t lds_flag_get(const uint32_t* f) {
  return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_set(uint32_t* f, uint32_t v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads/writes are done
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// global -> LDS copy of `bytes` (a multiple of 4) by the whole wave, 256 B a round
__device__ __forceinline__ void lds_copy(void* lds, const void* g, int bytes) {
  const int lane = threadIdx.x & 63;
  for (int b = 0; b < bytes; b += 256)
    if (b + 4 * lane < bytes)
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const char*>(g) + b + 4 * lane,
                                       (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(lds) + b),
                                       4, 0, 0);
}

template <int V>
__global__ __launch_bounds__((kLwWriters + 1) * 64) __attribute__((amdgpu_waves_per_eu(CG_LW_WPE)))
void k_write_lw(
    const DSpec* __restrict__ specs, PlanArgs p, const int64_t* __restrict__ run_anchor,
    const int32_t* __restrict__ run_count, const uint32_t* __restrict__ run_dmask,
    const int64_t* __restrict__ run_off, int64_t nruns, int64_t* __restrict__ chunk_run,
    int64_t cap, int64_t* __restrict__ times) {
  __shared__ LwSlot slots[kLwWriters];
  __shared__ WinRun win_all[kLwWriters][64];
  __shared__ uint32_t flags[kLwWriters];  // 1: filled by the loader, 0: free
  extern __shared__ __align__(16) char dyn[];  // the plan's G segments
  Segment* segs = reinterpret_cast<Segment*>(dyn);
  for (int i = threadIdx.x; i < p.G * int(sizeof(Segment) / 8); i += blockDim.x)
    reinterpret_cast<int64_t*>(segs)[i] = reinterpret_cast<const int64_t*>(p.segs)[i];
  for (int i = threadIdx.x; i < kLwWriters; i += blockDim.x) flags[i] = 0u;
  __syncthreads();

  const int G = p.G;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t E = run_off[nruns];
  if (E > cap) return;  // output buffer too small: host grows it and relaunches
  const int sh = super_shift(cap);
  const int64_t sup = int64_t(1) << sh;
  const int64_t nsup = (E + sup - 1) >> sh;
  unsigned long long* dbg =
      reinterpret_cast<unsigned long long*>(chunk_run + (cap >> sh) + 2 + kTicketWords);

  if (wave == kLwWriters) {
    // ---- loader.  Lane w < kLwWriters keeps writer w's state, three stages
    // deep: a ticket (the slice after next), the next slice's map entries,
    // and the slice being copied window by window.  Each round issues every
    // stage's loads for every writer at once -- atomics, slice-map reads,
    // window copies -- and waits once.
    const int ng = gridDim.x < kTicketGroups ? int(gridDim.x) : kTicketGroups;
    unsigned int* tickets = reinterpret_cast<unsigned int*>(chunk_run + (cap >> sh) + 2);
    const bool steal = sh == CG_SUPER_SHIFT_LARGE;
    int cur = int(blockIdx.x % unsigned(ng)), hops = 0;
    int64_t c = 0, jw0 = 0, jend = 0;   // the slice being copied
    int32_t k = 0, nw = 0;              // its next window, its windows
    int64_t nc = 0, njw0 = 0, njend = 0;  // the next slice (has_nx)
    int64_t tk = 0;                       // a ticket's slice (has_tk)
    bool has_nx = false, has_tk = false, no_more = false;
    bool fin = lane >= kLwWriters;  // writer `lane` has been sent its end item
    uint32_t idle = 0, idle_total = 0;
    while (__ballot(!fin)) {
      const bool live = !fin;
      const bool ready = live && lds_flag_get(&flags[lane]) == 0u;  // writer's slot free
      if (live && k == nw && has_nx) {  // the next slice becomes current
        c = nc;
        jw0 = njw0;
        jend = njend;
        nw = int32_t((jend - jw0 + 63) >> 6);
        k = 0;
        has_nx = false;
      }
      const bool go = ready && k < nw;
      if (ready && k == nw && !has_nx && no_more) {  // nothing left: the end item
        slots[lane].c = -1;
        lds_flag_set(&flags[lane], 1u);
        fin = true;
      }
      bool busy = go;
      // slice map of the ticket taken last round
      if (live && !has_nx && has_tk) {
        has_tk = false;
        busy = true;
        if (tk < nsup) {
          nc = tk;
          njw0 = chunk_run[tk];           // run_off[njw0] <= tk << sh
          njend = chunk_run[tk + 1] + 1;  // the run holding the slice's end (or the last run)
          has_nx = true;
        } else if (steal && ++hops < ng) {  // this group is used up: move to the next one
          cur = cur + 1 == ng ? 0 : cur + 1;
        } else {
          no_more = true;
        }
      }
      // a ticket, one slice ahead of the slice map
      if (live && !has_tk && !no_more) {
        const unsigned int t = atomicAdd(tickets + cur * kTicketStride, 1u);
        tk = cur + int64_t(ng) * int64_t(t);
        has_tk = true;
        busy = true;
      }
      // window copies, every writer's, then one wait for everything above
      for (uint64_t m = __ballot(go); m; m &= m - 1) {
        const int w = __builtin_ctzll(m);
        const int64_t jw = rl64(jw0, w) + 64 * int64_t(rl32(k, w));
        const int64_t je = rl64(jend, w);
        const int n = int(je - jw < 64 ? je - jw : 64);
        const int64_t r0 = G == 1 ? jw : jw / G, r1 = G == 1 ? jw + n - 1 : (jw + n - 1) / G;
        LwSlot& s = slots[w];
        lds_copy(s.off, run_off + jw, 8 * n);
        lds_copy(s.anchor, run_anchor + jw, 8 * n);
        lds_copy(s.count, run_count + jw, 4 * n);
        lds_copy(s.dmask, run_dmask + jw, 4 * n);
        lds_copy(s.spec, specs + r0, int(sizeof(DSpec)) * int(r1 - r0 + 1));
        if (lane == 0) {
          s.c = rl64(c, w);
          s.jw = jw;
          s.jend = je;
          s.seg0 = int32_t(jw - r0 * G);
          s.k = rl32(k, w);
          s.nw = rl32(nw, w);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // copies, map reads and tickets have landed
      if (go) {
        lds_flag_set(&flags[lane], 1u);
        k++;
      }
      if (!__ballot(busy)) {
        if (++idle > kLwSpin) {
          if (lane == 0) atomicOr(dbg, 1ull);
          break;
        }
        if (V & 32) idle_total++;
        __builtin_amdgcn_s_sleep(1);
      } else {
        idle = 0;
      }
    }
    if ((V & 32) && lane == 0) atomicAdd(dbg + 1, (unsigned long long)idle_total);
    return;
  }

  // ---- writer wave: its slices' windows, in order
  WinRun* win = win_all[wave];
  uint32_t* f = &flags[wave];
  const LwSlot& s = slots[wave];
  Pending pd;
  pd.blk = -1;
  pd.val = 0;
  int64_t pos = 0, S1 = 0;
  uint32_t waits = 0;
  for (;;) {
    for (uint32_t n = 0; lds_flag_get(f) != 1u; n++) {
      if (n > kLwSpin) {
        if (lane == 0) atomicOr(dbg, 2ull);
        return;
      }
      if (V & 32) waits++;
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    const int64_t c = s.c;
    if (c < 0) break;
    const int32_t k = s.k, nw = s.nw;
    const int64_t jw = s.jw, jend = s.jend;
    // the slot -> this wave's window (k_write_cf's layout), then the slot is free
    // lane index re-derived each window: addresses built from it are not
    // hoisted out of the loop (and spilled: scratch reloads wait on vmcnt)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int64_t j = jw + ln;
    int64_t woff = INT64_MAX;
    int32_t wcnt = 0;
    // field by field (a WinRun temporary lands in scratch: vector-memory
    // traffic the writer would wait for behind its stores)
    WinRun& r = win[ln];
    if (j < jend) {
      // run j = rule (jw / G + q), segment x - q G with x = jw % G + lane
      const uint32_t x = uint32_t(s.seg0 + ln);
      uint32_t q = x;
      if (G > 1) {  // x < G + 64 < 2^24: f32 quotient, one correction each way
        const float inv = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(1.0f / float(G))));
        q = uint32_t(float(x) * inv);
        const int32_t rem = int32_t(x) - int32_t(q * uint32_t(G));
        q = rem < 0 ? q - 1u : (rem >= G ? q + 1u : q);
      }
      const DSpec& sp = s.spec[q];
      const uint32_t seg = x - q * uint32_t(G);
      woff = s.off[ln];
      wcnt = s.count[ln];
      r.anchor = s.anchor[ln];
      r.count = wcnt;
      r.dmask = s.dmask[ln];
      r.sp.sec = sp.sec;
      r.sp.min = sp.min;
      r.sp.hour = sp.hour;
      r.sp.dom = sp.dom;
      r.sp.mondow = sp.mondow;
      r.sp.kind = sp.kind | (seg << 8);
    } else {
      r.anchor = 0;
      r.count = 0;
      r.dmask = 0;
      r.sp.sec = 0;
      r.sp.min = 0;
      r.sp.hour = 0;
      r.sp.dom = 0;
      r.sp.mondow = 0;
      r.sp.kind = 0;
    }
    lds_flag_set(f, 0u);  // also waits for this lane's window write
    int i = 0;
    if (k == 0) {
      pos = c << sh;  // multiple of 64: every store below is a whole 512 B block
      S1 = E - pos < sup ? E : pos + sup;
      pd.blk = -1;
      pd.val = 0;
      i = 63 - __builtin_clzll(__ballot(woff <= pos));  // the run holding pos
    }
    while (pos < S1 && i < 64) {
      const int32_t cnt = rl32(wcnt, i);
      if (cnt == 0) {
        i++;
        continue;
      }
      const int64_t roff = rl64(woff, i);
      const int64_t p1 = roff + cnt < S1 ? roff + cnt : S1;
      const WinRun& w = win[i];
      const Segment& sg = segs[win_seg(w)];
      if (V & 8) {
      } else if (win_every(w)) {
        coop_every(w, roff, pos, p1, pd, times);
      } else if (run_is_walked(sg, w.dmask)) {
        drive<true>([]() { return int64_t(0); }, []() {}, pos, p1, pd, times);
      } else if (p1 - pos >= 64) {
        coop_cf(w, roff, sg, pos, p1, pd, times);
      } else {
        tiny_cf(w, roff, sg, pos, p1, pd, times);
      }
      pos = p1;
      i++;
    }
    if (k == nw - 1) {
      // the slice ends inside a block
      if (pd.blk >= 0 && pd.blk + lane < S1 && !(V & 8)) put(times + pd.blk + lane, pd.val);
      pd.blk = -1;
    }
    // every lane is done with this window before the next one overwrites it
    __builtin_amdgcn_wave_barrier();
  }
  if ((V & 32) && lane == 0) atomicAdd(dbg + 2, (unsigned long long)waits);
}

// diagnostic store ceiling (CG_WRITE_PROBE): fill the writer's slices of the
// output with W*8-byte-per-lane stores, 64 lanes contiguous
template <int W>
__global__ __launch_bounds__(kWriteWaves * 64) void k_fill_probe(const int64_t* __restrict__ run_off,
                                                                 int64_t nruns, int64_t cap,
                                                                 int64_t* __restrict__ times) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t E = run_off[nruns];
  if (E > cap) return;
  const int64_t kSup = int64_t(1) << super_shift(cap);
  if (W == 6 || W == 7) {  // per-wave streams with a pause (s_sleep) after every 24 stores
    const int64_t nsup = (E + kSup - 1) / kSup;
    const int64_t nwaves = int64_t(gridDim.x) * kWriteWaves;
    for (int64_t c = int64_t(blockIdx.x) * kWriteWaves + wave; c < nsup; c += nwaves) {
      const int64_t p0 = c * kSup, p1 = E - p0 < kSup ? E : p0 + kSup;
      int k = 0;
      for (int64_t b = p0 + lane; b < p1; b += 64) {
        times[b] = b;
        if (++k == 24) {
          k = 0;
          if (W == 6) __builtin_amdgcn_s_sleep(16);
          else __builtin_amdgcn_s_sleep(64);
        }
      }
    }
    return;
  }
  if (W == 4) {  // block-wide streams: the 4 waves interleave 512 B pieces of one slice
    const int64_t nsup = (E + kSup - 1) / kSup;
    for (int64_t c = blockIdx.x; c < nsup; c += gridDim.x) {
      const int64_t p0 = c * kSup, p1 = E - p0 < kSup ? E : p0 + kSup;
      for (int64_t b = p0 + wave * 64 + lane; b < p1; b += 64 * kWriteWaves) times[b] = b;
    }
    return;
  }
  const int64_t nsup = (E + kSup - 1) / kSup;
  const int64_t nwaves = int64_t(gridDim.x) * kWriteWaves;
  for (int64_t c = int64_t(blockIdx.x) * kWriteWaves + wave; c < nsup; c += nwaves) {
    const int64_t p0 = c * kSup + (W == 3 ? 8 : 0), p1 = E - c * kSup < kSup ? E : c * kSup + kSup;
    for (int64_t b = p0 + lane * (W == 3 ? 1 : W); b < p1; b += 64 * (W == 3 ? 1 : W)) {
      if (W == 2 && b + 1 < p1) {
        longlong2 v;
        v.x = b;
        v.y = b + 1;
        *reinterpret_cast<longlong2*>(times + b) = v;
      } else {
        times[b] = b;
      }
    }
  }
}

}  // namespace

bool launch_write_diag(const DSpec* specs, const PlanArgs& p, const int64_t* run_anchor, const int32_t* run_count,
                       const uint32_t* run_dmask, const int64_t* run_off, int64_t nruns, int64_t* chunk_run,
                       int64_t cap, int64_t* times, int n_blocks, size_t lds, hipStream_t st) {
  static const int probe = [] {
    const char* e = getenv("CG_WRITE_PROBE");
    return e ? atoi(e) : 0;
  }();
  static const int variant = [] {
    const char* e = getenv("CG_WRITE_VARIANT");
    return e ? atoi(e) : 0;
  }();
  const dim3 grid(n_blocks), block(kWriteWaves * 64);
  switch (probe) {
    case 1: hipLaunchKernelGGL(k_fill_probe<1>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    case 2: hipLaunchKernelGGL(k_fill_probe<2>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    case 3: hipLaunchKernelGGL(k_fill_probe<3>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    case 4: hipLaunchKernelGGL(k_fill_probe<4>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    case 5: (void)hipMemsetAsync(times, 0, size_t(cap) * 8, st); return true;
    case 6: hipLaunchKernelGGL(k_fill_probe<6>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    case 7: hipLaunchKernelGGL(k_fill_probe<7>, grid, block, 0, st, run_off, nruns, cap, times); return true;
    default: break;
  }
  if (variant != 255 && variant != 256) return false;
  // persistent k_write_lw grid: as many blocks per CU as its registers and LDS allow
  int n = 0;
  if (variant == 256)
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_write_lw<32>, (kLwWriters + 1) * 64, lds);
  else
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_write_lw<0>, (kLwWriters + 1) * 64, lds);
  const int blocks = std::max(1, n_blocks / kWriteBlocksPerCU) * std::max(n, 1);
  if (variant == 255) {
    hipLaunchKernelGGL(k_write_lw<0>, dim3(blocks), dim3((kLwWriters + 1) * 64), lds, st, specs, p, run_anchor,
                       run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
    return true;
  }
  hipLaunchKernelGGL(k_write_lw<32>, dim3(blocks), dim3((kLwWriters + 1) * 64), lds, st, specs, p, run_anchor,
                     run_count, run_dmask, run_off, nruns, chunk_run, cap, times);
  unsigned long long d[8];
  (void)hipMemcpyAsync(d, chunk_run + (cap >> super_shift(cap)) + 2 + kTicketWords, sizeof d, hipMemcpyDeviceToHost,
                       st);
  (void)hipStreamSynchronize(st);
  fprintf(stderr, "[k_write_lw stats] blocks=%d err=%llu loader idle rounds=%llu writer waits=%llu\n", blocks, d[0],
          d[1], d[2]);
  return true;
}

}  // namespace cg
