// Store-pattern probe (diagnostic tool, not part of the library): times plain
// fills of one large HBM buffer in the access shapes the output-bound writers
// could use, beside hipMemsetAsync, to find the shape that reaches the store
// ceiling.   hipcc -O3 --offload-arch=gfx950 -o fill_patterns fill_patterns.hip
//   ./fill_patterns [GB=5.4] [reps=5]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef long long v2i64 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

// grid-stride: consecutive waves on consecutive 64*W*8-byte pieces (W = 1: 8 B/lane, 2: 16 B/lane)
template <int W, bool NT>
__global__ __launch_bounds__(256) void k_stride(long long* p, long long n) {
  const long long stride = (long long)gridDim.x * blockDim.x * W;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) * W; i < n; i += stride) {
    if (W == 2) {
      v2i64 v = {i, i + 1};
      if (NT) __builtin_nontemporal_store(v, (v2i64*)(p + i));
      else *(v2i64*)(p + i) = v;
    } else {
      if (NT) __builtin_nontemporal_store(i, p + i);
      else p[i] = i;
    }
  }
}

// per-wave slices of S events, handed out statically (wave w: slices w, w + nw, ...),
// 64*W events per store instruction
template <int W, bool NT>
__global__ __launch_bounds__(256) void k_slices(long long* p, long long n, int S) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * (blockDim.x / 64);
  const long long w = (long long)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
  for (long long c = w; c * S < n; c += nw) {
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + lane * W; i < e; i += 64 * W) {
      if (W == 2) {
        v2i64 v = {i, i + 1};
        if (NT) __builtin_nontemporal_store(v, (v2i64*)(p + i));
        else *(v2i64*)(p + i) = v;
      } else {
        if (NT) __builtin_nontemporal_store(i, p + i);
        else p[i] = i;
      }
    }
  }
}

// per-wave slices taken by ticket (one atomic per slice), as k_write_cf does
template <int W>
__global__ __launch_bounds__(256) void k_ticket(long long* p, long long n, int S, unsigned* ticket) {
  const int lane = threadIdx.x & 63;
  for (;;) {
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(ticket, 1u);
    const long long c = (long long)__builtin_amdgcn_readfirstlane((int)t);
    if (c * S >= n) break;
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + lane * W; i < e; i += 64 * W) {
      if (W == 2) {
        v2i64 v = {i, i + 1};
        *(v2i64*)(p + i) = v;
      } else {
        p[i] = i;
      }
    }
  }
}

// per-wave slices by ticket from G counters (blocks round-robin over the
// groups; group g hands out slices g, g + G, g + 2G, ...): k_write_cf's scheme
__global__ __launch_bounds__(256) void k_ticket_groups(long long* p, long long n, int S, unsigned* tickets, int G) {
  const int lane = threadIdx.x & 63;
  const int g = blockIdx.x % G;
  for (;;) {
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(tickets + g * 32, 1u);
    const long long c = g + (long long)G * __builtin_amdgcn_readfirstlane((int)t);
    if (c * S >= n) break;
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + lane; i < e; i += 64) p[i] = i;
  }
}

// range tickets: group g (blocks b with b % G == g) owns the contiguous slice
// range [g Q, (g + 1) Q) and hands it out in order; a wave whose group is used
// up moves on to the next group's counter (until every group is used up)
__global__ __launch_bounds__(256) void k_range_tickets(long long* p, long long n, int S, unsigned* tickets, int G) {
  const int lane = threadIdx.x & 63;
  const long long ns = (n + S - 1) / S, Q = (ns + G - 1) / G;
  int g = blockIdx.x % G, hops = 0;
  for (;;) {
    unsigned t = 0;
    if (lane == 0) t = atomicAdd(tickets + g * 32, 1u);
    const long long k = __builtin_amdgcn_readfirstlane((int)t);
    const long long c = g * Q + k;
    if (k >= Q || c >= ns) {
      if (++hops >= G) break;
      g = g + 1 == G ? 0 : g + 1;
      continue;
    }
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + lane; i < e; i += 64) p[i] = i;
  }
}

// static per-wave slices, XCD-grouped: the waves of XCD x (blocks x, x + 8, ...)
// take consecutive slices, so each XCD writes its own contiguous stretch per round
__global__ __launch_bounds__(256) void k_slices_xcd(long long* p, long long n, int S) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  const long long per_xcd = (long long)(gridDim.x / 8) * 4;
  const long long w = (long long)(blockIdx.x % 8) * per_xcd + (blockIdx.x / 8) * 4 + (threadIdx.x >> 6);
  for (long long c = w; c * S < n; c += nw) {
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + lane; i < e; i += 64) p[i] = i;
  }
}

// per-block slices: the block's 4 waves interleave 64*W-event pieces of one slice of S events
template <int W>
__global__ __launch_bounds__(256) void k_block_slices(long long* p, long long n, int S) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (long long c = blockIdx.x; c * S < n; c += gridDim.x) {
    const long long e = (c + 1) * S < n ? (c + 1) * S : n;
    for (long long i = c * S + (wave * 64 + lane) * W; i < e; i += 256 * W) {
      if (W == 2) {
        v2i64 v = {i, i + 1};
        *(v2i64*)(p + i) = v;
      } else {
        p[i] = i;
      }
    }
  }
}

int main(int argc, char** argv) {
  const double gb = argc > 1 ? atof(argv[1]) : 5.4;
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const long long n = (long long)(gb * 1e9 / 8) / 128 * 128;
  int cus = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  long long* p = nullptr;
  unsigned* ticket = nullptr;
  CHK(hipMalloc(&p, n * 8));
  CHK(hipMalloc(&ticket, 64 * 32 * 4));
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  auto timeit = [&](const char* name, auto&& launch) {
    launch();
    CHK(hipDeviceSynchronize());
    float best = 1e9f, sum = 0.f;
    for (int r = 0; r < reps; r++) {
      CHK(hipMemset(ticket, 0, 64 * 32 * 4));
      CHK(hipEventRecord(a));
      launch();
      CHK(hipEventRecord(b));
      CHK(hipEventSynchronize(b));
      float ms = 0.f;
      CHK(hipEventElapsedTime(&ms, a, b));
      sum += ms;
      best = ms < best ? ms : best;
    }
    CHK(hipGetLastError());
    printf("{\"pattern\": \"%s\", \"mean_ms\": %.4f, \"best_ms\": %.4f, \"TBps_mean\": %.3f}\n", name, sum / reps,
           best, n * 8 / (sum / reps) / 1e9);
    fflush(stdout);
  };
  timeit("hipMemsetAsync", [&] { CHK(hipMemsetAsync(p, 0, n * 8)); });
  for (int bpc : {1}) {
    char nm[128];
    snprintf(nm, sizeof nm, "stride 16B/lane %d blk/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stride<2, false>), dim3(cus * bpc), dim3(256), 0, 0, p, n); });
    snprintf(nm, sizeof nm, "stride 16B/lane nt %d blk/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stride<2, true>), dim3(cus * bpc), dim3(256), 0, 0, p, n); });
    snprintf(nm, sizeof nm, "stride 8B/lane %d blk/CU", bpc);
    timeit(nm, [&] { hipLaunchKernelGGL((k_stride<1, false>), dim3(cus * bpc), dim3(256), 0, 0, p, n); });
  }
  for (int S : {2048, 4096}) {
    for (int bpc : {4}) {
      char nm[128];
      snprintf(nm, sizeof nm, "wave slices S=%d 8B/lane %d blk/CU", S, bpc);
      timeit(nm, [&] { hipLaunchKernelGGL((k_slices<1, false>), dim3(cus * bpc), dim3(256), 0, 0, p, n, S); });
      snprintf(nm, sizeof nm, "32-group ticket slices S=%d 8B/lane %d blk/CU", S, bpc);
      timeit(nm, [&] { hipLaunchKernelGGL(k_ticket_groups, dim3(cus * bpc), dim3(256), 0, 0, p, n, S, ticket, 32); });
      for (int G : {8, 16, 32, 64}) {
        snprintf(nm, sizeof nm, "%d-range tickets S=%d 8B/lane %d blk/CU", G, S, bpc);
        timeit(nm, [&] { hipLaunchKernelGGL(k_range_tickets, dim3(cus * bpc), dim3(256), 0, 0, p, n, S, ticket, G); });
      }
    }
  }
  CHK(hipFree(p));
  return 0;
}
