// CU-mask probe (diagnostic tool): which CUs run the blocks of kernels
// launched on two CU-masked streams (every 8th CU vs the rest), and whether
// a short kernel on the small set progresses while a long persistent kernel
// holds the large set.   hipcc -O3 --offload-arch=gfx950 -o cumask_probe cumask_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <vector>

__global__ void k_where(int* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = int(__smid());
}
__global__ void k_spin(unsigned long long cycles) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  while (__builtin_amdgcn_s_memtime() - t0 < cycles) __builtin_amdgcn_s_sleep(8);
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint32_t words = (cus + 31) / 32;
  std::vector<uint32_t> mw(words, 0u), ms(words, 0u);
  for (int i = 0; i < cus; i++) (i % 8 == 7 ? ms : mw)[i / 32] |= 1u << (i % 32);
  hipStream_t sw, ss;
  if (hipExtStreamCreateWithCUMask(&sw, words, mw.data()) != hipSuccess ||
      hipExtStreamCreateWithCUMask(&ss, words, ms.data()) != hipSuccess) {
    printf("mask stream creation failed\n");
    return 1;
  }
  int* d = nullptr;
  const int nb = 4096;
  (void)hipMalloc(&d, nb * sizeof(int));
  std::vector<int> h(nb);
  for (hipStream_t s : {sw, ss}) {
    hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    (void)hipMemcpy(h.data(), d, nb * sizeof(int), hipMemcpyDeviceToHost);
    std::set<int> ids(h.begin(), h.end());
    printf("stream %s: %zu distinct CU ids (min %d max %d)\n", s == sw ? "large" : "small", ids.size(), *ids.begin(),
           *ids.rbegin());
  }
  // a long kernel filling the large set, then a short one on the small set
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(k_spin, dim3(cus * 8), dim3(256), 0, sw, 100000000ull);  // ~1 s at 100 MHz memtime
  (void)hipEventRecord(a, ss);
  hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, ss, d);
  (void)hipEventRecord(b, ss);
  (void)hipEventSynchronize(b);
  float ms_small = 0;
  (void)hipEventElapsedTime(&ms_small, a, b);
  (void)hipStreamSynchronize(sw);
  printf("short kernel on the small set beside a long kernel on the large set: %.3f ms\n", ms_small);
  return 0;
}
