// Probe: does ds_add_rtn_u32 (atomicAdd on LDS, return value used) hand out
// values in ascending lane order when several lanes of one wave hit the same
// address?  For every wave instruction: lanes with the same digit must get
// strictly increasing old values in lane order, continuing from the previous
// instruction.  Counts violations over many random and adversarial patterns.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_probe(const unsigned* __restrict__ digits, int items, int nbins, unsigned long long* bad) {
  __shared__ unsigned cnt[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane < 64) cnt[w][lane] = 0;
  __syncthreads();
  unsigned last[64];  // per digit, the expected next value (tracked per lane for its own digit only)
  const unsigned* d = digits + (size_t(blockIdx.x) * 4 + w) * items * 64;
  unsigned long long nb = 0;
  unsigned prev_rank = 0, prev_d = 0xffffffffu;
  (void)last;
  for (int j = 0; j < items; j++) {
    const unsigned dg = d[j * 64 + lane] % nbins;
    const unsigned r = atomicAdd(&cnt[w][dg], 1u);
    // expected: number of (earlier items, any lane) + (this item, lower lanes) with the same digit
    unsigned exp = 0;
    for (int jj = 0; jj <= j; jj++)
      for (int l = 0; l < 64; l++) {
        if (jj == j && l >= lane) break;
        exp += (d[jj * 64 + l] % nbins) == dg;
      }
    nb += r != exp;
  }
  (void)prev_rank; (void)prev_d;
  if (nb) atomicAdd(bad, nb);
}

int main() {
  const int blocks = 256, items = 16;
  const size_t n = size_t(blocks) * 4 * items * 64;
  unsigned* h = (unsigned*)malloc(n * 4);
  unsigned *dd; unsigned long long* bad;
  hipMalloc(&dd, n * 4); hipMalloc(&bad, 8);
  srand(12345);
  int total_bad = 0;
  for (int pat = 0; pat < 6; pat++) {
    for (size_t i = 0; i < n; i++) {
      switch (pat) {
        case 0: h[i] = 0; break;                           // every lane the same address
        case 1: h[i] = rand() % 2; break;
        case 2: h[i] = rand() % 64; break;
        case 3: h[i] = (i % 64) < 32 ? 5 : rand() % 64; break;
        case 4: h[i] = 63 - (i % 64) / 8; break;             // runs of 8 lanes, descending
        default: h[i] = rand() % 7; break;
      }
    }
    hipMemcpy(dd, h, n * 4, hipMemcpyHostToDevice);
    hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(k_probe, dim3(blocks), dim3(256), 0, 0, dd, items, 64, bad);
    unsigned long long b = 0;
    hipMemcpy(&b, bad, 8, hipMemcpyDeviceToHost);
    printf("pattern %d: %llu out-of-order ranks of %zu\n", pat, b, n);
    total_bad += b != 0;
  }
  printf(total_bad ? "LDS atomic ranks NOT in lane order\n" : "LDS atomic ranks in lane order on every pattern\n");
  return 0;
}
