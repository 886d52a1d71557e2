// Which XCD (HW_REG_XCC_ID) runs each block of a plain launch, against blockIdx % 8.
// hipcc --offload-arch=gfx950 -O2 -Wno-unused-value -o scripts/xcc_probe.bin scripts/xcc_probe.hip
#include <hip/hip_runtime.h>
__global__ void k(unsigned* out) {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  if (threadIdx.x == 0) out[blockIdx.x] = x;
}
int main() {
  unsigned* d; hipMalloc(&d, 4096 * 4);
  hipLaunchKernelGGL(k, dim3(4096), dim3(64), 0, 0, d);
  unsigned h[4096]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int match = 0, hist[16] = {0};
  for (int i = 0; i < 4096; ++i) { match += (h[i] & 15) == (unsigned)(i % 8); hist[h[i] & 15]++; }
  printf("blocks whose xcc == blockIdx %% 8: %d of 4096\n", match);
  for (int i = 0; i < 16; ++i) printf("%d ", hist[i]);
  printf("\nfirst 16: "); for (int i = 0; i < 16; ++i) printf("%u ", h[i]); printf("\n");
  return 0;
}
