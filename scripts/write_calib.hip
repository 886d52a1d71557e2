// WRITE_SIZE calibration for psrt_trace's record stores (MI355X_MICROARCH.md
// §HBM: WRITE_SIZE is exact only for 16-B-per-lane streaming stores; other
// widths need a calibration on a known byte count). Each kernel writes a
// known number of bytes with one access pattern; rocprofv3 --pmc WRITE_SIZE
// reports what the counter makes of it.
//
//   hipcc --offload-arch=gfx950 -O3 -o write_calib scripts/write_calib.hip
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d out -o run -- ./write_calib
//
// Kernels (N records; t: 8 B, k: 2 B, as psrt_trace's samples buffer):
//   lin16   16-B stores, lane-consecutive (the calibrated reference): 16 N B
//   lin8    8-B t stores, lane-consecutive: 8 N B
//   lin2    2-B k stores, lane-consecutive: 2 N B
//   lin10   t and k stores, lane-consecutive (psrt_trace's layout): 10 N B
//   perm10  t and k, each wave writing its 1024-unit window in a scrambled
//           order over 16 rounds of 64 (finish order): 10 N B
//   nt10    as perm10 with non-temporal stores (psrt_trace's stores)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); std::exit(1); } } while (0)

constexpr unsigned kWin = 1024;  // units per wave window

__global__ void lin16(double2* p, unsigned n) {
  const unsigned u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) p[u] = make_double2(u, u);
}
__global__ void lin8(double* t, unsigned n) {
  const unsigned u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) t[u] = u;
}
__global__ void lin2(unsigned short* k, unsigned n) {
  const unsigned u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) k[u] = (unsigned short)u;
}
__global__ void lin10(double* t, unsigned short* k, unsigned n) {
  const unsigned u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u < n) {
    t[u] = u;
    k[u] = (unsigned short)u;
  }
}
// one wave per window of kWin units; round r, lane l writes unit
// base + perm(r * 64 + l), perm a bijection of [0, kWin) that scatters
// consecutive slots across the window
template <bool kNT>
__global__ void perm10(double* t, unsigned short* k, unsigned n) {
  const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64, lane = threadIdx.x % 64;
  const unsigned base = wave * kWin;
  for (unsigned r = 0; r < kWin / 64; ++r) {
    const unsigned s = r * 64 + lane;
    const unsigned off = (s * 389u) % kWin;  // 389 odd: a bijection mod 1024
    const unsigned u = base + off;
    if (u < n) {
      if (kNT) {
        __builtin_nontemporal_store((double)u, t + u);
        __builtin_nontemporal_store((unsigned short)u, k + u);
      } else {
        t[u] = u;
        k[u] = (unsigned short)u;
      }
    }
  }
}

int main() {
  const unsigned n = 96u << 20;  // ~ a C3 frame's samples (96 M)
  double* t;
  unsigned short* k;
  double2* w;
  CHECK(hipMalloc(&t, (size_t)n * 8));
  CHECK(hipMalloc(&k, (size_t)n * 2));
  CHECK(hipMalloc(&w, (size_t)n * 16));
  const unsigned b = 256, g = (n + b - 1) / b;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(lin16, dim3(g), dim3(b), 0, 0, w, n);
    hipLaunchKernelGGL(lin8, dim3(g), dim3(b), 0, 0, t, n);
    hipLaunchKernelGGL(lin2, dim3(g), dim3(b), 0, 0, k, n);
    hipLaunchKernelGGL(lin10, dim3(g), dim3(b), 0, 0, t, k, n);
    const unsigned waves = (n + kWin - 1) / kWin, gp = (waves * 64 + b - 1) / b;
    hipLaunchKernelGGL(perm10<false>, dim3(gp), dim3(b), 0, 0, t, k, n);
    hipLaunchKernelGGL(perm10<true>, dim3(gp), dim3(b), 0, 0, t, k, n);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  std::printf("n = %u records: lin16 %.3f GB, lin8 %.3f GB, lin2 %.3f GB, lin10/perm10/nt10 %.3f GB\n",
              n, n * 16e-9, n * 8e-9, n * 2e-9, n * 10e-9);
  CHECK(hipFree(t));
  CHECK(hipFree(k));
  CHECK(hipFree(w));
  return 0;
}
