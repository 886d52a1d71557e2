// Co-residency probe (measurement only; DESIGN.md §7 "frames in flight"):
// can a small kernel's workgroups start on CUs that a persistent psrt_trace
// launch fills (6 waves per SIMD at 80 VGPRs, ~150 KB of LDS per CU)?
// probe_stamp: one 64-thread workgroup per entry writes s_memrealtime
// (100 MHz) at its start and spins `spin` ticks, so a caller sees when each
// workgroup got a slot. Built into gpurun_out by session Q (scripts/ARCHIVE.md,
// hipcc -shared) and loaded with ctypes by scripts/coresident_probe.py.
#include <hip/hip_runtime.h>

__global__ __launch_bounds__(64) void probe_stamp(unsigned long long* out, unsigned spin) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (spin) {
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = t0;
}

__global__ __launch_bounds__(64) void probe_stamp_prio(unsigned long long* out, unsigned spin) {
  __builtin_amdgcn_s_setprio(3);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (spin) {
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  }
  if (threadIdx.x == 0) out[blockIdx.x] = t0;
}

// psrt_reduce_lean's loop (a lane per pixel, four samples per step) on
// synthetic records, with each workgroup's start and end stamps: is it the
// loads or the issue that slows it beside a trace?
__global__ __launch_bounds__(64) void probe_reduce(const double* t, const unsigned short* k,
                                                   unsigned S, unsigned pixels,
                                                   unsigned long long* stamps, double* sums,
                                                   int prio) {
  if (prio) __builtin_amdgcn_s_setprio(3);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned q = blockIdx.x * 64 + threadIdx.x;
  double r = 0.0, g = 0.0, b = 0.0;
  if (q < pixels) {
    const double2* tp = (const double2*)(t + (size_t)q * S);
    const uint2* kp = (const uint2*)(k + (size_t)q * S);
    auto add = [&](double tt, unsigned kk) {
      const bool blk = kk == 0xffffu;
      const double w = 1.0 - tt;
      const double cr = __builtin_ldexp(w + tt * 0.5, -(int)kk);
      const double cg = __builtin_ldexp(w + tt * 0.7, -(int)kk);
      const double cb = __builtin_ldexp(w + tt * 1.0, -(int)kk);
      r += blk ? 0.0 : cr;
      g += blk ? 0.0 : cg;
      b += blk ? 0.0 : cb;
      __builtin_amdgcn_sched_barrier(0);
    };
#pragma unroll 1
    for (unsigned st = 0; st < S / 4; ++st) {
      const double2 t0v = tp[2 * st], t1v = tp[2 * st + 1];
      const uint2 kk = kp[st];
      add(t0v.x, kk.x & 0xffffu);
      add(t0v.y, kk.x >> 16);
      add(t1v.x, kk.y & 0xffffu);
      add(t1v.y, kk.y >> 16);
    }
    sums[q] = r + g + b;
  }
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t0;
    stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

extern "C" int probe_reduce_launch(void* stream, const double* t, const unsigned short* k,
                                   unsigned S, unsigned pixels, unsigned long long* stamps,
                                   double* sums, int prio) {
  hipLaunchKernelGGL(probe_reduce, dim3((pixels + 63) / 64), dim3(64), 0, (hipStream_t)stream, t,
                     k, S, pixels, stamps, sums, prio);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// N floats held live in VGPRs across the spin: which register counts still
// fit beside a resident trace?
template <int N>
__global__ __launch_bounds__(64) void probe_vgpr(unsigned long long* out, unsigned spin) {
  float v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = (float)(threadIdx.x * (i + 1));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
    __builtin_amdgcn_s_sleep(2);
  }
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < N; ++i) sum += v[i];
  if (threadIdx.x == 0) out[blockIdx.x] = t0 + (sum < -1.f ? 1 : 0);
}

extern "C" int probe_vgpr_launch(void* stream, unsigned long long* out, int nwg, unsigned spin,
                                 int n) {
  auto st = (hipStream_t)stream;
  switch (n) {
    case 8: hipLaunchKernelGGL(probe_vgpr<8>, dim3(nwg), dim3(64), 0, st, out, spin); break;
    case 14: hipLaunchKernelGGL(probe_vgpr<14>, dim3(nwg), dim3(64), 0, st, out, spin); break;
    case 20: hipLaunchKernelGGL(probe_vgpr<20>, dim3(nwg), dim3(64), 0, st, out, spin); break;
    case 26: hipLaunchKernelGGL(probe_vgpr<26>, dim3(nwg), dim3(64), 0, st, out, spin); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// N uniform ints held live in SGPRs across the spin
template <int N>
__global__ __launch_bounds__(64) void probe_sgpr(unsigned long long* out, unsigned spin, int seed) {
  int v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) v[i] = seed * (i + 3);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+s"(v[i]));
    __builtin_amdgcn_s_sleep(2);
  }
  int sum = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) sum += v[i];
  if (threadIdx.x == 0) out[blockIdx.x] = t0 + (sum == 12345 ? 1 : 0);
}

extern "C" int probe_sgpr_launch(void* stream, unsigned long long* out, int nwg, unsigned spin,
                                 int n) {
  auto st = (hipStream_t)stream;
  switch (n) {
    case 4: hipLaunchKernelGGL(probe_sgpr<4>, dim3(nwg), dim3(64), 0, st, out, spin, nwg); break;
    case 12: hipLaunchKernelGGL(probe_sgpr<12>, dim3(nwg), dim3(64), 0, st, out, spin, nwg); break;
    case 20: hipLaunchKernelGGL(probe_sgpr<20>, dim3(nwg), dim3(64), 0, st, out, spin, nwg); break;
    case 28: hipLaunchKernelGGL(probe_sgpr<28>, dim3(nwg), dim3(64), 0, st, out, spin, nwg); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int probe_launch(void* stream, unsigned long long* out, int nwg, unsigned spin, int prio) {
  if (nwg <= 0) return -1;
  if (prio)
    hipLaunchKernelGGL(probe_stamp_prio, dim3(nwg), dim3(64), 0, (hipStream_t)stream, out, spin);
  else
    hipLaunchKernelGGL(probe_stamp, dim3(nwg), dim3(64), 0, (hipStream_t)stream, out, spin);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
