// isa_rates.hip — diagnostic microbenchmark: issue cost of the VALU
// instruction classes the trace kernel is made of (FP64 add/mul/fma, the f64
// division/sqrt helpers, FP32, 32-bit integer multiply, 64-bit mad), on
// gfx950. Each kernel runs 8 independent chains of one instruction per lane,
// so the figure is throughput, not latency. Reported: cycles per
// wave-instruction on one SIMD, with 1 and with 8 waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 scripts/isa_rates.hip -o /tmp/isa_rates
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHAINS 8
#define UNROLL 16
#define ITERS 256

template <int kOp>
__global__ void __launch_bounds__(512) bench(unsigned long long* cyc, double* sink) {
  double d[CHAINS];
  float f[CHAINS];
  unsigned u[CHAINS];
  unsigned long long w[CHAINS];
  for (int c = 0; c < CHAINS; ++c) {
    d[c] = 1.0 + threadIdx.x * 1e-9 + c;
    f[c] = 1.0f + threadIdx.x * 1e-6f + c;
    u[c] = threadIdx.x * 2654435761u + c;
    w[c] = (unsigned long long)threadIdx.x * 0x9E3779B97F4A7C15ULL + c;
  }
  const double dy = 1.0000001;
  const float fy = 1.0000001f;
  const unsigned uy = 0x4C957F2Du;
  unsigned long long msk = __ballot(threadIdx.x & 1), mskw = 0;
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int k = 0; k < UNROLL; ++k) {
#pragma unroll
      for (int c = 0; c < CHAINS; ++c) {
        if constexpr (kOp == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dy));
        if constexpr (kOp == 1) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dy));
        if constexpr (kOp == 2) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d[c]) : "v"(dy));
        if constexpr (kOp == 3) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fy));
        if constexpr (kOp == 4) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(fy));
        if constexpr (kOp == 5) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 6)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w[c]) : "v"(u[c]), "v"(uy) : "vcc");
        if constexpr (kOp == 7) asm volatile("v_rcp_f64 %0, %0" : "+v"(d[c]));
        if constexpr (kOp == 8) asm volatile("v_rsq_f64 %0, %0" : "+v"(d[c]));
        if constexpr (kOp == 9) asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(d[c]) : "v"(u[c]));
        if constexpr (kOp == 10) asm volatile("v_ldexp_f64 %0, %0, %1" : "+v"(d[c]) : "v"(u[c]));
        if constexpr (kOp == 11) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 12) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 13) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(w[c]) : "v"(w[0]));
        if constexpr (kOp == 14) asm volatile("v_div_fixup_f64 %0, %0, %1, %1" : "+v"(d[c]) : "v"(dy));
        if constexpr (kOp == 15) asm volatile("v_cmp_gt_f64 vcc, %0, %1" ::"v"(d[c]), "v"(dy) : "vcc");
        if constexpr (kOp == 16) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(d[c]));
        if constexpr (kOp == 17) asm volatile("v_min_f64 %0, %0, %1" : "+v"(d[c]) : "v"(dy));
        if constexpr (kOp == 18) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(w[c]) : "v"(w[0]));
        if constexpr (kOp == 19) asm volatile("v_lshlrev_b64 %0, 7, %0" : "+v"(w[c]));
        if constexpr (kOp == 20) asm volatile("v_lshrrev_b64 %0, 9, %0" : "+v"(w[c]));
        if constexpr (kOp == 21) asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 22) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 23) asm volatile("v_xad_u32 %0, %0, %1, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 24) asm volatile("v_sqrt_f64 %0, %0" : "+v"(d[c]));
        if constexpr (kOp == 25) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 26) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 27) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(uy) : "vcc");
        if constexpr (kOp == 28) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[c]) : "v"(u[c]));
        if constexpr (kOp == 29) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 30) asm volatile("v_mov_b32 %0, %1" : "=v"(u[c]) : "v"(u[(c + 1) % CHAINS]));
        if constexpr (kOp == 31) asm volatile("v_cmp_gt_u32 vcc, %0, %1" ::"v"(u[c]), "v"(uy) : "vcc");
        if constexpr (kOp == 32) asm volatile("v_min_f32 %0, %0, %1" : "+v"(f[c]) : "v"(fy));
        if constexpr (kOp == 33) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(f[c]) : "v"(fy));
        if constexpr (kOp == 34) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(w[c]) : "v"(w[0]));
        if constexpr (kOp == 35) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 36) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(u[c]) : "v"(uy) : "vcc");
        if constexpr (kOp == 37) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(f[c]) : "v"(u[c]));
        if constexpr (kOp == 38) asm volatile("v_lshrrev_b32 %0, 7, %0" : "+v"(u[c]));
        if constexpr (kOp == 39) asm volatile("v_cmp_class_f64 vcc, %0, %1" ::"v"(d[c]), "v"(uy) : "vcc");
        if constexpr (kOp == 40) asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(d[c]) : "v"(dy) : "vcc");
        if constexpr (kOp == 41) asm volatile("v_div_fmas_f64 %0, %0, %1, %0" : "+v"(d[c]) : "v"(dy) : "vcc");
        if constexpr (kOp == 42) asm volatile("v_mov_b64 %0, %1" : "=v"(w[c]) : "v"(w[(c + 1) % CHAINS]));
        if constexpr (kOp == 44) asm volatile("v_cndmask_b32 %0, %0, %1, %2" : "+v"(u[c]) : "v"(uy), "s"(msk));
        if constexpr (kOp == 45) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(uy));
        if constexpr (kOp == 46) u[c] = (u[c] > uy) ? u[c] + uy : u[c] ^ uy;  // compiler-made cmp + select
        if constexpr (kOp == 47) asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(mskw) : "v"(u[c]), "v"(uy));
        if constexpr (kOp == 43) asm volatile("v_cndmask_b32 %0, %0, %1, vcc\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[c]) : "v"(uy) : "vcc");
      }
    }
  }
  unsigned long long t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  double acc = 0;
  for (int c = 0; c < CHAINS; ++c) acc += d[c] + f[c] + u[c] + (double)w[c];
  acc += (double)mskw;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x % 64 == 0) atomicMax(cyc, t1 - t0);
}

static const char* kNames[] = {"v_add_f64",    "v_mul_f64",     "v_fma_f64",     "v_add_f32",
                               "v_fma_f32",    "v_mul_lo_u32",  "v_mad_u64_u32", "v_rcp_f64",
                               "v_rsq_f64",    "v_cvt_f64_i32", "v_ldexp_f64",   "v_xor_b32",
                               "v_mul_hi_u32", "v_pk_fma_f32",  "v_div_fixup_f64", "v_cmp_gt_f64",
                               "v_cvt_f32_f64", "v_min_f64",    "v_lshl_add_u64",
                               "v_lshlrev_b64", "v_lshrrev_b64", "v_alignbit_b32", "v_lshl_add_u32",
                               "v_xad_u32",    "v_sqrt_f64",    "v_mul_u32_u24", "v_mad_u32_u24",
                               "v_cndmask_b32", "v_cvt_f64_u32", "v_add_u32", "v_mov_b32",
                               "v_cmp_gt_u32", "v_min_f32", "v_max3_f32", "v_pk_add_f32",
                               "v_and_b32", "v_add_co_u32", "v_cvt_f32_u32", "v_lshrrev_b32",
                               "v_cmp_class_f64", "v_div_scale_f64", "v_div_fmas_f64",
                               "v_mov_b64", "2x v_cndmask_b32", "v_cndmask_b32 s-mask",
                               "v_cndmask_b32_e32 vcc", "C select (cmp+cndmask+add+xor)",
                               "v_cmp_gt_u32 -> sgpr"};

static int g_first_op = 0;  // argv[1]: run only the ops from this one on

template <int kOp>
void run(int cus, double* sink, unsigned long long* dcyc) {
  if (kOp < g_first_op) return;
  const double n = (double)ITERS * UNROLL * CHAINS;
  double res[2];
  const int waves[3] = {1, 2, 8};
  double res3[3];
  for (int m = 0; m < 3; ++m) {
    // waves per SIMD x 4 SIMDs per CU; one 256-thread block = 1 wave per SIMD
    const int blocks = cus * waves[m];
    (void)hipMemset(dcyc, 0, sizeof *dcyc);
    hipLaunchKernelGGL(bench<kOp>, dim3(blocks), dim3(256), 0, 0, dcyc, sink);
    (void)hipDeviceSynchronize();
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dcyc, sizeof c, hipMemcpyDeviceToHost);
    // max over waves of its loop cycles; with w waves sharing a SIMD the SIMD
    // issued w * n instructions in that time
    res3[m] = (double)c / (n * waves[m]);
  }
  (void)res;
  std::printf("{\"insn\": \"%s\", \"cyc_per_wave_insn_1w\": %.3f, \"cyc_per_simd_insn_2w\": %.3f, "
              "\"cyc_per_simd_insn_8w\": %.3f}\n",
              kNames[kOp], res3[0], res3[1], res3[2]);
}

template <int... kOps>
void run_all(int cus, double* sink, unsigned long long* dcyc) {
  (run<kOps>(cus, sink, dcyc), ...);
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) {
    std::fprintf(stderr, "no device\n");
    return 1;
  }
  const int cus = p.multiProcessorCount;
  double* sink = nullptr;
  unsigned long long* dcyc = nullptr;
  if (hipMalloc(&sink, sizeof(double) * cus * 8 * 256) != hipSuccess ||
      hipMalloc(&dcyc, sizeof(unsigned long long)) != hipSuccess)
    return 1;
  run<0>(cus, sink, dcyc);  // warm-up (clocks)
  if (argc > 1) g_first_op = std::atoi(argv[1]);
  run_all<0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47>(cus, sink, dcyc);
  (void)hipFree(sink);
  (void)hipFree(dcyc);
  return 0;
}
