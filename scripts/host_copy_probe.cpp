// host_copy_probe.cpp — how fast can a frame's device buffers reach caller
// memory (DESIGN.md §7 "Host buffers")? Times the D2H of a
// C3 frame's outputs (23 MB of FP64 sums + 2.9 MB of bytes) into:
//   pageable   hipMemcpy into ordinary (pageable, already touched) memory
//   register   hipHostRegister the caller's buffer, hipMemcpy, unregister
//   bounce/T   hipMemcpyAsync into a pinned bounce buffer in row bands, each
//              band copied on to pageable memory by T host threads while the
//              next band's DMA runs
//   pinned     hipMemcpy into hipHostMalloc memory (a caller that allocates
//              its frame with rt_host_alloc)
// Build: hipcc -O2 -std=c++17 -o scripts/host_copy_probe scripts/host_copy_probe.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const size_t W = 1200, H = argc > 1 ? (size_t)std::atoi(argv[1]) : 800;
  const size_t bytes = W * H * 3 * 8 + W * H * 3;  // sums + write_color bytes
  const int reps = 10;
  void* d = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMemset(d, 1, bytes));
  CK(hipDeviceSynchronize());
  std::vector<unsigned char> page(bytes, 0);
  std::printf("{\"bytes\": %zu", bytes);
  auto report = [&](const char* name, double ms) {
    std::printf(", \"%s_ms\": %.4f, \"%s_GBps\": %.2f", name, ms, name, bytes / ms / 1e6);
  };
  auto best = [&](auto fn) {
    double b = 1e30;
    for (int r = 0; r < reps; ++r) {
      const double t0 = now_ms();
      fn();
      b = std::min(b, now_ms() - t0);
    }
    return b;
  };
  report("pageable", best([&] { CK(hipMemcpy(page.data(), d, bytes, hipMemcpyDeviceToHost)); }));
  report("register", best([&] {
           CK(hipHostRegister(page.data(), bytes, hipHostRegisterDefault));
           CK(hipMemcpy(page.data(), d, bytes, hipMemcpyDeviceToHost));
           CK(hipHostUnregister(page.data()));
         }));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int T : {1, 4, 8}) {
    for (size_t band : {(size_t)4 << 20, (size_t)8 << 20}) {
      unsigned char* pin[2];
      CK(hipHostMalloc((void**)&pin[0], band, hipHostMallocDefault));
      CK(hipHostMalloc((void**)&pin[1], band, hipHostMallocDefault));
      hipEvent_t ev[2];
      CK(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
      const double ms = best([&] {
        const size_t nb = (bytes + band - 1) / band;
        auto issue = [&](size_t b) {
          const size_t off = b * band, len = std::min(band, bytes - off);
          CK(hipMemcpyAsync(pin[b & 1], (const char*)d + off, len, hipMemcpyDeviceToHost, s));
          CK(hipEventRecord(ev[b & 1], s));
        };
        issue(0);
        for (size_t b = 0; b < nb; ++b) {
          CK(hipEventSynchronize(ev[b & 1]));
          if (b + 1 < nb) issue(b + 1);
          const size_t off = b * band, len = std::min(band, bytes - off);
          const size_t per = (len + T - 1) / T;
          std::vector<std::thread> th;
          for (int t = 1; t < T; ++t)
            th.emplace_back([&, t] {
              const size_t a = std::min(len, t * per), e = std::min(len, a + per);
              std::memcpy(page.data() + off + a, pin[b & 1] + a, e - a);
            });
          std::memcpy(page.data() + off, pin[b & 1], std::min(len, per));
          for (auto& x : th) x.join();
        }
      });
      char name[64];
      std::snprintf(name, sizeof name, "bounce%dMB_t%d", (int)(band >> 20), T);
      report(name, ms);
      CK(hipHostFree(pin[0]));
      CK(hipHostFree(pin[1]));
      CK(hipEventDestroy(ev[0]));
      CK(hipEventDestroy(ev[1]));
    }
  }
  unsigned char* pinned = nullptr;
  CK(hipHostMalloc((void**)&pinned, bytes, hipHostMallocDefault));
  report("pinned", best([&] { CK(hipMemcpy(pinned, d, bytes, hipMemcpyDeviceToHost)); }));
  // a pinned destination filled by an async copy on a non-blocking stream
  report("pinned_async", best([&] {
           CK(hipMemcpyAsync(pinned, d, bytes, hipMemcpyDeviceToHost, s));
           CK(hipStreamSynchronize(s));
         }));
  std::printf("}\n");
  CK(hipHostFree(pinned));
  CK(hipFree(d));
  return 0;
}
