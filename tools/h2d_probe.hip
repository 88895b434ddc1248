// Host -> device paths for a pageable host string (diagnostic, not part of the library): the
// R API's make.kmer.hash hands the library a pageable buffer of L chars.
//   hipcc --offload-arch=gfx950 -O3 -o tools/h2d_probe tools/h2d_probe.hip
//   ./tools/h2d_probe [MB]
// Each path runs on a fresh, written (faulted-in) malloc buffer, 8 reps, median printed:
//   pageable   hipMemcpyAsync from the pageable buffer (the runtime stages it)
//   register   hipHostRegister + hipMemcpyAsync + sync + hipHostUnregister
//   reg_only   hipHostRegister + hipHostUnregister (the pinning cost alone)
//   zerocopy   hipHostRegister + a kernel that reads the host pages over PCIe and writes HBM
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_pull(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                              size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    dst[i] = src[i];
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(
      std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::strtoul(argv[1], nullptr, 10) : 10;
  const size_t bytes = mb << 20;
  void* d = nullptr;
  CK(hipMalloc(&d, bytes));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  const char* names[4] = {"pageable", "register", "reg_only", "zerocopy"};
  for (int mode = 0; mode < 4; ++mode) {
    std::vector<double> t;
    for (int rep = 0; rep < 9; ++rep) {
      char* h = static_cast<char*>(std::malloc(bytes + 64));
      std::memset(h, 'A' + rep, bytes);                   // faulted in, as R's string is
      CK(hipStreamSynchronize(s));
      const double t0 = now_ms();
      if (mode == 0) {
        CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
      } else {
        CK(hipHostRegister(h, bytes, hipHostRegisterDefault));
        if (mode == 1) {
          CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
          CK(hipStreamSynchronize(s));
        } else if (mode == 3) {
          void* dp = nullptr;
          CK(hipHostGetDevicePointer(&dp, h, 0));
          hipLaunchKernelGGL(k_pull, dim3(1024), dim3(256), 0, s, static_cast<const uint4*>(dp),
                             static_cast<uint4*>(d), bytes / 16);
          CK(hipStreamSynchronize(s));
        }
        CK(hipHostUnregister(h));
      }
      const double t1 = now_ms();
      if (rep) t.push_back(t1 - t0);                     // rep 0 warms up
      std::free(h);
    }
    std::sort(t.begin(), t.end());
    const double med = t[t.size() / 2];
    std::printf("%-9s %5zu MB  median %.3f ms  min %.3f ms  %.1f GB/s\n", names[mode], mb, med,
                t.front(), bytes / med / 1e6);
  }
  CK(hipFree(d));
  return 0;
}
