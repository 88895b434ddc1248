// Write-pattern probe for the radix scatter passes (diagnostic, not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -o tools/scatter_pattern tools/scatter_pattern.hip
//   ./tools/scatter_pattern [n_elements]
// A radix pass writes each 2048-element tile as R digit runs: run d of tile t lands at
// base(d, t) = ntiles * tstart(d) + t * cnt(d) of the output (digit-major, tile-minor, like the
// scanned [digit][tile] histogram).  This kernel moves 12-B elements (u64 key + u32 position,
// two arrays, as the build's key streams) with exactly that output pattern and no other work,
// so the time per pass is the cost of the write pattern alone at each radix R.  Schedules:
// persistent workgroups over XCD-contiguous tile ranges (the build's), plain or nontemporal
// stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr int TB = 256, PT = 2048, PER = PT / TB;

__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, j = b >> 3;
  return x * q + (x < r ? x : r) + j;
}

// mode 0: persistent workgroups over XCD-contiguous tile ranges (the build's interleaved
// schedule); mode 1: chunked, workgroup w takes the consecutive tiles [w m, (w + 1) m).
// KEYS / POS: which of the two arrays is written (both read).
template <bool NT, int MODE = 0, bool KEYS = true, bool POS = true>
__global__ void __launch_bounds__(TB) k_pattern(const uint64_t* __restrict__ kin,
                                                const uint32_t* __restrict__ pin,
                                                uint64_t* __restrict__ kout,
                                                uint32_t* __restrict__ pout, uint32_t ntiles,
                                                uint32_t R) {
  const uint32_t G = gridDim.x;
  const uint32_t m = (ntiles + G - 1) / G;
  const uint32_t n_iter = MODE == 0 ? (ntiles - blockIdx.x + G - 1) / G
                                    : (blockIdx.x * m < ntiles ? min(m, ntiles - blockIdx.x * m) : 0u);
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t t = MODE == 0 ? xcd_remap(blockIdx.x + it * G, ntiles) : blockIdx.x * m + it;
    uint64_t k[PER];
    uint32_t p[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t e = (uint64_t)t * PT + j * TB + threadIdx.x;
      k[j] = kin[e];
      p[j] = pin[e];
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t i = j * TB + threadIdx.x;                 // sorted index inside the tile
      const uint32_t d = (uint32_t)(((uint64_t)i * R) / PT);    // its run
      const uint32_t ts = (uint32_t)(((uint64_t)d * PT + R - 1) / R);   // first index of run d
      const uint32_t te = (uint32_t)(((uint64_t)(d + 1) * PT + R - 1) / R);
      const uint64_t dst = (uint64_t)ntiles * ts + (uint64_t)t * (te - ts) + (i - ts);
      if (NT) {
        if (KEYS) __builtin_nontemporal_store(k[j], &kout[dst]);
        if (POS) __builtin_nontemporal_store(p[j], &pout[dst]);
      } else {
        if (KEYS) kout[dst] = k[j];
        if (POS) pout[dst] = p[j];
      }
    }
  }
}

// Element layouts (round 5): LAY 1 = one packed 12-B element {key lo, key hi, pos} per index
// (AoS, a run is one contiguous 12 c-byte piece instead of an 8 c- and a 4 c-byte piece in two
// arrays); LAY 2 = one 8-B element per index (a key stream with the position folded in); LAY 3 =
// 16-B elements {key, pos, pad}.
template <int LAY>
__global__ void __launch_bounds__(TB) k_layout(const uint64_t* __restrict__ kin,
                                               const uint32_t* __restrict__ pin,
                                               uint64_t* __restrict__ kout,
                                               uint32_t* __restrict__ pout, uint32_t ntiles,
                                               uint32_t R) {
  (void)pout;
  const uint32_t G = gridDim.x;
  const uint32_t n_iter = (ntiles - blockIdx.x + G - 1) / G;
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t t = xcd_remap(blockIdx.x + it * G, ntiles);
    uint64_t k[PER];
    uint32_t p[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint64_t e = (uint64_t)t * PT + j * TB + threadIdx.x;
      if (LAY == 1) {
        const uint3 v = reinterpret_cast<const uint3*>(kin)[e];
        k[j] = ((uint64_t)v.y << 32) | v.x;
        p[j] = v.z;
      } else if (LAY == 3) {
        const uint4 v = reinterpret_cast<const uint4*>(kin)[e];
        k[j] = ((uint64_t)v.y << 32) | v.x;
        p[j] = v.z;
      } else {
        k[j] = kin[e];
        p[j] = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t i = j * TB + threadIdx.x;
      const uint32_t d = (uint32_t)(((uint64_t)i * R) / PT);
      const uint32_t ts = (uint32_t)(((uint64_t)d * PT + R - 1) / R);
      const uint32_t te = (uint32_t)(((uint64_t)(d + 1) * PT + R - 1) / R);
      const uint64_t dst = (uint64_t)ntiles * ts + (uint64_t)t * (te - ts) + (i - ts);
      if (LAY == 1)
        reinterpret_cast<uint3*>(kout)[dst] = make_uint3((uint32_t)k[j], (uint32_t)(k[j] >> 32), p[j]);
      else if (LAY == 3)
        reinterpret_cast<uint4*>(kout)[dst] = make_uint4((uint32_t)k[j], (uint32_t)(k[j] >> 32), p[j], 0u);
      else
        kout[dst] = k[j] ^ p[j];
    }
  }
}

// Supertiles (round 4): workgroup w owns supertiles of S consecutive tiles and writes them one
// tile after another; the histogram unit is the supertile, so digit d's runs of the S tiles are
// adjacent in the output (one run of S * 2048 / R elements, written in S pieces by one
// workgroup a few microseconds apart) -- the layout a scatter with per-supertile histograms and
// running digit offsets in LDS would produce.
template <int S>
__global__ void __launch_bounds__(TB) k_super(const uint64_t* __restrict__ kin,
                                              const uint32_t* __restrict__ pin,
                                              uint64_t* __restrict__ kout,
                                              uint32_t* __restrict__ pout, uint32_t ntiles,
                                              uint32_t R) {
  const uint32_t G = gridDim.x;
  const uint32_t nsup = ntiles / S;
  for (uint32_t it = blockIdx.x; it < nsup; it += G) {
    const uint32_t T = xcd_remap(it, nsup);
    for (int sub = 0; sub < S; ++sub) {
      const uint32_t t = T * S + sub;
      uint64_t k[PER];
      uint32_t p[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint64_t e = (uint64_t)t * PT + j * TB + threadIdx.x;
        k[j] = kin[e];
        p[j] = pin[e];
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint32_t i = j * TB + threadIdx.x;
        const uint32_t d = (uint32_t)(((uint64_t)i * R) / PT);
        const uint32_t ts = (uint32_t)(((uint64_t)d * PT + R - 1) / R);
        const uint32_t te = (uint32_t)(((uint64_t)(d + 1) * PT + R - 1) / R);
        const uint64_t c = te - ts;                      // run length per tile
        const uint64_t dst = (uint64_t)nsup * S * ts + (uint64_t)T * S * c + sub * c + (i - ts);
        kout[dst] = k[j];
        pout[dst] = p[j];
      }
    }
  }
}

int main(int argc, char** argv) {
  const uint64_t n_req = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 100000000ull;
  const uint32_t ntiles = (uint32_t)(n_req / PT);
  const uint64_t n = (uint64_t)ntiles * PT;
  uint64_t *ka, *kb;
  uint32_t *pa, *pb;
  CK(hipMalloc(&ka, n * 16)); CK(hipMalloc(&kb, n * 16));   // LAY 3: 16 B per element
  CK(hipMalloc(&pa, n * 4)); CK(hipMalloc(&pb, n * 4));
  CK(hipMemset(ka, 1, n * 16)); CK(hipMemset(pa, 2, n * 4));
  int cus = 256, per = 1;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto run = [&](const void* kern, const char* tag, uint32_t R, int wpc, double bytes_per_elt) {
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, TB, 0));
    const uint32_t grid = (uint32_t)cus * (uint32_t)std::min(per, wpc);
    float best = 1e30f;
    for (int rep = 0; rep < 6; ++rep) {
      void* args[] = {&ka, &pa, &kb, &pb, (void*)&ntiles, &R};
      CK(hipEventRecord(e0));
      CK(hipLaunchKernel(kern, dim3(grid), dim3(TB), args, 0, 0));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) best = std::min(best, ms);
    }
    std::printf("%-22s wg/cu %d R %4u run %6.1f  %.3f ms  %.0f GB/s (%.0f B/elt)\n", tag,
                std::min(per, wpc), R, (double)PT / R, best, bytes_per_elt * n / (best * 1e-3) / 1e9,
                bytes_per_elt);
    std::fflush(stdout);
  };
  if (argc > 2 && std::string(argv[2]) == "layout") {
    for (uint32_t R : {1u, 47u, 79u, 156u, 313u}) {
      run((const void*)k_pattern<false, 0>, "SoA 8+4 (build)", R, 3, 24);
      run((const void*)k_layout<1>, "AoS 12 packed", R, 3, 24);
      run((const void*)k_layout<1>, "AoS 12 packed wg4", R, 4, 24);
      run((const void*)k_layout<2>, "8-B elements", R, 3, 16);
      run((const void*)k_layout<3>, "AoS 16", R, 3, 32);
    }
    return 0;
  }
  const uint32_t Rs[] = {1, 47, 156, 313};
  for (int wpc : {1, 2, 3})
    for (uint32_t R : Rs) {
      run((const void*)k_pattern<false, 0>, "interleaved", R, wpc, 24);
      run((const void*)k_pattern<false, 1>, "chunked", R, wpc, 24);
    }
  if (argc > 2 && std::string(argv[2]) == "super") {
    for (uint32_t R : {79u, 313u}) {
      run((const void*)k_super<1>, "super S=1", R, 4, 24);
      run((const void*)k_super<2>, "super S=2", R, 4, 24);
      run((const void*)k_super<4>, "super S=4", R, 4, 24);
      run((const void*)k_super<8>, "super S=8", R, 4, 24);
      run((const void*)k_super<4>, "super S=4 wg2", R, 2, 24);
    }
    return 0;
  }
  // aligned runs of G elements (R = 2048 / G): the write granularity each array needs
  for (uint32_t G : {2u, 4u, 8u, 16u, 32u, 64u}) {
    run((const void*)k_pattern<false, 0, true, false>, "keys-only aligned", PT / G, 3, 20);
    run((const void*)k_pattern<false, 0, false, true>, "pos-only aligned", PT / G, 3, 16);
  }
  return 0;
}
