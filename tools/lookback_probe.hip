// Look-back probe (diagnostic, not part of the library): can a radix scatter pass take its
// per-tile digit offsets from a decoupled look-back instead of a histogram pass + scan
// ("one-sweep digit offsets")?
//   hipcc --offload-arch=gfx950 -O3 -o tools/lookback_probe tools/lookback_probe.hip
//   ./tools/lookback_probe
// Persistent workgroups take tiles by ticket.  Per tile: `pre` ns of simulated work (the
// scatter's loads and digit counts), publish R aggregate words (flag | count, one u32 per
// digit, relaxed agent-scope stores), look back per digit until an inclusive word, publish the
// inclusive words, then `post` ns (the reorder and write-out).  Reported: the kernel time against
// the no-look-back ideal (tiles per workgroup x (pre + post)), the mean look-back hops per digit,
// and a check that every inclusive prefix is exact.
//   MODE 0: one thread per digit, one predecessor per round trip (serial chain)
//   MODE 1: one wave per digit at a time, 64 predecessors per round trip (CUB-style window)
//   MODE 8 / 16: one thread per digit, 8 / 16 predecessors per round trip (loads in flight)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); std::exit(1); } } while (0)

constexpr uint32_t FA = 1u << 30, FP = 2u << 30, VMASK = (1u << 30) - 1;
constexpr uint32_t AGG = 26;                      // every tile's count per digit

__device__ __forceinline__ uint32_t ldr(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void str(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void spin_ns(uint32_t ns) {
  if (!ns) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();       // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ns / 10) __builtin_amdgcn_s_sleep(2);
}

template <int MODE>
__global__ void __launch_bounds__(256) k_lb(uint32_t* __restrict__ status, uint32_t* __restrict__ ticket,
                                            uint32_t ntiles, uint32_t R, uint32_t pre, uint32_t post,
                                            unsigned long long* __restrict__ stats) {
  __shared__ uint32_t tsh;
  unsigned long long hops = 0, bad = 0;
  for (;;) {
    if (threadIdx.x == 0) tsh = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t t = tsh;
    __syncthreads();
    if (t >= ntiles) break;
    spin_ns(pre);
    for (uint32_t d = threadIdx.x; d < R; d += 256)
      str(&status[(size_t)t * R + d], (t == 0 ? FP : FA) | AGG);
    if (MODE == 0) {
      for (uint32_t d = threadIdx.x; d < R && t > 0; d += 256) {
        uint32_t sum = 0;
        int64_t j = (int64_t)t - 1;
        while (j >= 0) {
          const uint32_t w = ldr(&status[(size_t)j * R + d]);
          if ((w >> 30) == 0) { __builtin_amdgcn_s_sleep(1); continue; }
          sum += w & VMASK;
          ++hops;
          if ((w >> 30) == 2) break;
          --j;
        }
        bad += sum != AGG * t;
        str(&status[(size_t)t * R + d], FP | (sum + AGG));
      }
    } else if (MODE >= 2 && t > 0) {
      for (uint32_t d = threadIdx.x; d < R; d += 256) {
        uint32_t sum = 0;
        int64_t base = (int64_t)t - 1;
        for (;;) {
          uint32_t w[MODE >= 2 ? MODE : 1];
#pragma unroll
          for (int q = 0; q < (MODE >= 2 ? MODE : 1); ++q) {
            const int64_t j = base - q;
            w[q] = j >= 0 ? ldr(&status[(size_t)j * R + d]) : FP;
          }
          // consume up to the first inclusive word; stop at the first word not yet published
          uint32_t part = 0;
          int q = 0;
          bool done = false;
          for (; q < (MODE >= 2 ? MODE : 1); ++q) {
            const uint32_t f = w[q] >> 30;
            if (f == 0) break;
            part += w[q] & VMASK;
            if (f == 2) { done = true; ++q; break; }
          }
          sum += part;
          base -= q;
          ++hops;
          if (done) break;
          if (q < MODE) __builtin_amdgcn_s_sleep(1);
        }
        bad += sum != AGG * t;
        str(&status[(size_t)t * R + d], FP | (sum + AGG));
      }
    } else if (MODE == 1 && t > 0) {
      const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
      for (uint32_t d = wave; d < R; d += 4) {
        uint32_t sum = 0;
        int64_t base = (int64_t)t - 1;
        for (;;) {
          const int64_t j = base - lane;
          const uint32_t w = j >= 0 ? ldr(&status[(size_t)j * R + d]) : FP;
          const uint32_t f = w >> 30;
          const uint64_t m0 = __ballot(f == 0), m2 = __ballot(f == 2);
          const int first2 = m2 ? __ffsll((unsigned long long)m2) - 1 : 64;
          const uint64_t need = first2 == 64 ? ~0ull : ((2ull << first2) - 1ull);
          if (m0 & need) { __builtin_amdgcn_s_sleep(1); continue; }
          uint32_t v = lane <= first2 ? (w & VMASK) : 0u;
          for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
          sum += v;
          hops += lane == 0;
          if (first2 < 64) break;
          base -= 64;
        }
        if (lane == 0) {
          bad += sum != AGG * t;
          str(&status[(size_t)t * R + d], FP | (sum + AGG));
        }
      }
    }
    __syncthreads();
    spin_ns(post);
  }
  atomicAdd(&stats[0], hops);
  atomicAdd(&stats[1], bad);
}

template <int MODE>
static void run(uint32_t ntiles, uint32_t R, uint32_t pre, uint32_t post, int wg_per_cu) {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t G = (uint32_t)cus * wg_per_cu;
  uint32_t *status, *ticket;
  unsigned long long* stats;
  CK(hipMalloc(&status, (size_t)ntiles * R * 4));
  CK(hipMalloc(&ticket, 4));
  CK(hipMalloc(&stats, 16));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float best = 1e30f;
  unsigned long long h[2] = {0, 0};
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipMemset(status, 0, (size_t)ntiles * R * 4));
    CK(hipMemset(ticket, 0, 4));
    CK(hipMemset(stats, 0, 16));
    CK(hipEventRecord(a));
    hipLaunchKernelGGL(k_lb<MODE>, dim3(G), dim3(256), 0, 0, status, ticket, ntiles, R, pre, post, stats);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (ms < best) best = ms;
    CK(hipMemcpy(h, stats, 16, hipMemcpyDeviceToHost));
  }
  const double ideal = (double)((ntiles + G - 1) / G) * (pre + post) * 1e-6;
  std::printf("{\"mode\": %d, \"ntiles\": %u, \"R\": %u, \"wg\": %u, \"pre_ns\": %u, \"post_ns\": %u, "
              "\"ms\": %.4f, \"ideal_ms\": %.4f, \"hops_per_digit\": %.2f, \"errors\": %llu}\n",
              MODE, ntiles, R, G, pre, post, best, ideal,
              (double)h[0] / ((double)(ntiles - 1) * R), h[1]);
  CK(hipFree(status));
  CK(hipFree(ticket));
  CK(hipFree(stats));
}

int main() {
  // 500 Mbp k = 31: 244,141 tiles per pass, radix 79, a 4.0 ms pass at 3 workgroups per CU
  // (~12.6 us per tile); config 3: 48,829 tiles, radix 313, 0.88 ms
  struct Case { uint32_t nt, R, pre, post; } cases[] = {
      {244141, 79, 0, 0}, {244141, 79, 5000, 7500}, {244141, 79, 2500, 3700},
      {48829, 313, 0, 0}, {48829, 313, 5000, 8500}};
  for (const Case& c : cases) {
    run<0>(c.nt, c.R, c.pre, c.post, 3);
    run<8>(c.nt, c.R, c.pre, c.post, 3);
    run<16>(c.nt, c.R, c.pre, c.post, 3);
  }
  return 0;
}
