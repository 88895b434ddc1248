// Lane order of same-address LDS atomics (diagnostic, not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -o tools/lds_order tools/lds_order.hip && ./tools/lds_order
// The radix scatter ranks a wave's elements by digit with one ballot per digit bit
// (kmhg_build_v2.hip match_bits) so that equal digits keep lane order (a stable pass).  If a
// returning ds_add_u32 whose lanes hit the same address hands out the old values in increasing
// lane order, the count atomic alone gives those ranks.  This checks that property on random
// digits: for every instruction and every digit, the returned values must increase with the
// lane id; any violation is counted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint32_t xs(uint32_t x) {
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  return x;
}

template <int R>
__global__ void __launch_bounds__(256) k_order(unsigned long long* bad, unsigned long long* checked,
                                               uint32_t seed, int iters) {
  __shared__ uint32_t cnt[4][R];
  __shared__ uint32_t got[4][64];
  __shared__ uint32_t dig[4][64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t r = xs(seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u) | 1u;
  unsigned long long nbad = 0, nchk = 0;
  for (int it = 0; it < iters; ++it) {
    for (int d = lane; d < R; d += 64) cnt[w][d] = 0;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    r = xs(r);
    // skewed digits: half the lanes pick among the first 4 values (many conflicts)
    const uint32_t d = (r & 1) ? (r >> 8) % 4 : (r >> 8) % R;
    const bool act = ((r >> 20) & 7) != 0;             // some lanes inactive
    uint32_t v = 0;
    if (act) v = atomicAdd(&cnt[w][d], 1u);
    got[w][lane] = act ? v : 0xFFFFFFFFu;
    dig[w][lane] = d;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    // lane l checks against every lower lane with the same digit
    if (act) {
      for (int m = 0; m < lane; ++m) {
        if (got[w][m] != 0xFFFFFFFFu && dig[w][m] == d) {
          ++nchk;
          if (got[w][m] > v) ++nbad;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  atomicAdd(bad, nbad);
  atomicAdd(checked, nchk);
}

template <int R>
void run(int wgs_per_cu) {
  unsigned long long *bad, *chk;
  hipMalloc(&bad, 8);
  hipMalloc(&chk, 8);
  hipMemset(bad, 0, 8);
  hipMemset(chk, 0, 8);
  hipLaunchKernelGGL(k_order<R>, dim3(256 * wgs_per_cu), dim3(256), 0, 0, bad, chk, 12345u, 200);
  unsigned long long hb = 0, hc = 0;
  hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost);
  hipMemcpy(&hc, chk, 8, hipMemcpyDeviceToHost);
  printf("R %4d  %d WG/CU: same-digit lane pairs checked %llu, out of lane order %llu\n", R,
         wgs_per_cu, hc, hb);
  hipFree(bad);
  hipFree(chk);
}

int main() {
  run<8>(4);
  run<99>(4);
  run<313>(4);
  run<8>(8);
  return 0;
}
