// tools/calib/fetch_calib.hip -- what rocprofv3's FETCH_SIZE reports per random 16-B read on gfx950
// (MI355X_MICROARCH.md: calibrated only for wide coalesced streams, where it reads 1/2 of the
// bytes).  The query probes read one random 16-B slot-tag group per miss; this measures the
// counter for exactly that access shape, beyond the Infinity Cache (a 4 GiB table):
//   k_stream   : every byte of a 1 GiB buffer once, 16 B per lane coalesced (known: 1 GiB)
//   k_random16 : N random 16-B aligned reads (one per lane) of a 4 GiB table
//   k_random4  : N random 4-B reads
// Build: hipcc -O3 --offload-arch=gfx950 -o fetch_calib fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

__global__ void k_stream(const uint4* __restrict__ a, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;       // never taken in practice; keeps the loads
}

__global__ void k_random16(const uint4* __restrict__ a, uint64_t n16, uint64_t nreads,
                           uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nreads; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = a[mix(i) % n16];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_random4(const uint32_t* __restrict__ a, uint64_t n4, uint64_t nreads,
                          uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < nreads; i += (uint64_t)gridDim.x * 256)
    acc ^= a[mix(i) % n4];
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t table = 4ull << 30, stream = 1ull << 30, nreads = 64ull << 20;
  void *t = nullptr, *o = nullptr;
  CK(hipMalloc(&t, table));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(t, 1, table));
  CK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    k_stream<<<4096, 256>>>((const uint4*)t, stream / 16, (uint32_t*)o);
    k_random16<<<4096, 256>>>((const uint4*)t, table / 16, nreads, (uint32_t*)o);
    k_random4<<<4096, 256>>>((const uint32_t*)t, table / 4, nreads, (uint32_t*)o);
  }
  CK(hipDeviceSynchronize());
  printf("{\"stream_bytes\": %llu, \"random_reads\": %llu, \"table_bytes\": %llu}\n",
         (unsigned long long)stream, (unsigned long long)nreads, (unsigned long long)table);
  CK(hipFree(t));
  CK(hipFree(o));
  return 0;
}
