// LDS atomic throughput / latency probe (diagnostic, not part of the library).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/lds_atomics tools/lds_atomics.hip && /tmp/lds_atomics
// A group bucket's pass A (kmhg_build_v2.hip) is 64-bit CAS + 32-bit add on a 1,536-slot LDS
// table; this measures what those instructions cost on their own, with the bucket kernel's
// occupancy (256 threads, ~25 KB LDS per workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int CAP = 1536;
constexpr int ITERS = 256;

__device__ __forceinline__ uint32_t xs(uint32_t x) {
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  return x;
}

// mode 0: CAS rtn on random slots (always fails: table full of non-EMPTY), independent
// mode 1: atomicAdd u32 (no return) random
// mode 2: plain ds_read_b64 random, independent (sum)
// mode 3: CAS rtn, dependent chain (next address from the returned value)
// mode 4: CAS rtn succeeding (each lane its own fresh slot region, always EMPTY first)
// mode 5: atomicAdd u32 with return, random
template <int MODE>
__global__ void __launch_bounds__(256) k(uint64_t* out, uint32_t seed) {
  __shared__ uint64_t key[CAP + 1];
  __shared__ uint2 cc[CAP + 1];
  for (int j = threadIdx.x; j <= CAP; j += 256) {
    key[j] = MODE == 4 ? ~0ull : (uint64_t)j * 0x9E3779B97F4A7C15ull;
    cc[j] = make_uint2(0, 0);
  }
  __syncthreads();
  uint32_t r = xs(seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u) | 1u;
  uint64_t acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    r = xs(r);
    uint32_t j = r % CAP;
    if (MODE == 0) {
      acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    } else if (MODE == 1) {
      atomicAdd(&cc[j].x, 1u);
    } else if (MODE == 2) {
      acc += key[j];
    } else if (MODE == 3) {
      j = (uint32_t)(acc + r) % CAP;
      acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    } else if (MODE == 4) {
      // slot unique per (lane, iteration) in this workgroup: 256 * ITERS > CAP, so wrap and
      // let later iterations fail -- first CAP/256 iterations succeed
      j = (threadIdx.x * 6 + i) % CAP;
      acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    } else if (MODE == 5) {
      acc += atomicAdd(&cc[j].x, 1u);
    } else if (MODE == 6) {            // CAS rtn fails, only 8 lanes of each wave active
      if ((threadIdx.x & 63) < 8)
        acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    } else if (MODE == 7) {            // CAS rtn fails, one lane per wave
      if ((threadIdx.x & 63) == 0)
        acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    } else if (MODE == 9) {            // 32-bit CAS rtn fails, 64 lanes
      acc += atomicCAS(&cc[j].y, 0xFFFFFFFFu, r);
    } else if (MODE == 8) {            // CAS rtn fails, 32 lanes
      if ((threadIdx.x & 63) < 32)
        acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)r);
    }
  }
  __syncthreads();
  if (acc == 12345) out[0] = acc + cc[threadIdx.x].x;
}

// Pass A of a group bucket in isolation: 1,024 random 62-bit keys (4 per thread, elements
// c * 256 + t) inserted into a 1,536-slot table by CAS with linear probing, plus the count add.
// VARIANT 0: element by element (the library's form); 1: per-lane state machine.
__device__ __forceinline__ uint64_t mixk(uint64_t h) {
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}
__device__ __forceinline__ uint32_t homek(uint64_t h) {
  return (uint32_t)((((uint64_t)((uint32_t)h >> 16)) * CAP) >> 16);
}
template <int VARIANT>
__global__ void __launch_bounds__(256) kpa(uint64_t* out, uint32_t seed, int reps) {
  __shared__ uint64_t key[CAP + 1];
  __shared__ uint2 cc[CAP + 1];
  __shared__ uint64_t qk[(VARIANT == 4 || VARIANT == 5) ? 4 : 1][256];   // per-wave failure queue
  __shared__ uint16_t qj[(VARIANT == 4 || VARIANT == 5) ? 4 : 1][256];
  uint64_t acc = 0;
  for (int rep = 0; rep < reps; ++rep) {
    for (int j = threadIdx.x; j <= CAP; j += 256) { key[j] = ~0ull; cc[j] = make_uint2(0, 0); }
    __syncthreads();
    uint64_t kv[4];
    for (int c = 0; c < 4; ++c)
      kv[c] = mixk(((uint64_t)(blockIdx.x * 4096 + rep * 1024 + c * 256 + threadIdx.x) << 1) ^ seed) >> 2;
    int slot[4];
    if (VARIANT == 0) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t j = homek(mixk(kv[c]));
        for (;;) {
          const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kv[c]);
          if (prev == ~0ull || prev == kv[c]) break;
          if (++j == CAP) j = 0;
        }
        slot[c] = j;
        atomicAdd(&cc[j].x, 1u);
      }
    } else if (VARIANT == 2) {
      uint32_t hm[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hm[q] = homek(mixk(kv[q]));
      int c = 0;
      uint64_t kk = kv[0];
      uint32_t j = hm[0];
      bool live = true;
      while (live) {
        const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
        if (prev == ~0ull || prev == kk) {
          atomicAdd(&cc[j].x, 1u);
#pragma unroll
          for (int q = 0; q < 4; ++q) if (q == c) slot[q] = j;
          if (++c == 4) live = false;
          else {
#pragma unroll
            for (int q = 1; q < 4; ++q) if (q == c) { kk = kv[q]; j = hm[q]; }
          }
        } else if (++j == CAP) j = 0;
      }
    } else if (VARIANT == 3) {
      // home round for every element, then the failures alone, element by element
      uint32_t hm[4];
      bool pend[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hm[q] = homek(mixk(kv[q]));
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint64_t prev = atomicCAS((unsigned long long*)&key[hm[q]], ~0ull, (unsigned long long)kv[q]);
        pend[q] = !(prev == ~0ull || prev == kv[q]);
        if (!pend[q]) { slot[q] = hm[q]; atomicAdd(&cc[hm[q]].x, 1u); }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!__any(pend[q])) continue;
        uint32_t j = hm[q];
        while (pend[q]) {
          if (++j == CAP) j = 0;
          const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kv[q]);
          if (prev == ~0ull || prev == kv[q]) { pend[q] = false; slot[q] = j; atomicAdd(&cc[j].x, 1u); }
        }
      }
    } else if (VARIANT == 4 || VARIANT == 5) {
      // home round for every element (one CAS each); the failures of each wave are compacted
      // into a per-wave LDS queue and probed on 64 at a time, so a long probe chain holds up
      // only the queue's lanes, not every element round.  The resolved slot goes back to the
      // owner through the queue (VARIANT 5: no write-back, owners re-find in pass B instead).
      const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
      int qi[4];
      uint32_t nq = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t h = homek(mixk(kv[q]));
        const uint64_t prev = atomicCAS((unsigned long long*)&key[h], ~0ull, (unsigned long long)kv[q]);
        const bool ok = prev == ~0ull || prev == kv[q];
        if (ok) { slot[q] = h; atomicAdd(&cc[h].x, 1u); }
        const uint64_t fm = __ballot(!ok);
        qi[q] = -1;
        if (!ok) {
          const uint32_t r = nq + (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
          qk[w][r] = kv[q];
          qj[w][r] = h + 1 == CAP ? 0 : h + 1;
          qi[q] = (int)r;
        }
        nq += (uint32_t)__popcll(fm);
      }
      __builtin_amdgcn_wave_barrier();
      for (uint32_t b0 = 0; b0 < nq; b0 += 64) {
        const uint32_t i = b0 + lane;
        if (i < nq) {
          const uint64_t kk = qk[w][i];
          uint32_t j = qj[w][i];
          for (;;) {
            const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
            if (prev == ~0ull || prev == kk) break;
            if (++j == CAP) j = 0;
          }
          atomicAdd(&cc[j].x, 1u);
          if (VARIANT == 4) qj[w][i] = (uint16_t)j;
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (qi[q] >= 0) slot[q] = VARIANT == 4 ? (int)qj[w][qi[q]] : -1;
    } else if (VARIANT == 7 || VARIANT == 8) {   // calibration: no CAS (7: count adds at home)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t j = homek(mixk(kv[c]));
        slot[c] = j;
        if (VARIANT == 7) atomicAdd(&cc[j].x, 1u);
      }
    } else if (VARIANT == 9) {         // one CAS per element at its home, no probing
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t j = homek(mixk(kv[c]));
        acc += atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kv[c]);
        slot[c] = j;
      }
    } else if (VARIANT == 10 || VARIANT == 11) {
      // CAS at home; a collision scans on G slots per round trip with plain reads (ds_read2),
      // CAS-ing the first empty slot it sees (a lost race rescans from there)
      constexpr int G = VARIANT == 10 ? 4 : 8;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint64_t kk = kv[c];
        uint32_t j = homek(mixk(kk));
        uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
        if (!(prev == ~0ull || prev == kk)) {
          if (++j == CAP) j = 0;
          for (;;) {
            uint64_t g[G];
#pragma unroll
            for (int q = 0; q < G; ++q) {
              uint32_t jj = j + q;
              if (jj >= CAP) jj -= CAP;
              g[q] = key[jj];
            }
            int hit = -1;
#pragma unroll
            for (int q = G - 1; q >= 0; --q)
              if (g[q] == ~0ull || g[q] == kk) hit = q;
            if (hit < 0) { j += G; if (j >= CAP) j -= CAP; continue; }
            j += hit;
            if (j >= CAP) j -= CAP;
            if (g[hit] == kk) break;
            prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
            if (prev == ~0ull || prev == kk) break;
            if (++j == CAP) j = 0;
          }
        }
        slot[c] = j;
        atomicAdd(&cc[j].x, 1u);
      }
    } else if (VARIANT == 12) {
      // per-lane state machine over the lane's elements, ONE LDS instruction per trip (the CAS);
      // the count adds run after the loop, one full-wave instruction per element index
      uint32_t hm[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) hm[q] = homek(mixk(kv[q]));
      int c = 0;
      uint64_t kk = kv[0];
      uint32_t j = hm[0];
      bool live = true;
      while (__any(live)) {
        if (live) {
          const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
          if (prev == ~0ull || prev == kk) {
#pragma unroll
            for (int q = 0; q < 4; ++q) if (q == c) slot[q] = j;
            ++c;
            if (c == 4) live = false;
#pragma unroll
            for (int q = 1; q < 4; ++q) if (q == c) { kk = kv[q]; j = hm[q]; }
          } else if (++j == CAP) j = 0;
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(&cc[slot[q]].x, 1u);
    } else if (VARIANT == 6) {         // element by element without the count adds
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t j = homek(mixk(kv[c]));
        for (;;) {
          const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kv[c]);
          if (prev == ~0ull || prev == kv[c]) break;
          if (++j == CAP) j = 0;
        }
        slot[c] = j;
      }
    } else {
      int c = 0;
      uint64_t kk = kv[0];
      uint32_t j = homek(mixk(kk));
      bool live = true;
      while (live) {
        const uint64_t prev = atomicCAS((unsigned long long*)&key[j], ~0ull, (unsigned long long)kk);
        if (prev == ~0ull || prev == kk) {
          atomicAdd(&cc[j].x, 1u);
#pragma unroll
          for (int q = 0; q < 4; ++q) if (q == c) slot[q] = j;
          if (++c == 4) live = false;
          else {
#pragma unroll
            for (int q = 1; q < 4; ++q) if (q == c) kk = kv[q];
            j = homek(mixk(kk));
          }
        } else if (++j == CAP) j = 0;
      }
    }
    acc += slot[0] + slot[1] + slot[2] + slot[3];
    __syncthreads();
  }
  if (acc == 12345) out[0] = acc;
}

template <int VARIANT>
void run_pa(const char* name) {
  uint64_t* out;
  hipMalloc(&out, 64);
  const int grid = 256 * 6 * 8, reps = 8;
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(kpa<VARIANT>, dim3(grid), dim3(256), 0, 0, out, 7u, reps);
  hipEventRecord(a);
  hipLaunchKernelGGL(kpa<VARIANT>, dim3(grid), dim3(256), 0, 0, out, 9u, reps);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double buckets = (double)grid * reps;
  printf("%-34s %8.3f ms  %8.2f ns/bucket chip-wide  -> %.1f us per 9,766 buckets\n", name, ms,
         ms * 1e6 / buckets, ms * 1e3 / buckets * 9766);
  hipFree(out);
}

template <int MODE>
void run(const char* name, int wgs_per_cu) {
  uint64_t* out;
  hipMalloc(&out, 64);
  const int grid = 256 * wgs_per_cu * 8;
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, 7u);
  hipEventRecord(a);
  const int reps = 10;
  for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(k<MODE>, dim3(grid), dim3(256), 0, 0, out, 7u + w);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double ops = (double)grid * 256 * ITERS * reps;
  const double per_cu_cycle = ops / (ms * 1e-3) / 256 / 2.4e9;
  printf("%-34s %8.3f ms  %7.2f G lane-ops/s  %6.2f lane-ops/CU/cycle  %6.2f wave-instr/CU/kcycle\n",
         name, ms / reps, ops / (ms * 1e-3) / 1e9, per_cu_cycle, per_cu_cycle / 64 * 1000);
  hipFree(out);
}

int main() {
  run<2>("ds_read_b64 random (independent)", 6);
  run<0>("CAS64 rtn random, fails", 6);
  run<4>("CAS64 rtn distinct slots", 6);
  run<3>("CAS64 rtn dependent chain", 6);
  run<1>("add u32 no-rtn random", 6);
  run<5>("add u32 rtn random", 6);
  run<0>("CAS64 rtn random, fails (1 WG/CU)", 1);
  run<3>("CAS64 chain (1 WG/CU)", 1);
  run_pa<0>("pass A, element by element");
  run_pa<1>("pass A, per-lane state machine");
  run_pa<2>("pass A, state machine, homes first");
  run_pa<3>("pass A, home round then failures");
  run_pa<4>("pass A, home round + per-wave queue");
  run_pa<5>("pass A, home round + queue, no slot back");
  run_pa<6>("pass A, element by element, no adds");
  run_pa<0>("pass A, element by element (again)");
  run_pa<7>("calib: keys + clear + adds, no CAS");
  run_pa<8>("calib: keys + clear only");
  run_pa<9>("calib: one CAS per element, no probing");
  run_pa<10>("pass A, home CAS, then 4-slot read scans");
  run_pa<11>("pass A, home CAS, then 8-slot read scans");
  run_pa<0>("pass A, element by element (3rd)");
  run_pa<12>("pass A, state machine, one LDS op per trip");
  run<6>("CAS64 rtn fails, 8 lanes", 6);
  run<7>("CAS64 rtn fails, 1 lane", 6);
  run<8>("CAS64 rtn fails, 32 lanes", 6);
  run<9>("CAS32 rtn fails, 64 lanes", 6);
  return 0;
}
