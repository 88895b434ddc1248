// kmhg_join.hip -- kmer.pairs: positions of the k-mers two indices share.
//
// Replaces kmer_pair_pos (reference src/kmer_hash.c:1174-1203, R wrapper kmer_hash.R:30-34):
// for every k-mer of index a that index b also holds, the cross product of a's positions
// (outer) and b's positions (inner) as rows (a, b).  The reference walks a's buckets without a
// kh_exist check and calls kh_exist(b, kh_end(b)) out of bounds (test.R:330: "This crashes");
// here only a's live k-mers are visited, in a's kmer.pos row order.
//
//   J_probe  key c of a (readout order perm_a) -> one probe of b's table; jinfo[c] = {count_a,
//            ref_a, count_b, ref_b} (ref = the inline position for a count of 1, else the first
//            index in `positions`), per-tile row totals count_a * count_b
//   (k_scan_tiles_u64)
//   J_emit   rows dealt to lanes by binary search over the tile's LDS prefix (a k-mer shared
//            thousands of times does not serialise a lane); row t of key c is (i, j) =
//            (t / count_b, t mod count_b)
#include <hip/hip_runtime.h>
#include "kmhg_common.h"
#include "kmhg_device.h"
#include "kmhg_kernels.h"

namespace kmhg {

__global__ void __launch_bounds__(BLOCK)
k_join_probe(const uint32_t* __restrict__ perm_a, uint32_t Ua, const Slot* __restrict__ Ta,
             const Slot* __restrict__ Tb, Geom gb, uint4* __restrict__ jinfo,
             uint64_t* __restrict__ tile_rows) {
  __shared__ uint64_t sh[8];
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  uint64_t rows = 0;
#pragma unroll 2
  for (int j = 0; j < WPT; ++j) {
    const uint64_t c = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    if (c >= Ua) continue;
    const uint4 va = *reinterpret_cast<const uint4*>(&Ta[perm_a[c]]);
    const uint64_t key = ((uint64_t)va.y << 32) | va.x;
    uint32_t nb = 0, auxb = 0;
    table_find(Tb, gb, key, nb, auxb);
    const uint32_t na = va.z;
    jinfo[c] = make_uint4(na, na == 1 ? va.w : va.w - na, nb, nb == 1 ? auxb : auxb - nb);
    rows += (uint64_t)na * nb;
  }
  uint64_t tot;
  block_excl_scan(rows, sh, tot);
  if (threadIdx.x == 0) tile_rows[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK)
k_join_emit(const uint4* __restrict__ jinfo, uint32_t Ua, const int32_t* __restrict__ pos_a,
            const int32_t* __restrict__ pos_b, const uint64_t* __restrict__ tile_row0,
            int2* __restrict__ out) {
  __shared__ uint64_t incl[TILE];
  __shared__ uint64_t sh[8];
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  uint64_t loc[WPT];
  uint64_t run = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {         // thread-contiguous entries for the LDS prefix
    const uint64_t c = t0 + (uint64_t)threadIdx.x * WPT + j;
    uint64_t r = 0;
    if (c < Ua) {
      const uint4 v = jinfo[c];
      r = (uint64_t)v.x * v.z;
    }
    run += r;
    loc[j] = run;
  }
  uint64_t tot;
  const uint64_t ex = block_excl_scan(run, sh, tot);
#pragma unroll
  for (int j = 0; j < WPT; ++j) incl[threadIdx.x * WPT + j] = loc[j] + ex;
  __syncthreads();
  if (tot == 0) return;
  const uint64_t r0 = tile_row0[blockIdx.x];
  for (uint64_t r = threadIdx.x; r < tot; r += BLOCK) {
    int lo = 0, hi = TILE - 1;             // first entry with incl > r
    while (lo < hi) { const int mid = (lo + hi) >> 1; if (incl[mid] > r) hi = mid; else lo = mid + 1; }
    const uint64_t t = r - (lo ? incl[lo - 1] : 0);
    const uint4 v = jinfo[t0 + lo];
    const uint64_t i = t / v.z, jj = t - i * v.z;
    const int32_t a = v.x == 1 ? (int32_t)v.y : pos_a[v.y + i];
    const int32_t b = v.z == 1 ? (int32_t)v.w : pos_b[v.w + jj];
    out[r0 + r] = make_int2(a, b);
  }
}

static inline unsigned grid_n(uint64_t n, unsigned per) {
  const uint64_t g = (n + per - 1) / per;
  return (unsigned)(g ? g : 1);
}

void launch_join_probe(const uint32_t* perm_a, uint32_t Ua, const Slot* Ta, const Slot* Tb, Geom gb,
                       uint4* jinfo, uint64_t* tile_rows, hipStream_t s) {
  hipLaunchKernelGGL(k_join_probe, dim3(grid_n(Ua, TILE)), dim3(BLOCK), 0, s, perm_a, Ua, Ta, Tb,
                     gb, jinfo, tile_rows);
}
void launch_join_emit(const uint4* jinfo, uint32_t Ua, const int32_t* pos_a, const int32_t* pos_b,
                      const uint64_t* tile_row0, int2* out, hipStream_t s) {
  hipLaunchKernelGGL(k_join_emit, dim3(grid_n(Ua, TILE)), dim3(BLOCK), 0, s, jinfo, Ua, pos_a,
                     pos_b, tile_row0, out);
}

}  // namespace kmhg
