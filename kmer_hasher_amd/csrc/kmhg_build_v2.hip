// kmhg_build_v2.hip -- partitioned index build: no per-window global atomics.
//
// Replaces the same reference loops as K_insert/K_scatter/K_sort (src/kmer_pos.c:36-50, 66-98,
// 21-33; kvec growth src/kvec.h:74-80) with an HBM-streaming design for CDNA4:
//
//   V_hist0     LDS-staged 2-bit encode + N mask of every window (as K_insert) and a per-tile
//               histogram of the first radix digit of each window's bucket; keeps the sequence's
//               code words (the diagonal query path) and, for small inputs, every window's
//               bucket id
//   V_scan      exclusive scan of the [digit][tile] histograms (decoupled look-back)
//   V_scatter   stable radix pass: every wave ranks its 512 elements by digit with the
//               returned values of its LDS count atomics (lane-ordered; a device self-check picks
//               ballot ranks where that does not hold), elements land at histogram offsets --
//               LSD over 1-3 digits sorts the windows by bucket while keeping position order
//               inside a bucket
//   V_hist      digit histogram for the next radix pass
//   V_bounds    bucket start offsets in the bucket-sorted stream (from the histograms for <= 2
//               passes)
//   V_bucket_wg ONE WORKGROUP PER BUCKET of ~1,024 windows: the bucket's keys go into a shared
//               LDS hash table (LDS CAS + count atomics), the counts are scanned, repeated keys'
//               windows are ranked in position order, so positions are written ascending per key
//               by construction (no sort).  The LDS table is written out as the bucket's
//               sub-table of the global table.
//
// A bucket's windows are exactly its keys' positions, so the CSR slice of bucket b is
// [start[b], start[b+1]) of `positions` with no global coordination.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <type_traits>
#include "kmhg_common.h"
#include "kmhg_device.h"
#include "kmhg_kernels.h"

namespace kmhg {

// Diagnostic phase stamps (built only with -DKMHG_STAMPS into a separate library; the real
// kernels execute no stamp).  Lane 0 of each bucket's wave writes s_memtime per phase.
#ifdef KMHG_STAMPS
__device__ uint64_t* g_stamps;
#define STAMP(b, i)                                                                   \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    uint64_t _t = __builtin_amdgcn_s_memtime();                                       \
    if (lane_id() == 0 && g_stamps) g_stamps[(uint64_t)(b) * 8 + (i)] = _t;           \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#define STAMP_WG(b, i) do { if (threadIdx.x < 64) STAMP(b, i); } while (0)
// ... after this wave's outstanding loads have landed (splits load latency from the work after)
#define STAMP_WG_DRAIN(b, i) \
  do { __builtin_amdgcn_s_waitcnt(0); if (threadIdx.x < 64) STAMP(b, i); } while (0)
#else
#define STAMP(b, i) do {} while (0)
#define STAMP_WG(b, i) do {} while (0)
#define STAMP_WG_DRAIN(b, i) do {} while (0)
#endif

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Radix digit of a key's bucket: floor(b / div) mod R with host-computed magic multipliers,
// floor(x / d) = mulhi64(x, ceil(2^64 / d)) exactly for x, d < 2^32 (m = 0 encodes d = 1) --
// no integer division in the kernels.
__device__ __forceinline__ uint32_t div_magic(uint32_t x, uint64_t m) {
  return m ? (uint32_t)__umul64hi((uint64_t)x, m) : x;
}
// The bucket of hash h inside this build's part (Geom: whole table b0 = 0, nbh = nb); a key of
// another part's range gives a value >= g.nb (unsigned wrap below b0).
__device__ __forceinline__ uint32_t bucket_local(uint64_t h, const Geom& g) {
  return bucket_of(h, g.nbh ? g.nbh : g.nb) - g.b0;
}
__device__ __forceinline__ bool in_part(uint64_t h, const Geom& g) {
  return bucket_local(h, g) < g.nb;
}
// the side slot (key ~0 at k = 32) belongs to the bucket of mix64(~0) of the whole table
__device__ __forceinline__ bool side_bucket(uint32_t b, const Geom& g) {
  return b + g.b0 == bucket_of(mix64(EMPTY_KEY), g.nbh ? g.nbh : g.nb);
}
// radix digit of a bucket id (bucket-id streams carry it instead of the key)
__device__ __forceinline__ uint32_t digit_of_b(uint32_t b, const Digit& D) {
  const uint32_t q = div_magic(b, D.mdiv);
  return q - div_magic(q, D.mR) * D.R;
}
__device__ __forceinline__ uint32_t digit_of_h(uint64_t h, const Geom& g, const Digit& D) {
  return digit_of_b(bucket_local(h, g), D);
}
__device__ __forceinline__ uint32_t digit_of(uint64_t key, const Geom& g, const Digit& D) {
  return digit_of_h(mix64(key), g, D);
}

// Lanes of the wave holding the same `v` (nbits wide) among active lanes: one ballot per bit.
__device__ __forceinline__ uint64_t match_bits(uint32_t v, int nbits, bool act) {
  uint64_t m = __ballot(act);
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (v >> b) & 1u;
    const uint64_t x = __ballot(act && bit);
    m &= bit ? x : ~x;
  }
  return m;
}

// The diagonal query path's copy of the index sequence (DiagBlock, kmhg_kernels.h), written by
// V_hist0 from its stage: the tile's PTILE / 16 code words and N-flag words (the last tile also
// the words its last windows reach into).  Thread t stores the word it packed itself (stage word
// t), so no barrier is needed first.  ~0.4 B per window against the build's ~17.
constexpr int DIAG_TW = PTILE / 16;             // code words per tile
constexpr int DIAG_EXTRA = 3;                   // ... beyond the last tile's own
static_assert(PSTAGE_W16 <= BLOCK && HALO % 16 == 0 && HALO / 16 + DIAG_TW + DIAG_EXTRA <= PSTAGE_W16,
              "one stage word per thread; the last tile's extra words are staged");
__device__ __forceinline__ void diag_words_out(const PStage& st, uint32_t tile, uint32_t ntiles,
                                               uint32_t* __restrict__ code,
                                               uint16_t* __restrict__ nbit) {
  const int w = (int)threadIdx.x - HALO / 16;
  if (w >= 0 && w < (tile + 1 == ntiles ? DIAG_TW + DIAG_EXTRA : DIAG_TW)) {
    code[(uint64_t)tile * DIAG_TW + w] = st.code[threadIdx.x];
    nbit[(uint64_t)tile * DIAG_TW + w] = (uint16_t)st.nbit[threadIdx.x];
  }
}

// Persistent form for the interleaved schedule (one histogram column per tile): workgroup w
// walks virtual tiles w, w + G, ... (XCD-contiguous like the scatter) and loads the next tile's
// chars into registers while it encodes the current one, so the load latency of all but the
// first tile is hidden behind the encode.
// CODES (position indices): the diagonal query path's code and N-flag words ride along, each
// thread storing the words it packed right after the pack, BEFORE the next tile's loads are
// issued, so the wait for those loads never waits on these stores.  (A/B, config 2: validity
// ballots kept in the window loop and stored per tile cost 24 -> 30-41 us; a kernel of its own
// 18 us; these stores ~1 us.)
// BIDS (bucket-id builds): every window's bucket id (~0 for a window that is not indexed or
// outside this part) is stored in window order, one coalesced 4-B store per window, so the first
// scatter pass reads the ids instead of encoding and hashing every window a second time.
#ifndef KMHG_HIST0_WAVES
#define KMHG_HIST0_WAVES 6   // Win8: 80 VGPRs without spills (7 spills 44 B / lane)
#endif
// PARTC (a part build of an owner-computes build, key streams): the windows this part owns are
// written compacted per tile instead of counted -- (key, position) of tile t's owned windows in
// window order at [t * PTILE, t * PTILE + tcnt[t]) -- and V_part_dense packs them into one
// stream, which the radix passes read: ~1/n_parts of the windows instead of encoding and hashing
// every window of the sequence a second time.
template <bool CODES, bool BIDS = false, bool PARTC = false>
__global__ void __launch_bounds__(BLOCK, PARTC ? 5 : KMHG_HIST0_WAVES)   // PARTC: no spills
k_v2_hist0p(const uint8_t* __restrict__ seq, int64_t L, int k, int64_t Nw, Geom g, Digit D,
            uint32_t* __restrict__ hist, uint32_t ntiles, uint64_t* __restrict__ scan_status,
            uint32_t n_status, BuildMeta* __restrict__ meta, uint32_t* __restrict__ code,
            uint16_t* __restrict__ nbit, uint32_t* __restrict__ bids,
            uint64_t* __restrict__ ckeys, uint32_t* __restrict__ cpos,
            uint32_t* __restrict__ tcnt) {
  __shared__ PStage st;
  __shared__ uint32_t lh[V2_MAXR];
  __shared__ uint64_t scs[5];
  __shared__ uint64_t sk[PARTC ? PTILE : 1];     // PARTC: the tile's own windows, compacted
  __shared__ uint32_t sp[PARTC ? PTILE : 1];
  for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n_status; i += gridDim.x * BLOCK)
    scan_status[i] = 0;
  if (blockIdx.x == 0 && threadIdx.x < sizeof(BuildMeta) / 4)
    reinterpret_cast<uint32_t*>(meta)[threadIdx.x] = 0u;
  const uint32_t G = gridDim.x;
  const uint32_t n_iter = (ntiles - blockIdx.x + G - 1) / G;
  auto tile_at = [&](uint32_t i) -> uint32_t { return xcd_remap(blockIdx.x + i * G, ntiles); };
  for (uint32_t d = threadIdx.x; d < D.R; d += BLOCK) lh[d] = 0;
  StageRegs<PSTAGE_W16> regs;
  stage_load<PSTAGE_W16, true>(regs, seq, L, (int64_t)tile_at(0) * PTILE - HALO, true);
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t tile = tile_at(it);
    const int64_t tile0 = (int64_t)tile * PTILE;
    stage_pack(regs, st);                      // the previous tile's reads of st are done
    if (CODES) diag_words_out(st, tile, ntiles, code, nbit);
    if (it + 1 < n_iter)
      stage_load<PSTAGE_W16, true>(regs, seq, L, (int64_t)tile_at(it + 1) * PTILE - HALO, true);
    __syncthreads();
    // thread t takes the 8 consecutive windows [8 t, 8 t + 8) of the tile: their code and N
    // flags come from 8 LDS reads (Win8) instead of 6 per window -- this pass was bound
    // by those reads -- and their bucket ids leave as two 16-B stores
    static_assert(PWPT == 8, "Win8 covers 8 windows per thread");
    {
      const int w0 = PWPT * threadIdx.x;
      const int64_t s0 = tile0 + w0;
      const Win8 win(st, HALO + w0, s0, L, k);
      uint32_t bl[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bl[j] = ~0u;
        if (s0 + j < Nw && win.valid(j)) {
          const uint32_t b = bucket_local(mix64(win.key(j)), g);
          if (b < g.nb) {
            if (!PARTC) atomicAdd(&lh[digit_of_b(b, D)], 1u);
            bl[j] = b;
          }
        }
      }
      if (PARTC) {                 // this part's windows, compacted in window order
        uint32_t own = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) own |= (bl[j] != ~0u ? 1u : 0u) << j;
        uint64_t tot;
        uint32_t at = (uint32_t)block_excl_scan((uint64_t)__popc(own), scs, tot);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (own >> j & 1u) {
            sk[at] = win.key(j);
            sp[at] = (uint32_t)(s0 + j + 1);
            ++at;
          }
        }
        __syncthreads();
        // out of LDS in order: consecutive lanes, consecutive entries
        const uint64_t base = (uint64_t)tile * PTILE;
        for (uint32_t i = threadIdx.x; i < (uint32_t)tot; i += BLOCK) {
          ckeys[base + i] = sk[i];
          cpos[base + i] = sp[i];
        }
        if (threadIdx.x == 0) tcnt[tile] = (uint32_t)tot;
      }
      // the id array holds Nw + PTILE entries: a tile's last 16-B stores stay inside it
      if (BIDS && s0 < Nw) {
        uint4* o = reinterpret_cast<uint4*>(bids + s0);
        o[0] = make_uint4(bl[0], bl[1], bl[2], bl[3]);
        o[1] = make_uint4(bl[4], bl[5], bl[6], bl[7]);
      }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; !PARTC && d < D.R; d += BLOCK) {
      hist[(size_t)d * ntiles + tile] = lh[d];
      lh[d] = 0;                               // next tile's atomics follow a barrier
    }
  }
}

// ---------------------------------------------------------------- V_scan (u32, exclusive)
// Single pass: tiles in ticket order, decoupled look-back (kmhg_device.h) for the tile base.
// `status` holds one look-back word per tile and the ticket at status[ntiles]; the preceding
// histogram kernel zeroed them.  *total <- sum (the number of valid windows).
// J entries per thread (TILE = BLOCK * J per workgroup): J = 32 for long arrays (a 4x shorter
// look-back chain, 16-B loads).
template <int J>
__global__ void __launch_bounds__(BLOCK)
k_scan_lb_u32(uint32_t* __restrict__ a, uint64_t n, uint64_t* __restrict__ status,
              uint32_t ntiles, uint32_t* __restrict__ total) {
  __shared__ uint64_t sh[8];
  __shared__ uint32_t tk;
  __shared__ uint64_t base_sh;
  const uint32_t tile = take_ticket(reinterpret_cast<uint32_t*>(status + ntiles), &tk);
  const uint64_t base = (uint64_t)tile * (BLOCK * J) + (uint64_t)threadIdx.x * J;
  uint32_t v[J];
  uint64_t sum = 0;
  if (J % 4 == 0 && base + J <= n) {          // whole: 16-B loads (a is 16-B aligned, J % 4 == 0)
#pragma unroll
    for (int j = 0; j < J; j += 4) {
      const uint4 x = *reinterpret_cast<const uint4*>(a + base + j);
      v[j] = x.x; v[j + 1] = x.y; v[j + 2] = x.z; v[j + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j) v[j] = (base + j < n) ? a[base + j] : 0u;
  }
#pragma unroll
  for (int j = 0; j < J; ++j) sum += v[j];
  uint64_t tot;
  const uint64_t ex = block_excl_scan(sum, sh, tot);
  if (threadIdx.x < 64) {
    const uint64_t x = lookback_excl(status, tile, tot);
    if (threadIdx.x == 0) {
      base_sh = x;
      if (tile == ntiles - 1) *total = (uint32_t)(x + tot);
    }
  }
  __syncthreads();
  uint64_t run = ex + base_sh;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t x = v[j];
    v[j] = (uint32_t)run;
    run += x;
  }
  if (J % 4 == 0 && base + J <= n) {
#pragma unroll
    for (int j = 0; j < J; j += 4)
      *reinterpret_cast<uint4*>(a + base + j) = make_uint4(v[j], v[j + 1], v[j + 2], v[j + 3]);
  } else {
#pragma unroll
    for (int j = 0; j < J; ++j)
      if (base + j < n) a[base + j] = v[j];
  }
}

// ---------------------------------------------------------------- V_hist (passes >= 1)
// HLL (count-only builds, first pass): a HyperLogLog sketch of the distinct keys rides on the
// histogram pass, which hashes every key anyway.  A 1/HLL_SAMPLE key-space sample (h mod 64 == 0)
// updates register (h >> 6) mod 256 with rho = leading zeros of h's top 50 bits + 1; each
// workgroup leaves its registers as one 256-B row (bytes), V_hll reduces the rows.
constexpr uint32_t HLL_SAMPLE_BITS = 6;
constexpr uint32_t HLL_PART_ROWS = 256;        // V_hll workgroups (partial rows) at most
static_assert(HLL_PART_WORDS == HLL_PART_ROWS * 64 + 1, "V_hll partial rows + ticket");

// BID: the stream holds u32 bucket ids (BM scatter passes), digits without hashing.
template <bool HLL, bool BID = false>
__global__ void __launch_bounds__(BLOCK)
k_v2_hist(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ n_ptr, Geom g,
          Digit D, uint32_t* __restrict__ hist, uint32_t ntiles,
          uint64_t* __restrict__ scan_status, uint32_t n_status, uint32_t* __restrict__ hll_rows,
          uint32_t* __restrict__ hll_regs, uint32_t* __restrict__ save_col0, int skip_empty) {
  __shared__ uint32_t lh[V2_MAXR];
  __shared__ uint32_t hreg[HLL ? HLL_REGS : 1];
  for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n_status; i += gridDim.x * BLOCK)
    scan_status[i] = 0;
  // the previous pass's scanned column 0 (digit starts), kept for V_bounds_lo before this
  // workgroup -- the only writer of column 0 -- overwrites it
  const uint32_t c = xcd_remap(blockIdx.x, ntiles);      // one workgroup per tile
  if (save_col0 && c == 0)
    for (uint32_t d = threadIdx.x; d < D.R; d += BLOCK) save_col0[d] = hist[(size_t)d * ntiles];
  if (HLL) {
    for (uint32_t i = threadIdx.x; i < HLL_REGS; i += BLOCK) hreg[i] = 0;
  }
  const uint64_t n = *n_ptr;
  const uint64_t e0 = (uint64_t)c * PTILE;
  const uint64_t e1 = min(n, e0 + (uint64_t)PTILE);
  const uint32_t R = D.R;
  for (uint32_t d = threadIdx.x; d < R; d += BLOCK) lh[d] = 0;
  __syncthreads();
  constexpr int NL = BID ? 8 : 4;                 // loads in flight per lane
  const uint32_t* __restrict__ bids = reinterpret_cast<const uint32_t*>(keys);
  for (uint64_t e = e0 + threadIdx.x; e < e1; e += NL * BLOCK) {
    uint32_t dg[NL];
    bool in[NL];
    if (BID) {
#pragma unroll
      for (int j = 0; j < NL; ++j) {
        in[j] = e + j * BLOCK < e1;
        dg[j] = in[j] ? digit_of_b(bids[e + j * BLOCK], D) : 0u;
      }
    }
#pragma unroll
    for (int j = 0; j < NL && !BID; ++j) {
      in[j] = e + j * BLOCK < e1;
      const uint64_t key = in[j] ? keys[e + j * BLOCK] : 0ull;
      if (skip_empty && key == EMPTY_KEY) in[j] = false;      // a padded read's unused slot
      const uint64_t h = in[j] ? mix64(key) : 1ull;
      dg[j] = in[j] ? digit_of_h(h, g, D) : 0u;
      if (HLL && (h & ((1u << HLL_SAMPLE_BITS) - 1)) == 0)
        atomicMax(&hreg[(uint32_t)(h >> HLL_SAMPLE_BITS) & (HLL_REGS - 1)],
                  (uint32_t)__clzll(h | ((1ull << (HLL_SAMPLE_BITS + 8)) - 1)) + 1u);
    }
#pragma unroll
    for (int j = 0; j < NL; ++j)
      if (in[j]) atomicAdd(&lh[dg[j]], 1u);
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < R; d += BLOCK) hist[(size_t)d * ntiles + c] = lh[d];
  if (HLL && threadIdx.x < HLL_REGS / 4) {
    const uint32_t* h4 = hreg + 4 * threadIdx.x;
    hll_rows[(size_t)blockIdx.x * (HLL_REGS / 4) + threadIdx.x] =
        h4[0] | (h4[1] << 8) | (h4[2] << 16) | (h4[3] << 24);
  }
}

// Persistent form for the interleaved schedule (position builds' later passes): workgroup w walks
// virtual tiles w, w + G, ... (XCD-contiguous like the scatter), thread t taking the 8
// consecutive elements [8 t, 8 t + 8) of a tile with 16-B loads, the next tile's loads in flight
// while this one is counted -- the one-tile-per-workgroup form exposed every workgroup's load
// latency (config 2: 14.5 us for 40 MB).  `in` holds n + PTILE elements (the passes' padded
// streams), so whole-tile loads stay inside it.
// MODE: 0 = u64 keys, 1 = u32 bucket ids, 2 = packed 12-B {key lo, key hi, pos} elements (the
// position builds' key streams), 3 = packed 8-B elements (Pack8: the key is e >> sh), 4 = the
// previous pass's digit stream (u16 digits, DS in V_scatter), 5 = the same in u8 digits.
template <int MODE>
__global__ void __launch_bounds__(BLOCK)
k_v2_histp(const uint64_t* __restrict__ in, const uint32_t* __restrict__ n_ptr, Geom g, Digit D,
           uint32_t* __restrict__ hist, uint32_t ntiles, uint64_t* __restrict__ scan_status,
           uint32_t n_status, uint32_t* __restrict__ save_col0, int sh) {
  __shared__ uint32_t lh[V2_MAXR];
  for (uint32_t i = blockIdx.x * BLOCK + threadIdx.x; i < n_status; i += gridDim.x * BLOCK)
    scan_status[i] = 0;
  const uint64_t n = *n_ptr;
  const uint32_t G = gridDim.x, R = D.R;
  const uint32_t n_iter = (ntiles - blockIdx.x + G - 1) / G;
  auto tile_at = [&](uint32_t i) -> uint32_t { return xcd_remap(blockIdx.x + i * G, ntiles); };
  // the previous pass's scanned column 0, saved by the workgroup that writes column 0 (tile 0)
  // before it does
  if (save_col0 && tile_at(0) == 0)
    for (uint32_t d = threadIdx.x; d < R; d += BLOCK) save_col0[d] = hist[(size_t)d * ntiles];
  for (uint32_t d = threadIdx.x; d < R; d += BLOCK) lh[d] = 0;
  constexpr bool BID = MODE == 1;
  if constexpr (MODE == 2) {
    // packed 12-B elements: thread t takes elements t + 256 j of the tile (j < 8), so every
    // load instruction reads 768 contiguous bytes per wave (one element per lane, dwordx3); a
    // thread's 96 consecutive bytes would spread each instruction over 48 lines
    uint3 nx[8];
    auto prefetch = [&](uint32_t tile) {
      const uint3* src = reinterpret_cast<const uint3*>(in) + (uint64_t)tile * PTILE + threadIdx.x;
#pragma unroll
      for (int j = 0; j < 8; ++j) nx[j] = src[j * BLOCK];
    };
    prefetch(tile_at(0));
    for (uint32_t it = 0; it < n_iter; ++it) {
      const uint32_t tile = tile_at(it);
      uint3 cur[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) cur[j] = nx[j];
      if (it + 1 < n_iter) prefetch(tile_at(it + 1));
      __syncthreads();                                 // lh zeroed (previous tile written out)
      const uint64_t e0 = (uint64_t)tile * PTILE + threadIdx.x;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (e0 + (uint64_t)j * BLOCK < n) {
          const uint64_t key = ((uint64_t)cur[j].y << 32) | cur[j].x;
          atomicAdd(&lh[digit_of_h(mix64(key), g, D)], 1u);
        }
      }
      __syncthreads();
      for (uint32_t d = threadIdx.x; d < R; d += BLOCK) {
        hist[(size_t)d * ntiles + tile] = lh[d];
        lh[d] = 0;
      }
    }
    return;
  }
  constexpr bool DIG = MODE == 4, DIG8 = MODE == 5;
  constexpr int NV = DIG || DIG8 ? 1 : MODE == 1 ? 2 : 4;   // 16-B loads per thread per tile
  uint4 nx[NV];
  auto prefetch = [&](uint32_t tile) {
    if constexpr (DIG8) {                              // 8 u8 digits: one 8-B load
      const uint2 v = reinterpret_cast<const uint2*>(in)[(uint64_t)tile * (PTILE / 8) + threadIdx.x];
      nx[0] = make_uint4(v.x, v.y, 0u, 0u);
      return;
    }
    const uint4* src = reinterpret_cast<const uint4*>(in) +
                       ((uint64_t)tile * PTILE + 8u * threadIdx.x) / (DIG ? 8 : BID ? 4 : 2);
#pragma unroll
    for (int v = 0; v < NV; ++v) nx[v] = src[v];
  };
  prefetch(tile_at(0));
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t tile = tile_at(it);
    uint4 cur[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) cur[v] = nx[v];
    if (it + 1 < n_iter) prefetch(tile_at(it + 1));
    __syncthreads();                                   // lh zeroed (previous tile written out)
    const uint64_t e0 = (uint64_t)tile * PTILE + 8u * threadIdx.x;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (e0 + j < n) {
        uint32_t dg;
        if (DIG8) {
          const uint32_t wj = (j >> 2) == 0 ? cur[0].x : cur[0].y;
          dg = (wj >> (8 * (j & 3))) & 0xFFu;
        } else if (DIG) {
          const uint4 w = cur[0];
          const uint32_t wj = (j >> 1) == 0 ? w.x : (j >> 1) == 1 ? w.y : (j >> 1) == 2 ? w.z : w.w;
          dg = (j & 1) ? wj >> 16 : wj & 0xFFFFu;
        } else if (BID) {
          const uint4 w = cur[j >> 2];
          const uint32_t id = (j & 3) == 0 ? w.x : (j & 3) == 1 ? w.y : (j & 3) == 2 ? w.z : w.w;
          dg = digit_of_b(id, D);
        } else {
          const uint4 w = cur[j >> 1];
          const uint64_t e = (j & 1) ? (((uint64_t)w.w << 32) | w.z) : (((uint64_t)w.y << 32) | w.x);
          dg = digit_of_h(mix64(MODE == 3 ? e >> sh : e), g, D);
        }
        atomicAdd(&lh[dg], 1u);
      }
    }
    __syncthreads();
    for (uint32_t d = threadIdx.x; d < R; d += BLOCK) {
      hist[(size_t)d * ntiles + tile] = lh[d];
      lh[d] = 0;
    }
  }
}

// V_hll: register-wise max of the histogram workgroups' HLL rows.  V_hll_part: workgroup g
// reduces rows [g * rpw, (g + 1) * rpw) into partial row g (thread t takes packed word t mod 64
// of every 16th row: each row one coalesced 256-B read, eight rows in flight per thread);
// V_hll_final (one workgroup) reduces the partial rows and turns the registers into the estimate
// of distinct keys (Flajolet et al. 2007, linear counting in the small range, x 64 for the
// sample), published to pinned host memory.  Two launches instead of a last-workgroup ticket:
// the ticket's release fence per workgroup (an XCD L2 write-back) cost ~35 us.
__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) r |= max((a >> (8 * j)) & 0xFFu, (b >> (8 * j)) & 0xFFu) << (8 * j);
  return r;
}

// rows r0 + q, r0 + q + HLL_RG, ... below r1, word w: eight independent loads per trip
constexpr uint32_t HLL_T = 1024;               // V_hll threads: 16 row groups x 64 words
constexpr uint32_t HLL_RG = HLL_T / 64;
__device__ __forceinline__ uint32_t hll_rows_max(const uint32_t* rows, uint32_t r0, uint32_t r1,
                                                 uint32_t w, uint32_t q) {
  uint32_t m = 0;
  uint32_t r = r0 + q;
  for (; r + 7 * HLL_RG < r1; r += 8 * HLL_RG) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = rows[(size_t)(r + j * HLL_RG) * 64 + w];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = max_u8x4(m, x[j]);
  }
  for (; r < r1; r += HLL_RG) m = max_u8x4(m, rows[(size_t)r * 64 + w]);
  return m;
}

__global__ void __launch_bounds__(HLL_T)
k_v2_hll_part(const uint32_t* __restrict__ rows, uint32_t n_rows, uint32_t* __restrict__ part) {
  __shared__ uint32_t pw[HLL_RG][64];
  const uint32_t w = threadIdx.x & 63, q = threadIdx.x >> 6;
  const uint32_t rpw = (n_rows + gridDim.x - 1) / gridDim.x;
  const uint32_t r0 = blockIdx.x * rpw, r1 = min(n_rows, r0 + rpw);
  pw[q][w] = hll_rows_max(rows, r0, r1, w, q);
  __syncthreads();
  if (q == 0) {
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < HLL_RG; ++j) m = max_u8x4(m, pw[j][w]);
    part[(size_t)blockIdx.x * 64 + w] = m;
  }
}

__global__ void __launch_bounds__(HLL_T)
k_v2_hll_final(const uint32_t* __restrict__ part, uint32_t n_part, double* __restrict__ host_est,
               const uint32_t* __restrict__ n_valid, uint64_t* __restrict__ host_n) {
  __shared__ uint32_t pw[HLL_RG][64];
  __shared__ double zs[HLL_REGS / 64];
  __shared__ uint32_t zc[HLL_REGS / 64];
  const uint32_t w = threadIdx.x & 63, q = threadIdx.x >> 6;
  pw[q][w] = hll_rows_max(part, 0, n_part, w, q);
  __syncthreads();
  if (threadIdx.x < HLL_REGS) {                // one thread per register
    const uint32_t reg = threadIdx.x, wr = reg >> 2, sh = 8 * (reg & 3);
    uint32_t v = 0;
#pragma unroll
    for (uint32_t j = 0; j < HLL_RG; ++j) v = max(v, (pw[j][wr] >> sh) & 0xFFu);
    double z = ldexp(1.0, -(int)v);
    uint32_t zero = v == 0;
    for (int d = 32; d >= 1; d >>= 1) {
      z += __shfl_xor(z, d);
      zero += __shfl_xor(zero, d);
    }
    if (lane_id() == 0) { zs[threadIdx.x >> 6] = z; zc[threadIdx.x >> 6] = zero; }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double mm = HLL_REGS;
    const double zt = zs[0] + zs[1] + zs[2] + zs[3];
    const uint32_t zeros = zc[0] + zc[1] + zc[2] + zc[3];
    double e = 0.7213 / (1.0 + 1.079 / mm) * mm * mm / zt;
    if (e <= 2.5 * mm && zeros) e = mm * log(mm / (double)zeros);
    *host_est = e * (double)(1u << HLL_SAMPLE_BITS);
    if (host_n) *host_n = *n_valid;            // the keys the estimate is set against
  }
}

// ---------------------------------------------------------------- V_scatter (stable)
// Tile t = elements [t*PTILE, (t+1)*PTILE); wave w of the NWV waves owns the contiguous
// PTILE/NWV elements [t*PTILE + w*PTILE/NWV, ...), lane l holds element 64c + l of them.
// Element order inside the tile = (wave, c, lane) = input order, so ranks assigned in that
// order keep the pass stable.  FROM_SEQ (pass 0) encodes the windows from LDS-staged chars and
// drops invalid ones; later passes read the (key, pos) stream.  The tile is re-ordered by digit
// in LDS first and written out run by run, so each wave store covers a few contiguous runs
// instead of 64 scattered addresses.
// Persistent workgroup b walks virtual tiles b, b + G, ...: every XCD owns one contiguous tile
// range (xcd_remap), so the tiles running at the same time on an XCD are neighbours and their
// partial output lines merge in that XCD's L2.  Histograms are per tile; each tile's digit bases
// are prefetched with its inputs.
// (Removed in round 4 after measurement: 8-wave workgroups, +10 % at config 3, and a chunked
// schedule with per-chunk histograms, -10 %: each workgroup's open digit-run heads overflow the
// L2.)
constexpr int SC_NWV = 4;                       // waves per scatter workgroup
template <class KT>
struct ScatterLDS {
  static constexpr uint32_t MAXR = V2_MAXR_IL;
  uint32_t wc[SC_NWV][MAXR];   // per-wave digit counts -> per-wave tile-local cursors
  uint32_t tstart[MAXR];       // tile-local start of each digit
  uint32_t gbase[MAXR];        // global start of each digit for this tile (scanned histogram)
  KT skey[PTILE];
  uint32_t spos[PTILE];
  uint32_t sdst[PTILE];
  PStage st;
};

// Exclusive scan over the NWV * 64 threads of a block (one value per thread), lds >= NWV u64.
template <int NWV>
__device__ __forceinline__ uint64_t block_excl_scan_n(uint64_t v, uint64_t* lds, uint64_t& total) {
  const int wid = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(v);
  if (lane_id() == 63) lds[wid] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NWV; ++w) {
    const uint64_t x = lds[w];
    if (w < wid) off += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

// The same for u32 values whose block total fits 32 bits, the wave scans by DPP (no LDS permutes).
template <int NWV>
__device__ __forceinline__ uint32_t block_excl_scan_n32(uint32_t v, uint64_t* lds, uint64_t& total) {
  const int wid = threadIdx.x >> 6;
  const uint32_t inc = wave_incl_scan_u32(v);
  if (lane_id() == 63) lds[wid] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < NWV; ++w) {
    const uint64_t x = lds[w];
    if (w < wid) off += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return (uint32_t)off + inc - v;
}

// KEYS0: the first pass over a caller's key stream (a table rebuilt from keys): `kin` holds
// exactly n keys (loads clamped, no pad) and positions are implicit (e + 1), so the stream is
// neither copied nor paired with an iota array first.  NOPOS: keys only (count-only builds:
// nobody reads the positions), 8 B per element in and out instead of 12.
// BM (bucket-id streams, position builds that keep code words): 0 = (key u64, pos) elements;
// 1 = (bucket id u32, pos) in and out -- the digit needs no hash, and the key is cut from the
// code words by the bucket kernel; 2 = the last pass: (bucket id, pos) in, positions only out.
// kin / kout then point at u32 arrays.  8 B per element instead of 12 through the middle passes,
// 4 B out of the last.
// 3 = packed (key, pos) elements, 12 B each in kin / kout ({key lo, key hi, pos}; pin / pout
// unused): a tile's digit run leaves as ONE contiguous piece instead of an 8 c-byte piece of
// keys and a 4 c-byte piece of positions in two arrays; 4 = (key, pos) arrays in, packed out
// (the last pass of a build whose earlier streams stay unpacked for their histogram passes);
// 6 = the first pass from the sequence writing packed 8-B elements (Pack8, small k), 7 = the
// second pass reading them (each element's position restored from its segment, found in
// pk.segb by its place in the stream) and writing packed 12-B elements.  Write-pattern probe
// (tools/scatter_pattern.hip layout, profiles/r5a_scatter_layout.txt, 100 M elements): radix 313
// 1.09 -> 0.87 ms, radix 79 0.72 -> 0.61 ms.
// BALLOT: stable ranks from one ballot per digit bit instead of the count atomics' lane-ordered
// returns -- chosen at run time where the device self-check finds that order violated.
// DS (digit stream): the pass also writes every element's digit of the NEXT pass (u16, at the
// element's place in the output), which that pass's histogram reads instead of the keys.
template <bool FROM_SEQ, bool KEYS0 = false, bool NOPOS = false, int BM = 0, bool BALLOT = false,
          bool DS = false>
__global__ void __launch_bounds__(SC_NWV * 64)
k_v2_scatter(const uint8_t* __restrict__ seq, int64_t L, int k, int64_t Nw,
             const uint64_t* __restrict__ kin, const uint32_t* __restrict__ pin,
             const uint32_t* __restrict__ n_ptr, Geom g, Digit D,
             const uint32_t* __restrict__ hist, uint32_t ntiles,
             uint64_t* __restrict__ kout, uint32_t* __restrict__ pout, uint32_t pad,
             int skip_empty, BoundsFuse bf, Pack8 pk, DigitOut dso) {
  constexpr bool BIDS = BM == 1 || BM == 2;      // bucket-id streams
  constexpr bool AOS = BM == 3 || BM == 4 || BM == 7;   // packed 12-B (key, pos) elements out
  constexpr bool AIN = BM == 3;                   // ... and in
  constexpr bool P8OUT = BM == 6;                 // packed 8-B (key << sh | window) out
  constexpr bool P8IN = BM == 7;                  // ... in
  using KT = typename std::conditional<BIDS, uint32_t, uint64_t>::type;
  using SL = ScatterLDS<KT>;
  static_assert(!DS || BM != 2, "the last bucket-id pass has no next pass");
  static_assert(BM == 0 || !NOPOS, "bucket-id and packed streams carry positions");
  static_assert(!(AOS && KEYS0), "packed streams start from the sequence");
  // KEYS0 with BM: the first pass over V_hist0's per-window bucket ids (~0: not indexed)
  const KT* __restrict__ kinT = reinterpret_cast<const KT*>(kin);
  KT* __restrict__ koutT = reinterpret_cast<KT*>(kout);
  constexpr int NWV = SC_NWV;
  constexpr int TB = NWV * 64;                  // threads per workgroup
  constexpr int PER = PTILE / NWV / 64;         // elements per lane
  constexpr int DPT = (int)((SL::MAXR + TB - 1) / TB);   // digits owned per thread
  __shared__ SL S;
  __shared__ uint64_t sh[8];
  const uint32_t R = D.R;
  const int wave = threadIdx.x >> 6, lane = lane_id();
  const uint32_t wbase = (uint32_t)wave * (PTILE / NWV);
  // elements to read: every window (FROM_SEQ) or the caller's whole key stream (KEYS0, passed
  // as Nw: with skip_empty it is longer than the valid count the scan left in *n_ptr)
  const uint64_t n = (FROM_SEQ || KEYS0) ? (uint64_t)Nw : (uint64_t)*n_ptr;
  // thread t owns digits [DPT t, DPT t + DPT)
  const uint32_t G = gridDim.x;
  const uint32_t n_iter = (ntiles - blockIdx.x + G - 1) / G;
  // Each XCD walks its tile range from the END: the histogram pass before this one read the
  // same input ascending, so the tail it read last is still in the Infinity Cache when this
  // pass starts (-DKMHG_NO_REVERSE: ascending, A/B)
#ifndef KMHG_NO_REVERSE
  auto tile_at = [&](uint32_t i) -> uint32_t {
    return xcd_remap(blockIdx.x + (n_iter - 1 - i) * G, ntiles);
  };
#else
  auto tile_at = [&](uint32_t i) -> uint32_t { return xcd_remap(blockIdx.x + i * G, ntiles); };
#endif
  uint32_t ngb[DPT];
  auto load_bases = [&](uint32_t tv) {     // unconditional (clamped) loads: static count
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = min(threadIdx.x * DPT + q, R - 1);
      ngb[q] = hist[(size_t)d * ntiles + tv];
    }
  };
  // the folded bucket-start work (last pass only), before any tile's loads are issued
  if (bf.start)
    for (uint32_t lo = blockIdx.x; lo < bf.div; lo += gridDim.x)
      bounds_lo_body(lo, &S.wc[0][0], bf.kprev, *n_ptr, g, bf.Dlast, bf.div, hist, ntiles,
                     bf.lo_start, bf.spread, bf.start, bf.bid, TB, bf.nlim, bf.sh);
  // the next tile's inputs are in flight while this one is processed
  KT nkey[PER];
  uint32_t npos[PER];
  StageRegs<PSTAGE_W16> nchars;
  auto prefetch = [&](uint32_t tv) {
    const uint64_t t0 = (uint64_t)tv * PTILE;
    load_bases(tv);
    if (FROM_SEQ) {
      stage_load<PSTAGE_W16, true>(nchars, seq, L, (int64_t)t0 - HALO, true);
    } else {
#pragma unroll
      for (int cc = 0; cc < PER; ++cc) {   // e < ntiles * PTILE <= n_max + pad: in bounds
        const uint64_t e = t0 + wbase + (uint32_t)cc * 64 + lane;
        if (KEYS0) {
          nkey[cc] = kinT[e < n ? e : n - 1];    // positions implicit: e + 1 (below)
        } else if (AIN) {
          const uint3 v = reinterpret_cast<const uint3*>(kin)[e];
          nkey[cc] = ((uint64_t)v.y << 32) | v.x;
          npos[cc] = v.z;
        } else if (P8IN) {
          nkey[cc] = kinT[e];                  // position restored from the segment table
          npos[cc] = 0u;
        } else {
          nkey[cc] = kinT[e];
          npos[cc] = NOPOS ? 0u : pin[e];
        }
      }
    }
  };
  // Every path into the loop top has [prefetch loads][PTILE/TB x 2 stores] in flight, so the
  // compiler waits for the prefetch with a counted vmcnt: the pad stores below stand in for the
  // previous tile's write-out on the first iteration.
  prefetch(tile_at(0));
#pragma unroll
  for (int j = 0; j < PTILE / TB; ++j) {
    if (AOS) {
      reinterpret_cast<uint3*>(kout)[pad + threadIdx.x] = make_uint3(0u, 0u, 0u);
    } else {
      if (BM != 2) koutT[pad + threadIdx.x] = 0;
      if (!NOPOS && !P8OUT) pout[pad + threadIdx.x] = 0;
    }
    if constexpr (DS) {
      if (dso.out8) dso.out8[pad + threadIdx.x] = 0;
      else dso.out[pad + threadIdx.x] = 0;
    }
  }
  for (uint32_t it = 0; it < n_iter; ++it) {
    const uint32_t tile = tile_at(it);
    const uint64_t tile0 = (uint64_t)tile * PTILE;
    KT key[PER];
    uint32_t ps[PER], dg[PER];
    bool act[PER];
    uint32_t cursor[DPT];
#pragma unroll
    for (int q = 0; q < DPT; ++q) cursor[q] = ngb[q];
    if (FROM_SEQ) {
      stage_pack(nchars, S.st);
    } else {
#pragma unroll
      for (int cc = 0; cc < PER; ++cc) {
        key[cc] = nkey[cc];
        ps[cc] = KEYS0 ? (uint32_t)(tile0 + wbase + (uint32_t)cc * 64 + lane + 1) : npos[cc];
      }
    }
    prefetch(tile_at(min(it + 1, n_iter - 1)));   // unconditional: static vmcnt
    for (uint32_t d = lane; d < R; d += 64) S.wc[wave][d] = 0;
    __syncthreads();                       // stage packed; previous tile's write-out done
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const uint32_t w = wbase + (uint32_t)c * 64 + lane;     // element index inside the tile
      const uint64_t e = tile0 + w;
      if (FROM_SEQ) {
        uint64_t kk = 0;
        act[c] = e < n && window_key(S.st, HALO + (int)w, (int64_t)e, L, k, kk);
        ps[c] = (uint32_t)(e + 1);
        const uint64_t h = mix64(kk);
        const uint32_t bl = bucket_local(h, g);
        act[c] = act[c] && bl < g.nb;                        // a part build keeps its buckets
        key[c] = BIDS ? (KT)bl
                      : P8OUT ? (KT)((kk << pk.sh) | (e & ((1ull << pk.sh) - 1ull))) : (KT)kk;
        dg[c] = act[c] ? digit_of_b(bl, D) : 0;
      } else if (P8IN) {
        // key and window index from the packed element; the segment from the element's place
        // in its pass-0 digit run (segb row of that digit: the largest s with segb[s] <= e)
        act[c] = e < n;
        const uint64_t kk = (uint64_t)key[c] >> pk.sh;
        const uint64_t h = mix64(kk);
        dg[c] = act[c] ? digit_of_h(h, g, D) : 0;
        const uint32_t* row = pk.segb + (uint64_t)digit_of_h(h, g, pk.d0) * (pk.nseg + 1);
        uint32_t lo = 0, hi = pk.nseg;                       // row[0] <= e < row[nseg]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if ((uint64_t)row[mid] <= e) lo = mid; else hi = mid;
        }
        ps[c] = (uint32_t)((((uint64_t)lo << pk.sh) | ((uint64_t)key[c] & ((1ull << pk.sh) - 1ull))) + 1);
        key[c] = (KT)kk;
      } else if (BIDS) {
        act[c] = e < n && !(KEYS0 && (uint32_t)key[c] == ~0u);
        dg[c] = act[c] ? digit_of_b((uint32_t)key[c], D) : 0;
      } else {
        act[c] = e < n && !(KEYS0 && skip_empty && key[c] == EMPTY_KEY);
        const uint64_t hk = mix64((uint64_t)key[c]);
        dg[c] = act[c] ? digit_of_h(hk, g, D) : 0;
      }
    }
    if (!BALLOT) {
      // Stable ranks from the count atomics themselves: the lanes of one LDS instruction that
      // hit the same counter are served in lane order (CDNA4; kmhg_check_lds_lane_order checks
      // it on the device before the first build), and a wave's instructions run in program
      // order, so the returned running count is the element's rank among the wave's elements
      // of its digit in (c, lane) = input order.
      // (the rank rides in the digit's register, bits 16+: digit < 2^16, rank < PTILE)
#pragma unroll
      for (int c = 0; c < PER; ++c)
        if (act[c]) dg[c] |= atomicAdd(&S.wc[wave][dg[c]], 1u) << 16;
    } else {
#pragma unroll
      for (int c = 0; c < PER; ++c)          // counts only: order-free LDS atomics
        if (act[c]) atomicAdd(&S.wc[wave][dg[c]], 1u);
    }
    __syncthreads();
    // tile-local digit starts: thread t owns digits [DPT t, DPT t + DPT)
    uint32_t dsum[DPT];
    uint64_t own = 0;
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = threadIdx.x * DPT + q;
      uint32_t sum = 0;
      if (d < R) {
#pragma unroll
        for (int w = 0; w < NWV; ++w) sum += S.wc[w][d];
      }
      dsum[q] = sum;
      own += sum;
    }
    uint64_t tile_n;
#ifndef KMHG_NO_DPP_SCAN
    uint32_t run = block_excl_scan_n32<NWV>((uint32_t)own, sh, tile_n);   // own <= PTILE
#else
    uint32_t run = (uint32_t)block_excl_scan_n<NWV>(own, sh, tile_n);
#endif
#pragma unroll
    for (int q = 0; q < DPT; ++q) {
      const uint32_t d = threadIdx.x * DPT + q;
      if (d < R) {
        S.tstart[d] = run;
        S.gbase[d] = cursor[q];
        uint32_t cur = run;
#pragma unroll
        for (int w = 0; w < NWV; ++w) {
          const uint32_t t = S.wc[w][d];
          S.wc[w][d] = cur;
          cur += t;
        }
        run += dsum[q];
      }
    }
    __syncthreads();
    if (!BALLOT) {
#pragma unroll
      for (int c = 0; c < PER; ++c) {
        if (act[c]) {
          const uint32_t d = dg[c] & 0xFFFFu;
          const uint32_t ld = S.wc[wave][d] + (dg[c] >> 16);
          if (BM != 2) S.skey[ld] = key[c];      // the last bucket-id pass writes positions only
          S.spos[ld] = ps[c];
          S.sdst[ld] = S.gbase[d] + (ld - S.tstart[d]);
        }
      }
    } else {
#pragma unroll
      for (int c = 0; c < PER; ++c) {        // stable ranks: ballots over the digit bits
        const uint64_t grp = match_bits(dg[c], D.nbits, act[c]);
        const int leader = act[c] ? __ffsll((unsigned long long)grp) - 1 : lane;
        uint32_t cur = 0;
        if (act[c] && leader == lane) {
          cur = S.wc[wave][dg[c]];
          S.wc[wave][dg[c]] = cur + (uint32_t)__popcll(grp);
        }
        cur = __shfl(cur, leader);
        wave_sync();
        if (act[c]) {
          const uint32_t ld = cur + (uint32_t)__popcll(grp & lanemask_lt());
          if (BM != 2) S.skey[ld] = key[c];
          S.spos[ld] = ps[c];
          S.sdst[ld] = S.gbase[dg[c]] + (ld - S.tstart[dg[c]]);
        }
      }
    }
    __syncthreads();
    // a static count of store instructions per lane (masked, fully unrolled), so the wait for
    // the next tile's prefetched loads at the loop top is vmcnt(#stores), not vmcnt(0): the
    // prefetch was issued before these stores and must not queue behind their completion
#pragma unroll
    for (int j = 0; j < PTILE / TB; ++j) {
      const uint32_t i = (uint32_t)(j * TB) + threadIdx.x;
      // lanes past the tile's end store into the PTILE-element pad behind the outputs
      const uint32_t dst = i < (uint32_t)tile_n ? S.sdst[i] : pad + threadIdx.x;
      if (AOS) {
        const uint64_t kk = S.skey[i];
        reinterpret_cast<uint3*>(kout)[dst] = make_uint3((uint32_t)kk, (uint32_t)(kk >> 32), S.spos[i]);
      } else {
        if (BM != 2) koutT[dst] = S.skey[i];
        if (!NOPOS && !P8OUT) pout[dst] = S.spos[i];
      }
      if constexpr (DS) {       // the next pass's digit, from the staged key (no more LDS)
        const uint64_t kk = P8OUT ? (uint64_t)S.skey[i] >> pk.sh : (uint64_t)S.skey[i];
        const uint32_t dnx = BIDS ? digit_of_b((uint32_t)kk, dso.Dn) : digit_of(kk, g, dso.Dn);
        // (plain stores: the partial lines merge in the XCD's L2; nontemporal digit stores cost
        // the 500 Mbp build 16.86 -> 19.04 ms, profiles/r5y_variants_large_build_only.txt)
        if (dso.out8) dso.out8[dst] = (uint8_t)dnx;
        else dso.out[dst] = (uint16_t)dnx;
      }
    }
  }
}

// ---------------------------------------------------------------- V_bounds_lo
// Bucket starts from the radix histograms instead of a pass over the sorted keys.  With LSD
// passes, pass p's input is sorted by lo = c mod div (c = the element's digits 0 .. p combined,
// div = R^p) and the pass places elements by its own digit hi, stably, so
//   S_p[hi * div + lo] = #(digit < hi) + #(digit == hi and lo' < lo)
//                      = hist_p[hi][t] + #(digit hi among the pass's input [t * PTILE, P_lo))
// where P_lo = S_(p-1)[lo] = #(lo' < lo) is the start of lo in that input (for p = 1 pass 0's
// scanned column 0, saved by V_hist) and t = P_lo / PTILE: one workgroup per lo value counts at
// most one partial tile.  S_p of the last pass are the bucket starts; the earlier levels (3+
// passes) keep S_p (R^(p+1) entries, `nlim`) for the next.  Each level rides in its pass's
// scatter (BoundsFuse) -- it needs that pass's scanned histogram and its input, both live
// there -- so no key pass and no launch of its own.  Interleaved schedule only (one histogram
// column per tile).  `spread` (count-only builds): start[b / spread] for the buckets b that are
// multiples of spread.
__device__ __forceinline__ void bounds_lo_body(uint32_t lo, uint32_t* cnt,
                                               const uint64_t* __restrict__ kprev, uint32_t n,
                                               Geom g, Digit Dlast, uint32_t div,
                                               const uint32_t* __restrict__ hist, uint32_t C,
                                               const uint32_t* __restrict__ lo_start,
                                               uint32_t spread, uint32_t* __restrict__ start,
                                               int bid, int tb, uint32_t nlim, int sh = 0) {
  const uint32_t R = Dlast.R;
  const uint32_t P = lo_start ? lo_start[lo] : 0u;
  for (uint32_t d = threadIdx.x; d < R; d += tb) cnt[d] = 0;
  __syncthreads();
  const uint32_t tile = P / PTILE;
  for (uint32_t i = tile * PTILE + threadIdx.x; i < P; i += tb) {
    uint32_t dg;
    if (bid == 1) {                        // bucket ids
      dg = digit_of_b(reinterpret_cast<const uint32_t*>(kprev)[i], Dlast);
    } else if (bid == 2) {                 // packed (key, pos) elements
      const uint32_t* w = reinterpret_cast<const uint32_t*>(kprev) + 3 * (uint64_t)i;
      dg = digit_of(((uint64_t)w[1] << 32) | w[0], g, Dlast);
    } else if (bid == 3) {                 // packed 8-B elements: key << sh | window
      dg = digit_of(kprev[i] >> sh, g, Dlast);
    } else {
      dg = digit_of(kprev[i], g, Dlast);
    }
    atomicAdd(&cnt[dg], 1u);
  }
  __syncthreads();
  for (uint32_t hi = threadIdx.x; hi < R; hi += tb) {
    const uint64_t b = (uint64_t)hi * div + lo;
    if (b >= nlim || b % spread) continue;
    // P == n on a tile boundary past the last column: the end of digit hi
    const uint32_t base = tile < C ? hist[(size_t)hi * C + tile]
                                   : (hi + 1 < R ? hist[(size_t)(hi + 1) * C] : n);
    start[b / spread] = base + cnt[hi];
  }
  if (lo == 0 && threadIdx.x == 0) start[nlim / spread] = n;
  __syncthreads();                         // cnt is the caller's LDS: free again
}

__global__ void __launch_bounds__(BLOCK)
k_v2_bounds_lo(const uint64_t* __restrict__ kprev, const uint32_t* __restrict__ n_ptr, Geom g,
               Digit Dlast, uint32_t div, const uint32_t* __restrict__ hist, uint32_t C,
               const uint32_t* __restrict__ lo_start, uint32_t spread,
               uint32_t* __restrict__ start, int bid, uint32_t nlim, int sh) {
  __shared__ uint32_t cnt[V2_MAXR];
  bounds_lo_body(blockIdx.x, cnt, kprev, *n_ptr, g, Dlast, div, hist, C, lo_start, spread, start,
                 bid, BLOCK, nlim, sh);
}

// Pack8's segment table: segb[d * (nseg + 1) + s] = where segment s (tiles [s tps, (s + 1) tps))
// of pass-0 digit d starts in pass 0's output -- the scanned histogram entry (d, s tps), or the
// end of digit d's run past the last tile.
__global__ void __launch_bounds__(BLOCK)
k_seg_bounds(const uint32_t* __restrict__ hist, uint32_t ntiles, uint32_t R, uint32_t nseg,
             uint32_t tps, const uint32_t* __restrict__ n_valid, uint32_t* __restrict__ segb) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= R * (nseg + 1)) return;
  const uint32_t d = i / (nseg + 1), sg = i % (nseg + 1);
  const uint64_t t = (uint64_t)sg * tps;
  segb[i] = t < ntiles ? hist[(size_t)d * ntiles + t]
                       : (d + 1 < R ? hist[(size_t)(d + 1) * ntiles] : *n_valid);
}

// The radix passes are stable by the lane order of the LDS count atomics (V_scatter), so a
// bucket's stream lists its windows in ascending position -- the order the position lists keep.
// The bucket kernels check it with one neighbour load per element and report a violation like
// an LDS table overflow, which rebuilds the index with the global-atomic build (finish_build).
// (pos: the stream's positions, every `stride`-th word: 3 in a packed (key, pos) stream)
template <int STRIDE = 1>
__device__ __forceinline__ bool stream_out_of_order(const uint32_t* __restrict__ pos, uint32_t i,
                                                    uint32_t s0, uint32_t s1, uint32_t p) {
  return i > s0 && i < s1 && pos[(uint64_t)(i - 1) * STRIDE] >= p;
}

// ---------------------------------------------------------------- V_bucket_wg (group per bucket)
// ONE WORKGROUP per bucket (V2_BW_WG windows on average) with one shared LDS sub-table of
// V2_CAPW slots, 12 B per slot (8-B key + one u32 `val`: 18.4 KB, so 8 workgroups fit a CU's
// LDS).  `val` is the count during pass A; the counts pass moves every slot's count into the
// registers of the thread that owns the slot for the write-out (slot q * TB + t), and `val`
// becomes the inline position of a key seen once or the list cursor of a repeated key, tagged
// VAL_MULTI so that pass B can tell them apart.
// (Removed in round 4 after measurement, see DESIGN.md §5: one wave per 256-window bucket, a
// 16-B-per-slot table, 8-wave workgroups, a one-atomic fingerprint insert, a sort-based bucket
// build, and slot tags written by the build.)
struct GroupTableC {
  uint64_t key[V2_CAPW + 1];
  uint32_t val[V2_CAPW + 1];
};
constexpr uint32_t VAL_MULTI = 0x80000000u;    // positions and list offsets are < 2^31

// Find-or-insert by CAS only.  (Measured, 10 Mbp: a plain read before the CAS 0.098 -> 0.186 ms;
// the claiming occurrence skipping its count atomic 0.098 -> 0.136 ms; a per-lane state machine
// over a lane's elements, one CAS per trip, 0.098 -> 0.204 ms.)
__device__ __forceinline__ int lds_insert_g(GroupTableC& W, uint64_t key, uint64_t h) {
  if (key == EMPTY_KEY) return (int)V2_CAPW;
  uint32_t j = local_home(h, V2_CAPW);
  for (uint32_t n = 0; n < V2_CAPW; ++n) {
    const uint64_t prev = atomicCAS((unsigned long long*)&W.key[j],
                                    (unsigned long long)EMPTY_KEY, (unsigned long long)key);
    if (prev == EMPTY_KEY || prev == key) return (int)j;
    if (++j == V2_CAPW) j = 0;
  }
  return -1;
}

__device__ __forceinline__ int lds_find_g(const GroupTableC& W, uint64_t key) {
  if (key == EMPTY_KEY) return (int)V2_CAPW;
  uint32_t j = local_home(mix64(key), V2_CAPW);
  for (uint32_t n = 0; n < V2_CAPW; ++n) {
    if (W.key[j] == key) return (int)j;
    if (++j == V2_CAPW) j = 0;
  }
  return -1;
}

// COUNT_ONLY (occurrence counts of a key stream, kmhg_sh.hip's read counting): pass B -- the
// positions -- is skipped; slots get {key, count, unspecified aux}.
// CK (bucket-id streams): the stream holds positions only; each window's key is cut from the
// sequence's code words (`code`, 16 chars per u32) at its position -- three loads per window
// from a 0.25 B/window array, against 8 B of key per window carried through every radix pass.
// BALLOT: repeated keys' windows ranked by ballots instead of the cursor atomic's lane order.
// Every key must hash to this bucket: a stream entry that does not (an unstable pass moving
// another bucket's window in) is reported like an LDS overflow.
#ifndef KMHG_NO_NT_TABLE
constexpr bool NT_TABLE = true;                // (-DKMHG_NO_NT_TABLE: plain stores, A/B)
#else
constexpr bool NT_TABLE = false;
#endif
struct Words3 {                                // three consecutive code words, 4-B aligned
  uint32_t a, b, c;
};
// AOS: the stream is packed 12-B (key, pos) elements in `keys` (`pos` unused).
// TAGS (position builds beyond the cache, round 6): the diagonal query path's preparation comes
// with the build -- each slot's tag byte TG[slot] (0 empty, else slot_tag of its key's hash: the
// same bytes V_diag_prep would write), and for every window of a repeated key its bit in `rep`
// (u32 word (pos - 1) / 32, zeroed before the launch), so the first query runs V_diag_valid
// alone (uniq = indexed windows AND NOT rep).
template <bool COUNT_ONLY, bool CK, bool BALLOT, bool AOS = false, bool TAGS = false>
__global__ void __launch_bounds__(BLOCK, BALLOT ? 4 : KMHG_BUCKET_WGS)
k_v2_bucket_wg(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ pos,
               const uint32_t* __restrict__ start, Geom g, Slot* __restrict__ T,
               int32_t* __restrict__ positions, BucketStats* __restrict__ bstats,
               BuildMeta* __restrict__ meta, const uint32_t* __restrict__ code, int k,
               const uint32_t* __restrict__ n_ptr, uint32_t nw, uint8_t* __restrict__ TG,
               uint32_t* __restrict__ rep) {
  static_assert(!(CK && COUNT_ONLY), "code-word keys belong to position builds");
  static_assert(!(TAGS && (CK || COUNT_ONLY)), "build-time tags: key-stream position builds");
  static_assert(!(AOS && (CK || COUNT_ONLY)), "packed streams carry keys and positions");
  static_assert(V2_CAPW % BLOCK == 0, "the side slot V2_CAPW is slot q = V2_CAPW / TB of thread 0");
  constexpr int TB = BLOCK;
  constexpr int NW = TB / 64;                         // waves of the workgroup
  __shared__ GroupTableC W;
  __shared__ uint64_t sh[2 * NW];
  __shared__ uint32_t red[2][NW];
  const uint32_t b = blockIdx.x;
  // elements per thread per batch: 2x the mean (code words: 1.5x, for the VGPR budget of
  // 8 waves / SIMD); a larger bucket takes more batches
  constexpr int PER = (CK ? 3 : 4) * V2_BW_WG / 2 / TB;
  constexpr int EW = (PER + 1) & ~1;                  // edge row: PER positions, written as pairs
  __shared__ __attribute__((aligned(16))) uint32_t edge[EW * NW + 1];   // stream-order check
  constexpr uint32_t BATCH = TB * PER;
  const int wave = threadIdx.x >> 6, lane = lane_id();
  const uint32_t s0 = start[b], s1 = start[b + 1];
  // a bucket range outside the stream (a bounds error) is reported like an overflow, never
  // dereferenced: the index is rebuilt by the global-atomic build
  if (s0 > s1 || s1 > *n_ptr) {
    if (threadIdx.x == 0) atomicOr(&meta->overflow, 1u);
    return;
  }
  const bool one_batch = s1 - s0 <= BATCH;
  uint64_t key[PER];
  uint32_t ps[PER];
  int slot[PER];
  // element c of thread t in a batch: i0 + c * TB + t, so position order = (c, wave, lane)
  auto elem = [&](uint32_t i0, int c) { return i0 + (uint32_t)c * TB + threadIdx.x; };
  uint32_t wa[PER], wb[PER], wc[PER];                 // CK: each window's three code words
  bool ovf = false;                                   // LDS table full
  bool disorder = false;                              // the bucket's stream out of position order
  // CK: load() issues the positions, then the code words, all in flight at once; cut() turns
  // them into keys -- after the table clear for the first batch, so the clear hides the loads
  auto load = [&](uint32_t i0) {
    if (CK) {
#pragma unroll
      for (int c = 0; c < PER; ++c) {
        const uint32_t i = elem(i0, c);
#ifdef KMHG_EXP_NTLOAD
        ps[c] = i < s1 ? __builtin_nontemporal_load(pos + i) : 1u;
#else
        ps[c] = i < s1 ? pos[i] : 1u;               // 1-based window start
#endif
        if (!one_batch) disorder |= stream_out_of_order(pos, i, s0, s1, ps[c]);
      }
#pragma unroll
      for (int c = 0; c < PER; ++c) {       // one 12-B load per window (global_load_dwordx3)
        // clamped: a position outside [1, nw] (a stream error, flagged in pass A) never
        // turns into a code-word address outside the array
        const Words3 w3 = *reinterpret_cast<const Words3*>(code + (min(ps[c] - 1u, nw - 1u) >> 4));
        wa[c] = w3.a;
        wb[c] = w3.b;
        wc[c] = w3.c;
      }
      return;
    }
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const uint32_t i = elem(i0, c);
      if (AOS) {
        const uint3 v = i < s1 ? reinterpret_cast<const uint3*>(keys)[i] : make_uint3(0u, 0u, 0u);
        key[c] = ((uint64_t)v.y << 32) | v.x;
        ps[c] = v.z;
      } else {
        key[c] = i < s1 ? keys[i] : 0;
        ps[c] = (!COUNT_ONLY && i < s1) ? pos[i] : 0;
      }
      if (!COUNT_ONLY && i < s1 && ps[c] - 1u >= nw) disorder = true;   // outside [1, nw]
      if (!COUNT_ONLY && !one_batch)
        disorder |= AOS ? stream_out_of_order<3>(reinterpret_cast<const uint32_t*>(keys) + 2, i,
                                                  s0, s1, ps[c])
                        : stream_out_of_order(pos, i, s0, s1, ps[c]);
    }
  };
  auto cut = [&](uint32_t i0) {
    if (CK) {
#pragma unroll
      for (int c = 0; c < PER; ++c)
        key[c] = elem(i0, c) < s1 ? code_key(wa[c], wb[c], wc[c], (int64_t)ps[c] - 1, k) : 0;
    }
  };
  STAMP_WG(b, 0);
  load(s0);                                           // in flight while the table is cleared
  for (uint32_t j = threadIdx.x; j <= V2_CAPW; j += TB) {
    W.key[j] = EMPTY_KEY;
    W.val[j] = 0u;
  }
  __syncthreads();
  cut(s0);
  STAMP_WG(b, 1);
  STAMP_WG_DRAIN(b, 6);
  // pass A: distinct keys + counts (CAS on a table shared by the four waves).  (Measured round
  // 3, A/B in one run: letting the claiming occurrence skip the count add -- counts pass adds 1
  // per occupied slot -- made the kernel 100 -> 142 us, as in round 2; and issuing the first
  // CAS of all 8 elements of a lane back to back before resolving any, 98 -> 112 us.)
  for (uint32_t i0 = s0; i0 < s1; i0 += BATCH) {
    if (i0 != s0) { load(i0); cut(i0); }
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      slot[c] = -1;
      if (elem(i0, c) < s1) {
        // bucket membership (one multiply-high: CK keys are cut from the code words at the
        // stream's positions, so this checks the positions too)
        const uint64_t h = mix64(key[c]);
        if (bucket_local(h, g) != b) disorder = true;
        slot[c] = lds_insert_g(W, key[c], h);
        if (slot[c] < 0) ovf = true;
        else atomicAdd(&W.val[slot[c]], 1u);
      }
    }
    if (CK) {                      // positions in [1, nw] (checked after the cut: fewer live VGPRs)
#pragma unroll
      for (int c = 0; c < PER; ++c)
        if (elem(i0, c) < s1 && ps[c] - 1u >= nw) disorder = true;
    }
  }
  // Stream order of a one-batch bucket (multi-batch buckets check it with a neighbour load per
  // element in load()): element (c, wave, lane) follows (c, wave, lane - 1) -- a DPP shift --
  // and lane 0 follows lane 63 of the wave before (of row c - 1 for wave 0), exchanged through
  // `edge` and read after the barrier below.  Here, after pass A, the positions have long
  // arrived, so the check makes no load wait earlier than it did.
  const bool chk = !COUNT_ONLY && one_batch;
  // (edge: row `wave` holds that wave's lane-63 positions, EW per row, written and read as
  // pairs -- a handful of LDS instructions per wave: single-lane LDS instructions cost nearly a
  // full one each in this LDS-bound kernel)
  if (chk) {
    if (threadIdx.x == 0) edge[EW * NW] = 0u;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      // lane - 1's position by a DPP wave shift (a VALU move; __shfl_up is an LDS permute)
      const uint32_t up = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)ps[c], 0x138 /* wave_shr:1 */,
                                                                0xF, 0xF, false);
      if (lane > 0 && elem(s0, c) < s1 && up >= ps[c]) disorder = true;
    }
    if (lane == 63) {
#pragma unroll
      for (int q = 0; q < PER; q += 2)
        *reinterpret_cast<uint2*>(&edge[EW * wave + q]) = make_uint2(ps[q], q + 1 < PER ? ps[q + 1] : 0u);
    }
  }
  if (__syncthreads_or(ovf || disorder)) {
    if (threadIdx.x == 0) atomicOr(&meta->overflow, 1u);
    return;
  }
  if (chk && lane == 0) {
    // lane 0 of wave w follows lane 63 of wave w - 1 (same row); wave 0 follows wave NW - 1
    const uint32_t* row = edge + EW * (wave ? wave - 1 : NW - 1);
    uint32_t pv[PER + 1];
#pragma unroll
    for (int q = 0; q < PER; q += 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(&row[q]);
      pv[q] = v.x;
      pv[q + 1] = v.y;
    }
    bool bad = false;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const uint32_t e = elem(s0, c);
      const uint32_t prev = wave ? pv[c] : (c ? pv[c - 1] : 0u);   // wave 0: row c - 1
      bad |= e > s0 && e < s1 && prev >= ps[c];
    }
    if (bad) edge[EW * NW] = 1u;             // read after the counts pass's barrier
  }
  STAMP_WG(b, 2);
  // counts: thread t owns slots t, t + TB, ... (lane-contiguous: conflict-free LDS; thread-
  // contiguous runs of 6 slots ran 0.104 ms against 0.096 for the kernel)
  constexpr uint32_t SPT = (V2_CAPW + 1 + TB - 1) / TB;
  uint32_t cnt[SPT];
  uint32_t cs = 0;
#ifndef KMHG_NO_LEAN_COUNTS
  // The bucket's distinct keys by ballots (no cross-lane shuffles: each __shfl_xor is an LDS
  // permute, in a kernel bound by its LDS instructions); the count maximum and the pairs only
  // when some key is repeated, which the i.i.d. buckets of a large build almost never have.
  uint32_t occ_w = 0;                      // wave-uniform
  bool multi = false;
#pragma unroll
  for (uint32_t q = 0; q < SPT; ++q) {
    const uint32_t j = q * TB + threadIdx.x;
    const uint32_t c = j <= V2_CAPW ? W.val[j] : 0u;
    cnt[q] = c;
    cs += c;
    multi |= c > 1;
    occ_w += (uint32_t)__popcll(__ballot(c != 0));
  }
  if (lane == 0) red[0][wave] = occ_w;
  const bool has_multi = __syncthreads_or(multi);
  if (has_multi) {                         // block-uniform
    uint32_t mx = 0;
    uint64_t pairs = 0;
#pragma unroll
    for (uint32_t q = 0; q < SPT; ++q) {
      mx = max(mx, cnt[q]);
      pairs += (uint64_t)cnt[q] * (cnt[q] - (cnt[q] ? 1u : 0u)) / 2;
    }
    for (int d = 32; d >= 1; d >>= 1) {
      pairs += __shfl_xor(pairs, d);
      mx = max(mx, (uint32_t)__shfl_xor(mx, d));
    }
    if (lane == 0) {
      red[1][wave] = mx;
      sh[NW + wave] = pairs;               // sh[NW..2NW): the block scan below uses sh[0..NW)
    }
    __syncthreads();
  }
#else
  uint32_t occ = 0, mx = 0;
  uint64_t pairs = 0;
#pragma unroll
  for (uint32_t q = 0; q < SPT; ++q) {
    const uint32_t j = q * TB + threadIdx.x;
    const uint32_t c = j <= V2_CAPW ? W.val[j] : 0u;
    cnt[q] = c;
    cs += c;
    occ += c ? 1u : 0u;
    mx = max(mx, c);
    pairs += (uint64_t)c * (c - (c ? 1u : 0u)) / 2;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    pairs += __shfl_xor(pairs, d);
    occ += __shfl_xor(occ, d);
    mx = max(mx, (uint32_t)__shfl_xor(mx, d));
  }
  if (lane == 0) {
    red[0][wave] = occ;
    red[1][wave] = mx;
    sh[NW + wave] = pairs;                 // sh[NW..2NW): the block scan below uses sh[0..NW)
  }
  const bool has_multi = __syncthreads_or(mx > 1);
#endif
  if (chk && edge[EW * NW]) {                // stream out of order at a wave / row boundary
    if (threadIdx.x == 0) atomicOr(&meta->overflow, 1u);
    return;
  }
  // list offsets (only repeated keys have lists): any slot order gives each key a contiguous
  // range of [s0, s1), here slot q * TB + t in (t, q) order
  if (!COUNT_ONLY && has_multi) {
    uint64_t tot;
    uint32_t off_run = s0 + (uint32_t)block_excl_scan_n<NW>(cs, sh, tot);
#pragma unroll
    for (uint32_t q = 0; q < SPT; ++q) {
      const uint32_t j = q * TB + threadIdx.x;
      if (j <= V2_CAPW) W.val[j] = cnt[q] > 1 ? (VAL_MULTI | off_run) : off_run;
      off_run += cnt[q];
    }
    __syncthreads();
  }
  STAMP_WG(b, 3);
  if (threadIdx.x == 0) {
    BucketStats st;
    st.n_kmers = 0;
    st.max_count = 0;
    st.n_pairs = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) st.n_kmers += red[0][w];
#ifndef KMHG_NO_LEAN_COUNTS
    if (!has_multi) {
      st.max_count = st.n_kmers ? 1u : 0u;
    } else
#endif
    {
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        st.max_count = max(st.max_count, red[1][w]);
        st.n_pairs += sh[NW + w];
      }
    }
    bstats[b] = st;
  }
  // pass B: keys seen once keep their position inline (val); repeated keys are ranked in
  // position order, the waves taking turns so that wave w follows waves < w
  for (uint32_t i0 = s0; i0 < (COUNT_ONLY ? s0 : s1); i0 += BATCH) {
    if (!one_batch) {
      load(i0);
      cut(i0);
#pragma unroll
      for (int c = 0; c < PER; ++c) slot[c] = elem(i0, c) < s1 ? lds_find_g(W, key[c]) : -1;
    }
    if (!has_multi) {                    // every key seen once: positions go inline
#pragma unroll
      for (int c = 0; c < PER; ++c)
        if (elem(i0, c) < s1) W.val[slot[c]] = ps[c];
      continue;
    }
    for (int c = 0; c < PER; ++c) {
      const bool act = elem(i0, c) < s1;
      // waves take turns on this c: wave w ranks after waves < w have advanced the cursors
      for (int turn = 0; turn < NW; ++turn) {
        if (wave == turn) {
          const uint32_t v = act ? W.val[slot[c]] : 0u;
          const bool multi = act && (v & VAL_MULTI);
          if (act && !multi) W.val[slot[c]] = ps[c];
          if (!BALLOT) {
            // the cursor atomic's lane-ordered returns rank the wave's windows of one key
            if (multi) {
              const uint32_t at = atomicAdd(&W.val[slot[c]], 1u) & ~VAL_MULTI;
              positions[at] = (int32_t)ps[c];
              if (TAGS) atomicOr(&rep[(ps[c] - 1u) >> 5], 1u << ((ps[c] - 1u) & 31u));
            }
          } else if (__ballot(multi)) {
            const uint64_t m = match_bits((uint32_t)slot[c], V2_SLOT_BITS_WG, multi);
            const int leader = multi ? __ffsll((unsigned long long)m) - 1 : lane;
            if (multi && leader == lane) W.val[slot[c]] = v + (uint32_t)__popcll(m);
            const uint32_t cur = (uint32_t)__shfl((int)v, leader) & ~VAL_MULTI;
            if (multi) positions[cur + (uint32_t)__popcll(m & lanemask_lt())] = (int32_t)ps[c];
            if (TAGS && multi) atomicOr(&rep[(ps[c] - 1u) >> 5], 1u << ((ps[c] - 1u) & 31u));
          }
        }
        __syncthreads();
      }
    }
  }
  __syncthreads();
  STAMP_WG(b, 4);
  // the bucket's sub-table, coalesced 16-B slots, counts from the registers of the slot's owner
  Slot* Tb = T + (uint64_t)b * V2_CAPW;
#ifdef KMHG_EXP_SLOT8
  // EXPERIMENT ONLY (timing variant, wrong tables): the write-out of 8-B {count, aux} slots
  uint2* T8 = reinterpret_cast<uint2*>(T) + (uint64_t)b * V2_CAPW;
#pragma unroll
  for (uint32_t q = 0; q < SPT; ++q) {
    const uint32_t j = q * TB + threadIdx.x;
    if (j < V2_CAPW) T8[j] = make_uint2(cnt[q], COUNT_ONLY ? 0u : (W.val[j] & ~VAL_MULTI));
  }
#else
#pragma unroll
  for (uint32_t q = 0; q < SPT; ++q) {
    const uint32_t j = q * TB + threadIdx.x;
    if (j < V2_CAPW) {
      const uint64_t kk = W.key[j];
      const uint32_t aux = COUNT_ONLY ? 0u : (W.val[j] & ~VAL_MULTI);
      if (CK && NT_TABLE) {
        // code-word keys: the table streams past the L2 (nontemporal), which keeps the code
        // words every bucket gathers from resident there
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 sv = {(uint32_t)kk, (uint32_t)(kk >> 32), cnt[q], aux};
        __builtin_nontemporal_store(sv, reinterpret_cast<u32x4*>(&Tb[j]));
      } else {
        *reinterpret_cast<uint4*>(&Tb[j]) = make_uint4((uint32_t)kk, (uint32_t)(kk >> 32), cnt[q], aux);
      }
      if (TAGS)      // one byte per slot: 64 consecutive bytes per wave and row q
        TG[(uint64_t)b * V2_CAPW + j] = kk == EMPTY_KEY ? (uint8_t)0 : slot_tag(mix64(kk));
    }
  }
#endif
  if (threadIdx.x == 0 && side_bucket(b, g)) {
    const uint2 c = make_uint2(cnt[V2_CAPW / TB], COUNT_ONLY ? 0u : (W.val[V2_CAPW] & ~VAL_MULTI));
    *reinterpret_cast<uint4*>(&T[side_slot(g)]) = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, c.x, c.y);
  }
  STAMP_WG(b, 5);
}

// V_stats: reduce the per-bucket partials (grid-stride, one atomic per workgroup; meta was
// zeroed by V_hist0).  The last workgroup to finish copies the totals into `host_meta`, a
// pinned host record, so the host reads them without a copy launch.
constexpr int STATS_PER = 8;
__global__ void __launch_bounds__(BLOCK)
k_v2_stats(const BucketStats* __restrict__ bs, uint32_t nb, const uint32_t* __restrict__ n_valid,
           BuildMeta* __restrict__ meta, BuildMeta* __restrict__ host_meta) {
  __shared__ uint64_t su[4], sp[4];
  __shared__ uint32_t sm[4];
  uint64_t u = 0, p = 0;
  uint32_t m = 0;
  // STATS_PER buckets per thread and trip, their loads all in flight before any is summed (a
  // plain grid-stride loop waits out one load latency per bucket)
  const uint32_t stride = gridDim.x * BLOCK;
  for (uint32_t b0 = blockIdx.x * BLOCK + threadIdx.x; b0 < nb; b0 += stride * STATS_PER) {
    BucketStats x[STATS_PER];
#pragma unroll
    for (int q = 0; q < STATS_PER; ++q) {
      const uint32_t b = b0 + q * stride;
      x[q] = b < nb ? bs[b] : BucketStats{0u, 0u, 0ull};
    }
#pragma unroll
    for (int q = 0; q < STATS_PER; ++q) {
      u += x[q].n_kmers;
      p += x[q].n_pairs;
      m = max(m, x[q].max_count);
    }
  }
  u = wave_sum(u);
  p = wave_sum(p);
  m = (uint32_t)lane63(wave_incl_max(m));
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) { su[w] = u; sp[w] = p; sm[w] = m; }
  __syncthreads();
  if (threadIdx.x == 0) {
    u = su[0] + su[1] + su[2] + su[3];
    p = sp[0] + sp[1] + sp[2] + sp[3];
    m = max(max(sm[0], sm[1]), max(sm[2], sm[3]));
    if (u) atomicAdd((unsigned long long*)&meta->n_kmers, (unsigned long long)u);
    if (p) atomicAdd((unsigned long long*)&meta->n_pairs, (unsigned long long)p);
    if (m) atomicMax(&meta->max_count, m);
    __threadfence();
    const uint32_t done = atomicAdd(&meta->blocks_done, 1u);
    if (done == gridDim.x - 1) {           // every other block's atomics are visible
      __threadfence();
      BuildMeta r;
      r.n_kmers = __hip_atomic_load(&meta->n_kmers, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.n_pairs = __hip_atomic_load(&meta->n_pairs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.max_count = __hip_atomic_load(&meta->max_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.overflow = __hip_atomic_load(&meta->overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      r.n_positions = *n_valid;
      r.n_small = 0;
      r.n_large = 0;
      r.blocks_done = done + 1;
      r.distinct_est = 0;
      *host_meta = r;
      __threadfence_system();
    }
  }
}

#ifdef KMHG_STAMPS
void set_stamp_buffer(uint64_t* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &p, sizeof(p)); }
#endif

// ---------------------------------------------------------------- V_part_dense
// A part build's compacted tiles (V_hist0 PARTC) into one dense stream: tile t's off[t+1] -
// off[t] elements (off = the scanned tile counts, off[ntiles] = *n_total) move from
// [t * PTILE, ...) to [off[t], ...), keys and positions, order kept.
// AOS: the dense stream is packed 12-B (key, pos) elements in dk (dp unused).
template <bool AOS>
__global__ void __launch_bounds__(BLOCK)
k_part_dense(const uint64_t* __restrict__ ck, const uint32_t* __restrict__ cp,
             const uint32_t* __restrict__ off, uint32_t ntiles,
             const uint32_t* __restrict__ n_total, uint64_t* __restrict__ dk,
             uint32_t* __restrict__ dp) {
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t o0 = off[t], o1 = t + 1 < ntiles ? off[t + 1] : *n_total;
    const uint64_t src = (uint64_t)t * PTILE;
    for (uint32_t i = threadIdx.x; i < o1 - o0; i += BLOCK) {
      if (AOS) {
        const uint64_t kk = ck[src + i];
        reinterpret_cast<uint3*>(dk)[o0 + i] = make_uint3((uint32_t)kk, (uint32_t)(kk >> 32), cp[src + i]);
      } else {
        dk[o0 + i] = ck[src + i];
        dp[o0 + i] = cp[src + i];
      }
    }
  }
}

// ---------------------------------------------------------------- launchers
// Persistent grids: as many workgroups as are resident at once (CUs x the occupancy the
// kernel's VGPR/LDS budget allows), so no workgroup waits for another to finish.
static unsigned resident_blocks(const void* kernel, int threads = BLOCK) {
  int dev = 0, cus = 256, per = 1;
  if (hipGetDevice(&dev) == hipSuccess)
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, threads, 0) != hipSuccess ||
      per < 1)
    per = 1;
  return (unsigned)(cus > 0 ? cus : 256) * (unsigned)per;
}

static inline unsigned grid_of(uint64_t n, unsigned per) {
  uint64_t g = (n + per - 1) / per;
  return (unsigned)(g ? g : 1);
}

// The lane order of same-address LDS atomics, checked once per device (kmhg_check_lds_lane_order
// runs the same kernel for the tests): where it does not hold, every build takes the ballot-rank
// kernels.  KMHG_TEST_BALLOT=1 (tests) forces them.
bool ballot_ranks();

#define KMHG_SCATTER_X(FS, K0, NP, BM, DSF, DSO, ...)                                         \
  do {                                                                                       \
    if (ballot_ranks()) {                                                                    \
      static const unsigned cap_ =                                                           \
          resident_blocks((const void*)k_v2_scatter<FS, K0, NP, BM, true, DSF>, SC_NWV * 64); \
      hipLaunchKernelGGL((k_v2_scatter<FS, K0, NP, BM, true, DSF>), dim3(std::min(ntiles, cap_)), \
                         dim3(SC_NWV * 64), 0, s, __VA_ARGS__, DSO);                         \
    } else {                                                                                 \
      static const unsigned cap_ =                                                           \
          resident_blocks((const void*)k_v2_scatter<FS, K0, NP, BM, false, DSF>, SC_NWV * 64); \
      hipLaunchKernelGGL((k_v2_scatter<FS, K0, NP, BM, false, DSF>), dim3(std::min(ntiles, cap_)), \
                         dim3(SC_NWV * 64), 0, s, __VA_ARGS__, DSO);                         \
    }                                                                                        \
  } while (0)
#define KMHG_SCATTER_BM(FS, K0, NP, BM, ...) KMHG_SCATTER_X(FS, K0, NP, BM, false, kNoDigits, __VA_ARGS__)
// the same pass also writing the next pass's digits (dso)
#define KMHG_SCATTER_BMD(FS, K0, NP, BM, DSO, ...)                                            \
  do {                                                                                       \
    if (DSO.out || DSO.out8) KMHG_SCATTER_X(FS, K0, NP, BM, true, DSO, __VA_ARGS__);                      \
    else KMHG_SCATTER_X(FS, K0, NP, BM, false, kNoDigits, __VA_ARGS__);                       \
  } while (0)
#define KMHG_SCATTER(FS, K0, NP, ...) KMHG_SCATTER_BM(FS, K0, NP, 0, __VA_ARGS__)

void launch_v2_hist0(const uint8_t* seq, int64_t L, int k, int64_t Nw, Geom g, Digit D,
                     uint32_t* hist, uint32_t ntiles, uint64_t* scan_status, uint32_t n_status,
                     BuildMeta* meta, hipStream_t s, uint32_t* code, uint16_t* nbit,
                     uint32_t* bids, uint64_t* ckeys, uint32_t* cpos, uint32_t* tcnt) {
  if (ckeys) {                 // a part build's compacted windows (keep the code words)
    static const unsigned cap_p = resident_blocks((const void*)k_v2_hist0p<true, false, true>);
    hipLaunchKernelGGL((k_v2_hist0p<true, false, true>), dim3(std::min<unsigned>(ntiles, cap_p)),
                       dim3(BLOCK), 0, s, seq, L, k, Nw, g, D, hist, ntiles, scan_status,
                       n_status, meta, code, nbit, nullptr, ckeys, cpos, tcnt);
  } else if (bids) {           // bucket-id builds (keep the code words)
    static const unsigned cap_b = resident_blocks((const void*)k_v2_hist0p<true, true>);
    hipLaunchKernelGGL((k_v2_hist0p<true, true>), dim3(std::min<unsigned>(ntiles, cap_b)),
                       dim3(BLOCK), 0, s, seq, L, k, Nw, g, D, hist, ntiles, scan_status,
                       n_status, meta, code, nbit, bids, nullptr, nullptr, nullptr);
  } else if (code && nbit) {
    static const unsigned cap_c = resident_blocks((const void*)k_v2_hist0p<true, false>);
    hipLaunchKernelGGL((k_v2_hist0p<true, false>), dim3(std::min<unsigned>(ntiles, cap_c)),
                       dim3(BLOCK), 0, s, seq, L, k, Nw, g, D, hist, ntiles, scan_status,
                       n_status, meta, code, nbit, nullptr, nullptr, nullptr, nullptr);
  } else {
    static const unsigned cap_n = resident_blocks((const void*)k_v2_hist0p<false, false>);
    hipLaunchKernelGGL((k_v2_hist0p<false, false>), dim3(std::min<unsigned>(ntiles, cap_n)),
                       dim3(BLOCK), 0, s, seq, L, k, Nw, g, D, hist, ntiles, scan_status,
                       n_status, meta, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr);
  }
}
// Beyond 64 tiles of 2048 entries: the 32-per-thread look-back scan at any length.  Measured
// (A/B in one run, `profiles/rd3n_ab_scan_*`): config 3's 15 M-entry histograms 89 -> 60 us per
// scan (three launches of reduce-then-scan before), config 2's 0.5 M 7.7 -> 7.0 us.
void launch_scan_u32(uint32_t* a, uint64_t n, uint64_t* status, uint32_t* total, hipStream_t s) {
  const uint32_t nt = grid_of(n, TILE);
  // entries per thread by length (round 5, `profiles/r5n_scan_width_build_only.txt`): config 2's
  // 0.5 M entries 16 per thread (7.3 -> 6.1 us per scan against 32), config 3's 15 M 64 per
  // thread (59 -> 51 us): a short array wants more workgroups, a long one a shorter look-back
  if (nt > 64) {
    if (n < (1ull << 21)) {
      const uint32_t t16 = grid_of(n, BLOCK * 16);
      hipLaunchKernelGGL(k_scan_lb_u32<16>, dim3(t16), dim3(BLOCK), 0, s, a, n, status, t16, total);
    } else if (n < (1ull << 23)) {
      const uint32_t t32 = grid_of(n, BLOCK * 32);
      hipLaunchKernelGGL(k_scan_lb_u32<32>, dim3(t32), dim3(BLOCK), 0, s, a, n, status, t32, total);
    } else {
      const uint32_t t64 = grid_of(n, BLOCK * 64);
      hipLaunchKernelGGL(k_scan_lb_u32<64>, dim3(t64), dim3(BLOCK), 0, s, a, n, status, t64, total);
    }
  } else {
    hipLaunchKernelGGL(k_scan_lb_u32<WPT>, dim3(nt), dim3(BLOCK), 0, s, a, n, status, nt, total);
  }
}
void launch_v2_hist_bid(const uint32_t* bids, const uint32_t* n_ptr, Geom g, Digit D,
                        uint32_t* hist, uint32_t ntiles, uint64_t* scan_status, uint32_t n_status,
                        hipStream_t s, uint32_t* save_col0) {
  static const unsigned cap = resident_blocks((const void*)k_v2_histp<1>);
  hipLaunchKernelGGL(k_v2_histp<1>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0, s,
                     reinterpret_cast<const uint64_t*>(bids), n_ptr, g, D, hist, ntiles,
                     scan_status, n_status, save_col0, 0);
}
void launch_v2_hist_digits(const void* digits, bool u8, const uint32_t* n_ptr, Geom g, Digit D,
                           uint32_t* hist, uint32_t ntiles, uint64_t* scan_status,
                           uint32_t n_status, hipStream_t s, uint32_t* save_col0) {
  if (u8) {
    static const unsigned cap = resident_blocks((const void*)k_v2_histp<5>);
    hipLaunchKernelGGL(k_v2_histp<5>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0, s,
                       reinterpret_cast<const uint64_t*>(digits), n_ptr, g, D, hist, ntiles,
                       scan_status, n_status, save_col0, 0);
    return;
  }
  static const unsigned cap = resident_blocks((const void*)k_v2_histp<4>);
  hipLaunchKernelGGL(k_v2_histp<4>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0, s,
                     reinterpret_cast<const uint64_t*>(digits), n_ptr, g, D, hist, ntiles,
                     scan_status, n_status, save_col0, 0);
}
void launch_v2_hist(const uint64_t* keys, const uint32_t* n_ptr, Geom g, Digit D, uint32_t* hist,
                    uint32_t ntiles, uint64_t* scan_status, uint32_t n_status, hipStream_t s,
                    uint32_t* hll_rows, uint32_t* hll_regs, uint32_t* save_col0, bool skip_empty,
                    bool padded, bool aos, int sh8) {
  if (sh8) {                   // packed 8-B (key << sh | window) stream
    static const unsigned cap = resident_blocks((const void*)k_v2_histp<3>);
    hipLaunchKernelGGL(k_v2_histp<3>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0,
                       s, keys, n_ptr, g, D, hist, ntiles, scan_status, n_status, save_col0, sh8);
    return;
  }
  if (aos) {                   // packed (key, pos) stream (padded by construction)
    static const unsigned cap = resident_blocks((const void*)k_v2_histp<2>);
    hipLaunchKernelGGL(k_v2_histp<2>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0,
                       s, keys, n_ptr, g, D, hist, ntiles, scan_status, n_status, save_col0, 0);
    return;
  }
  if (padded && !hll_rows && !skip_empty) {
    static const unsigned cap = resident_blocks((const void*)k_v2_histp<0>);
    hipLaunchKernelGGL(k_v2_histp<0>, dim3(std::min<unsigned>(ntiles, cap)), dim3(BLOCK), 0,
                       s, keys, n_ptr, g, D, hist, ntiles, scan_status, n_status, save_col0, 0);
    return;
  }
  if (hll_rows)
    hipLaunchKernelGGL(k_v2_hist<true>, dim3(ntiles), dim3(BLOCK), 0, s, keys, n_ptr, g, D, hist,
                       ntiles, scan_status, n_status, hll_rows, hll_regs, save_col0,
                       skip_empty ? 1 : 0);
  else
    hipLaunchKernelGGL(k_v2_hist<false>, dim3(ntiles), dim3(BLOCK), 0, s, keys, n_ptr, g, D, hist,
                       ntiles, scan_status, n_status, nullptr, nullptr, save_col0,
                       skip_empty ? 1 : 0);
}
void launch_v2_bounds_lo(const uint64_t* kprev, const uint32_t* n_ptr, Geom g, Digit Dlast,
                         uint32_t div, const uint32_t* hist, uint32_t C, const uint32_t* lo_start,
                         uint32_t spread, uint32_t* start, uint32_t nlim, hipStream_t s,
                         const uint32_t* bprev, bool aos, int sh8) {
  hipLaunchKernelGGL(k_v2_bounds_lo, dim3(div), dim3(BLOCK), 0, s,
                     bprev ? reinterpret_cast<const uint64_t*>(bprev) : kprev, n_ptr, g, Dlast,
                     div, hist, C, lo_start, spread, start, bprev ? 1 : sh8 ? 3 : aos ? 2 : 0,
                     nlim, sh8);
}
void launch_seg_bounds(const uint32_t* hist, uint32_t ntiles, uint32_t R, uint32_t nseg,
                       uint32_t tps, const uint32_t* n_valid, uint32_t* segb, hipStream_t s) {
  hipLaunchKernelGGL(k_seg_bounds, dim3(grid_of((uint64_t)R * (nseg + 1), BLOCK)), dim3(BLOCK),
                     0, s, hist, ntiles, R, nseg, tps, n_valid, segb);
}
void launch_v2_hll(const uint32_t* hll_rows, uint32_t n_rows, uint32_t* hll_regs, double* host_est,
                   const uint32_t* n_valid, uint64_t* host_n, hipStream_t s) {
  const uint32_t g = std::max(1u, std::min(HLL_PART_ROWS, (n_rows + 127) / 128));
  hipLaunchKernelGGL(k_v2_hll_part, dim3(g), dim3(HLL_T), 0, s, hll_rows, n_rows, hll_regs);
  hipLaunchKernelGGL(k_v2_hll_final, dim3(1), dim3(HLL_T), 0, s, hll_regs, g, host_est, n_valid,
                     host_n);
}
static const BoundsFuse kNoFuse{nullptr, nullptr, nullptr, Digit{}, 0u, 1u, 0, 0u};
static const Pack8 kNoPack{0, nullptr, 0u, Digit{}};
void launch_v2_scatter_seq(const uint8_t* seq, int64_t L, int k, int64_t Nw, Geom g, Digit D,
                           const uint32_t* hist, uint32_t ntiles, uint64_t* kout, uint32_t* pout,
                           uint32_t pad, hipStream_t s, bool aos, const Pack8* pk,
                           const DigitOut* ds) {
  const DigitOut dso = ds ? *ds : kNoDigits;
  if (pk && pk->sh)
    KMHG_SCATTER_BMD(true, false, false, 6, dso, seq, L, k, Nw, nullptr, nullptr, nullptr, g, D,
                     hist, ntiles, kout, nullptr, pad, 0, kNoFuse, *pk);
  else if (aos)
    KMHG_SCATTER_BMD(true, false, false, 3, dso, seq, L, k, Nw, nullptr, nullptr, nullptr, g, D,
                     hist, ntiles, kout, nullptr, pad, 0, kNoFuse, kNoPack);
  else
    KMHG_SCATTER_BMD(true, false, false, 0, dso, seq, L, k, Nw, nullptr, nullptr, nullptr, g, D,
                     hist, ntiles, kout, pout, pad, 0, kNoFuse, kNoPack);
}
void launch_part_dense(const uint64_t* ck, const uint32_t* cp, const uint32_t* off,
                       uint32_t ntiles, const uint32_t* n_total, uint64_t* dk, uint32_t* dp,
                       hipStream_t s, bool aos) {
  if (aos)
    hipLaunchKernelGGL(k_part_dense<true>, dim3(std::min<uint32_t>(ntiles, 8192u)), dim3(BLOCK), 0,
                       s, ck, cp, off, ntiles, n_total, dk, dp);
  else
    hipLaunchKernelGGL(k_part_dense<false>, dim3(std::min<uint32_t>(ntiles, 8192u)), dim3(BLOCK), 0,
                       s, ck, cp, off, ntiles, n_total, dk, dp);
}
void launch_v2_scatter_bid0(const uint32_t* bids, int64_t Nw, Geom g, Digit D,
                            const uint32_t* hist, uint32_t ntiles, uint32_t* bout, uint32_t* pout,
                            uint32_t pad, hipStream_t s, const DigitOut* ds) {
  const uint64_t* ki = reinterpret_cast<const uint64_t*>(bids);
  uint64_t* ko = reinterpret_cast<uint64_t*>(bout);
  const DigitOut dso = ds ? *ds : kNoDigits;
  if (bout)
    KMHG_SCATTER_BMD(false, true, false, 1, dso, nullptr, (int64_t)0, 0, Nw, ki, nullptr, nullptr,
                     g, D, hist, ntiles, ko, pout, pad, 0, kNoFuse, kNoPack);
  else
    KMHG_SCATTER_BM(false, true, false, 2, nullptr, (int64_t)0, 0, Nw, ki, nullptr, nullptr, g,
                    D, hist, ntiles, ko, pout, pad, 0, kNoFuse, kNoPack);
}
void launch_v2_scatter_bid(const uint32_t* bin, const uint32_t* pin, const uint32_t* n_ptr,
                           Geom g, Digit D, const uint32_t* hist, uint32_t ntiles, uint32_t* bout,
                           uint32_t* pout, uint32_t pad, hipStream_t s, const BoundsFuse* bf,
                           const DigitOut* ds) {
  const uint64_t* ki = reinterpret_cast<const uint64_t*>(bin);
  uint64_t* ko = reinterpret_cast<uint64_t*>(bout);
  const BoundsFuse f = bf ? *bf : kNoFuse;
  const DigitOut dso = ds ? *ds : kNoDigits;
  if (bout)
    KMHG_SCATTER_BMD(false, false, false, 1, dso, nullptr, (int64_t)0, 0, (int64_t)0, ki, pin,
                     n_ptr, g, D, hist, ntiles, ko, pout, pad, 0, f, kNoPack);
  else
    KMHG_SCATTER_BM(false, false, false, 2, nullptr, (int64_t)0, 0, (int64_t)0, ki, pin, n_ptr,
                    g, D, hist, ntiles, ko, pout, pad, 0, f, kNoPack);
}
void launch_v2_scatter(const uint64_t* kin, const uint32_t* pin, const uint32_t* n_ptr, Geom g,
                       Digit D, const uint32_t* hist, uint32_t ntiles, uint64_t* kout,
                       uint32_t* pout, uint32_t pad, hipStream_t s, const BoundsFuse* bf,
                       bool aos, bool aos_in, const Pack8* pk, const DigitOut* ds) {
  const DigitOut dso = ds ? *ds : kNoDigits;
  if (pk && pk->sh)            // packed 8-B elements in, packed 12-B out (a last pass)
    KMHG_SCATTER_BM(false, false, false, 7, nullptr, (int64_t)0, 0, (int64_t)0, kin, nullptr,
                    n_ptr, g, D, hist, ntiles, kout, nullptr, pad, 0, bf ? *bf : kNoFuse, *pk);
  else if (aos && aos_in)
    KMHG_SCATTER_BMD(false, false, false, 3, dso, nullptr, (int64_t)0, 0, (int64_t)0, kin,
                     nullptr, n_ptr, g, D, hist, ntiles, kout, nullptr, pad, 0,
                     bf ? *bf : kNoFuse, kNoPack);
  else if (aos)
    KMHG_SCATTER_BMD(false, false, false, 4, dso, nullptr, (int64_t)0, 0, (int64_t)0, kin, pin,
                     n_ptr, g, D, hist, ntiles, kout, nullptr, pad, 0, bf ? *bf : kNoFuse,
                     kNoPack);
  else
    KMHG_SCATTER_BMD(false, false, false, 0, dso, nullptr, (int64_t)0, 0, (int64_t)0, kin, pin,
                     n_ptr, g, D, hist, ntiles, kout, pout, pad, 0, bf ? *bf : kNoFuse, kNoPack);
}
void launch_v2_scatter_keys0(const uint64_t* kin, uint64_t n_keys, const uint32_t* n_ptr, Geom g,
                             Digit D, const uint32_t* hist, uint32_t ntiles, uint64_t* kout,
                             uint32_t* pout, uint32_t pad, bool nopos, bool skip_empty,
                             hipStream_t s) {
  if (nopos)
    KMHG_SCATTER(false, true, true, nullptr, (int64_t)0, 0, (int64_t)n_keys, kin, nullptr, n_ptr,
                 g, D, hist, ntiles, kout, nullptr, pad, skip_empty ? 1 : 0, kNoFuse, kNoPack);
  else
    KMHG_SCATTER(false, true, false, nullptr, (int64_t)0, 0, (int64_t)n_keys, kin, nullptr,
                 n_ptr, g, D, hist, ntiles, kout, pout, pad, skip_empty ? 1 : 0, kNoFuse, kNoPack);
}
void launch_v2_scatter_nopos(const uint64_t* kin, const uint32_t* n_ptr, Geom g, Digit D,
                             const uint32_t* hist, uint32_t ntiles, uint64_t* kout, uint32_t pad,
                             hipStream_t s, const BoundsFuse* bf) {
  KMHG_SCATTER(false, false, true, nullptr, (int64_t)0, 0, (int64_t)0, kin, nullptr, n_ptr, g, D,
               hist, ntiles, kout, nullptr, pad, 0, bf ? *bf : kNoFuse, kNoPack);
}
void launch_v2_bucket_wg(const uint64_t* keys, const uint32_t* pos, const uint32_t* start, Geom g,
                         Slot* T, int32_t* positions, BucketStats* bstats, BuildMeta* meta,
                         bool count_only, hipStream_t s, const uint32_t* n_ptr, uint32_t nw,
                         const uint32_t* code, int k, bool aos, uint8_t* TG, uint32_t* rep) {
  const bool ballot = ballot_ranks();
  const bool tags = TG != nullptr && !count_only && !code;
  const dim3 gr(g.nb), bl(BLOCK);
#define KMHG_BUCKET(CO, CKK, BAL, AO, TG_)                                                     \
  hipLaunchKernelGGL((k_v2_bucket_wg<CO, CKK, BAL, AO, TG_>), gr, bl, 0, s, keys, pos, start, g, \
                     T, positions, bstats, meta, CKK ? code : nullptr, CKK ? k : 0, n_ptr, nw,   \
                     TG, rep)
  if (aos && tags)
    { if (ballot) KMHG_BUCKET(false, false, true, true, true); else KMHG_BUCKET(false, false, false, true, true); }
  else if (aos)
    { if (ballot) KMHG_BUCKET(false, false, true, true, false); else KMHG_BUCKET(false, false, false, true, false); }
  else if (count_only)              // no positions: nothing is ranked
    KMHG_BUCKET(true, false, false, false, false);
  else if (code)
    { if (ballot) KMHG_BUCKET(false, true, true, false, false); else KMHG_BUCKET(false, true, false, false, false); }
  else if (tags)
    { if (ballot) KMHG_BUCKET(false, false, true, false, true); else KMHG_BUCKET(false, false, false, false, true); }
  else
    { if (ballot) KMHG_BUCKET(false, false, true, false, false); else KMHG_BUCKET(false, false, false, false, false); }
#undef KMHG_BUCKET
}
// The hardware property the radix passes' ranks rest on, checked on the device itself
// (tools/lds_order.hip is the stand-alone probe): the lanes of one returning LDS add that hit
// the same address get old values in increasing lane order.  Every wave draws skewed random
// digits, adds, and compares each lane with every lower lane of the same digit.
__global__ void __launch_bounds__(BLOCK)
k_lane_order_check(unsigned long long* __restrict__ res, uint32_t seed, int iters) {
  __shared__ uint32_t cnt[BLOCK / 64][128];
  __shared__ uint32_t got[BLOCK / 64][64], dig[BLOCK / 64][64];
  const int w = threadIdx.x >> 6, lane = lane_id();
  uint32_t r = (seed ^ (blockIdx.x * BLOCK + threadIdx.x) * 2654435761u) | 1u;
  unsigned long long bad = 0, chk = 0;
  for (int it = 0; it < iters; ++it) {
    for (int d = lane; d < 128; d += 64) cnt[w][d] = 0;
    wave_sync();
    r ^= r << 13; r ^= r >> 17; r ^= r << 5;
    const uint32_t d = (r & 1) ? (r >> 8) % 4 : (r >> 8) % 99;
    const bool act = ((r >> 20) & 7) != 0;
    const uint32_t v = act ? atomicAdd(&cnt[w][d], 1u) : 0u;
    got[w][lane] = act ? v : 0xFFFFFFFFu;
    dig[w][lane] = d;
    wave_sync();
    if (act)
      for (int m = 0; m < lane; ++m)
        if (got[w][m] != 0xFFFFFFFFu && dig[w][m] == d) {
          ++chk;
          bad += got[w][m] > v ? 1u : 0u;
        }
    wave_sync();
  }
  atomicAdd(&res[0], bad);
  atomicAdd(&res[1], chk);
}
void launch_lane_order_check(unsigned long long* res, hipStream_t s, int blocks) {
  hipLaunchKernelGGL(k_lane_order_check, dim3(blocks), dim3(BLOCK), 0, s, res, 12345u, 64);
}

// Test knob (KMHG_TEST_DISORDER=<mode>, tests only), each of which the bucket kernel must report
// (the build then falls back) instead of faulting: 1 swaps the first two positions of bucket 0's
// stream; 2 zeroes its first position (an entry no pass wrote: the pad's value); 3 moves bucket
// 1's start past the end of the stream.
// (pos: the stream's positions, every `stride`-th word)
__global__ void k_v2_test_disorder(uint32_t* __restrict__ pos, uint32_t* __restrict__ start,
                                   const uint32_t* __restrict__ n_ptr, int mode, uint32_t stride) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const uint64_t a = start[0], b = start[1];
    if (mode == 1 && b - a >= 2) {
      const uint32_t t = pos[a * stride];
      pos[a * stride] = pos[(a + 1) * stride];
      pos[(a + 1) * stride] = t;
    } else if (mode == 2 && b > a) {
      pos[a * stride] = 0u;
    } else if (mode == 3) {
      start[1] = *n_ptr + 4096u;
    }
  }
}
void launch_v2_test_disorder(uint32_t* pos, uint32_t* start, const uint32_t* n_ptr, int mode,
                             hipStream_t s, uint32_t stride) {
  hipLaunchKernelGGL(k_v2_test_disorder, dim3(1), dim3(64), 0, s, pos, start, n_ptr, mode, stride);
}
void launch_v2_stats(const BucketStats* bstats, uint32_t nb, const uint32_t* n_valid,
                     BuildMeta* meta, BuildMeta* host_meta, hipStream_t s) {
  // one bucket per thread up to 64 workgroups (config 2: 40), then STATS_PER per trip
  // (measured: 5 workgroups of 8 buckets per thread 6.1 us at config 2, 40 of one 4.8; 256
  // workgroups at config 3 16 us against 9 -- their device atomics and arrival tickets)
  unsigned gr = grid_of(nb, BLOCK);
  if (gr > 64) gr = 64;
  hipLaunchKernelGGL(k_v2_stats, dim3(gr), dim3(BLOCK), 0, s, bstats, nb, n_valid, meta, host_meta);
}

}  // namespace kmhg
