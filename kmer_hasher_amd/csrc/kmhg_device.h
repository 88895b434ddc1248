// kmhg_device.h -- device helpers shared by the kernel translation units (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include "kmhg_common.h"

namespace kmhg {

// ------------------------------------------------------------------ small wave/block helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// DPP move of a u64 (both halves by the same lane pattern); lanes without a source, or in a row
// the row mask leaves out, read 0
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, ROWS, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, ROWS, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive wave scan (64 lanes, every lane active): row shifts by 1, 2, 4, 8 inside each
// 16-lane row, then row broadcasts of lanes 15 and 31 -- VALU moves, where a __shfl_up chain is
// six dependent LDS permutes (ds_bpermute) per 32-bit half.
#ifndef KMHG_SHFL_SCAN
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
  v += dpp_u64<0x111, 0xf>(v);             // row_shr:1
  v += dpp_u64<0x112, 0xf>(v);             // row_shr:2
  v += dpp_u64<0x114, 0xf>(v);             // row_shr:4
  v += dpp_u64<0x118, 0xf>(v);             // row_shr:8
  v += dpp_u64<0x142, 0xa>(v);             // row_bcast:15 into rows 1 and 3
  v += dpp_u64<0x143, 0xc>(v);             // row_bcast:31 into rows 2 and 3
  return v;
}
#else
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t t = __shfl_up(v, d);
    if (lane_id() >= d) v += t;
  }
  return v;
}
#endif

// inclusive wave max-scan of u32 values (identity 0), the DPP pattern of wave_incl_scan
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));
  return v;
}

// lane 63's value in every lane (a scalar read, not an LDS permute)
__device__ __forceinline__ uint64_t lane63(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}
// the sum over the wave's 64 lanes, in every lane
__device__ __forceinline__ uint64_t wave_sum(uint64_t v) { return lane63(wave_incl_scan(v)); }

// Inclusive wave scan of u32 values by DPP row shifts and row broadcasts: six VALU adds, no LDS
// permute (a __shfl_up is a ds_bpermute, an LDS round trip per step).  All 64 lanes must call it.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
  return v;
}

// XCD-contiguous work mapping: a bijection of [0, n) that gives the blocks of one XCD (blocks
// are dealt round-robin, b and b + 8 share an XCD -- MI355X_MICROARCH.md "Workgroup dispatch")
// one contiguous range of work items.  Neighbouring tiles then write the partial cache lines at
// their shared output boundaries through the SAME L2, which merges them before write-back,
// instead of two XCDs each writing back a partial line.  Speed only: any placement is correct.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n >> 3, r = n & 7u, x = b & 7u, j = b >> 3;
  return x * q + (x < r ? x : r) + j;
}

// Exclusive scan over the 256 threads of a block (one value per thread).  `lds` needs 5 u64.
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* lds, uint64_t& total) {
  const int wid = threadIdx.x >> 6;
  uint64_t inc = wave_incl_scan(v);
  if (lane_id() == 63) lds[wid] = inc;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BLOCK / 64; ++w) {
    uint64_t x = lds[w];
    if (w < wid) off += x;
    tot += x;
  }
  __syncthreads();
  total = tot;
  return off + inc - v;
}

// Ranks of the flagged elements of a tile of J x BLOCK elements, element e = j * BLOCK + t
// (lane-contiguous), in element order, from `base` on: per-(j, wave) ballots and one wave scan,
// no look-back (the caller knows the tile's first rank).  `cw` = LDS for J * (BLOCK / 64) + 1
// u64 (J * BLOCK / 64 < 64).  Returns the tile's flag count.
template <int J>
__device__ __forceinline__ uint32_t tile_rank_at(const bool (&flag)[J], uint64_t (&rk)[J],
                                                 uint64_t* cw, uint64_t base) {
  const int wave = threadIdx.x >> 6, lane = lane_id();
  constexpr int NW = BLOCK / 64;
  uint64_t m[J];
#pragma unroll
  for (int j = 0; j < J; ++j) m[j] = __ballot(flag[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < J; ++j) cw[j * NW + wave] = (uint64_t)__popcll(m[j]);
  }
  __syncthreads();
  if (wave == 0) {                       // lanes 0 .. J*NW-1 own one (j, wave) count each
    const uint64_t c = lane < J * NW ? cw[lane] : 0;
    const uint64_t inc = wave_incl_scan(c);
    if (lane < J * NW) cw[lane] = base + inc - c;
    if (lane == 63) cw[J * NW] = inc;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j)
    rk[j] = cw[j * NW + wave] + (uint64_t)__popcll(m[j] & lanemask_lt());
  return (uint32_t)cw[J * NW];
}

// ------------------------------------------------------------------ decoupled look-back
// status word: [63:62] = 0 not ready / 1 aggregate / 2 inclusive prefix, [61:0] payload.
// Each word is a self-describing 8-B granule written by ONE relaxed agent-scope store and read
// by relaxed agent-scope loads (sc1), so no separate flag, fence or payload hand-off exists.
// Tiles come from a ticket counter so every tile a block waits on is already running.
constexpr uint64_t LB_MASK = (1ull << 62) - 1;

// Wave-parallel look-back: called by ALL 64 lanes of one wave (same tile/agg in every lane).
// Each round the 64 lanes read the 64 nearest predecessors at once; the window is consumed up
// to (and including) the nearest inclusive prefix once every word in front of it is ready.
// With `prepublished`, the caller already stored the aggregate (lookback_publish) earlier, so
// successors could start summing it while this wave did other work.
__device__ inline void lookback_publish(uint64_t* status, uint32_t tile, uint64_t agg) {
  if (lane_id() == 0) st_relaxed(&status[tile], ((tile == 0 ? 2ull : 1ull) << 62) | agg);
}

__device__ inline uint64_t lookback_excl(uint64_t* status, uint32_t tile, uint64_t agg,
                                         bool prepublished = false) {
  const int lane = lane_id();
  if (tile == 0) {
    if (lane == 0 && !prepublished) st_relaxed(&status[0], (2ull << 62) | agg);
    return 0;
  }
  if (lane == 0 && !prepublished) st_relaxed(&status[tile], (1ull << 62) | agg);
  uint64_t excl = 0;
  int64_t base = (int64_t)tile - 1;
  for (;;) {
    int64_t j = base - lane;
    uint64_t w = (j >= 0) ? ld_relaxed(&status[j]) : (2ull << 62);   // before tile 0: prefix 0
    uint64_t f = w >> 62;
    uint64_t m0 = __ballot(f == 0), m2 = __ballot(f == 2);
    int first2 = m2 ? __ffsll((unsigned long long)m2) - 1 : 64;
    uint64_t need = first2 == 64 ? ~0ull : ((2ull << first2) - 1ull);   // lanes 0..first2
    if (m0 & need) { __builtin_amdgcn_s_sleep(1); continue; }
    excl += wave_sum((lane <= first2) ? (w & LB_MASK) : 0ull);
    if (first2 < 64) break;
    base -= 64;
  }
  if (lane == 0) st_relaxed(&status[tile], (2ull << 62) | (excl + agg));
  return excl;
}

// Grab a tile ticket (thread 0) and broadcast it.
__device__ __forceinline__ uint32_t take_ticket(uint32_t* counter, uint32_t* lds) {
  if (threadIdx.x == 0) *lds = atomicAdd(counter, 1u);
  __syncthreads();
  uint32_t t = *lds;
  __syncthreads();
  return t;
}

// ------------------------------------------------------------------ LDS staging of a tile
// Chars [base, base + STAGE) are loaded coalesced (16 B per lane when the sequence is 16-B
// aligned) and packed into 2-bit codes (MSB-first, 16 chars per u32) and N flags (16 chars per
// u16 kept in a u32).  Chars outside [0, L) are flagged N: a window that touches them is never
// valid, and position -1 acting as N gives the reference's "start of sequence" rule.
template <int W16>
struct StageN {
  static constexpr int kWords = W16;
  uint32_t code[W16];
  uint32_t nbit[W16];
};
using Stage = StageN<STAGE_W16>;             // one TILE of windows
using PStage = StageN<PSTAGE_W16>;           // one partition tile (PTILE windows)

__device__ __forceinline__ void pack16(const uint8_t* c, uint32_t& code, uint32_t& nb) {
  uint32_t cd = 0, n = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t ch = c[i];
    cd = (cd << 2) | ((ch >> 1) & 3u);       // UPDATE_OFFSET, src/kmer_util.h:8
    n = (n << 1) | (((ch | 0x20u) == 'n') ? 1u : 0u);   // LC(c)=='n', src/kmer_util.h:10
  }
  code = cd; nb = n;
}

__device__ __forceinline__ void pack16v(uint4 v, uint32_t& code, uint32_t& nb) {
  const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
  uint32_t cd = 0, n = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t ch = (wv[i >> 2] >> (8 * (i & 3))) & 0xFFu;
    cd = (cd << 2) | ((ch >> 1) & 3u);       // UPDATE_OFFSET, src/kmer_util.h:8
    n = (n << 1) | (((ch | 0x20u) == 'n') ? 1u : 0u);   // LC(c)=='n', src/kmer_util.h:10
  }
  code = cd; nb = n;
}

// One 16-char word of the stage (word w starts at char base + 16 w), loaded coalesced when the
// sequence is 16-B aligned; chars outside [0, L) read as 'N'.
__device__ __forceinline__ uint4 stage_word(const uint8_t* __restrict__ seq, int64_t L,
                                            int64_t base, int w, bool aligned) {
  const int64_t c0 = base + 16 * (int64_t)w;
  if (aligned) {
    // exactly ONE 16-B load on every path (a static vector-memory count lets the compiler wait
    // for it with a counted vmcnt in pipelined loops).  c0 % 16 == 0 and the chunk never leaves
    // the 16-B aligned block of a valid byte, so it cannot touch an unmapped page; chunks wholly
    // outside [0, L) load chunk 0 instead and read as 'N'.
    const bool any = c0 + 16 > 0 && c0 < L;
    uint4 v = *reinterpret_cast<const uint4*>(seq + (any ? c0 : 0));
    if (!any) return make_uint4(0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu, 0x4E4E4E4Eu);
    if (c0 < 0 || c0 + 16 > L) {
      uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int64_t p = c0 + i;
        if (p < 0 || p >= L) x[i >> 2] = (x[i >> 2] & ~(0xFFu << (8 * (i & 3)))) | (0x4Eu << (8 * (i & 3)));
      }
      v = make_uint4(x[0], x[1], x[2], x[3]);
    }
    return v;
  }
  uint32_t x[4] = {0u, 0u, 0u, 0u};          // register-only byte assembly (no private array)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t p = c0 + i;
    const uint32_t ch = (p >= 0 && p < L) ? (uint32_t)seq[p] : (uint32_t)'N';
    x[i >> 2] |= ch << (8 * (i & 3));
  }
  return make_uint4(x[0], x[1], x[2], x[3]);
}

// Split form for software pipelining: stage_load fetches this thread's 16-char words of the
// stage (word threadIdx.x + j * BLOCK) into registers; stage_pack encodes them into LDS later.
template <int W16>
struct StageRegs {
  static constexpr int kPer = (W16 + BLOCK - 1) / BLOCK;
  uint4 v[kPer];
};
// ALWAYS_ALIGNED: the caller guarantees a 16-B aligned sequence (the partitioned build copies
// an unaligned input first), so the byte-wise path is not even compiled in.
template <int W16, bool ALWAYS_ALIGNED = false>
__device__ __forceinline__ void stage_load(StageRegs<W16>& r, const uint8_t* __restrict__ seq,
                                           int64_t L, int64_t base, bool aligned) {
#pragma unroll
  for (int j = 0; j < StageRegs<W16>::kPer; ++j) {   // clamped word: one load on every path
    const int w = min((int)threadIdx.x + j * BLOCK, W16 - 1);
    r.v[j] = stage_word(seq, L, base, w, ALWAYS_ALIGNED || aligned);
  }
}
template <int W16>
__device__ __forceinline__ void stage_pack(const StageRegs<W16>& r, StageN<W16>& st) {
#pragma unroll
  for (int j = 0; j < StageRegs<W16>::kPer; ++j) {
    const int w = threadIdx.x + j * BLOCK;
    if (w < W16) {
      uint32_t cd, nb;
      pack16v(r.v[j], cd, nb);
      st.code[w] = cd;
      st.nbit[w] = nb;
    }
  }
}

template <bool ALWAYS_ALIGNED = false, int W16>
__device__ __forceinline__ void stage_tile(const uint8_t* __restrict__ seq, int64_t L,
                                           int64_t base, StageN<W16>& st, bool aligned) {
  StageRegs<W16> r;
  stage_load<W16, ALWAYS_ALIGNED>(r, seq, L, base, aligned);
  stage_pack(r, st);
}

// Window whose first char is stage offset o (global start s).  Returns validity per the
// reference walk: no N in [s, s+k), s+k <= L, and NOT (s+k == L and the char
// before s is N or s == 0) -- the end-drop quirk of init_kmer (src/kmer_pos.c:81-83).
template <class ST>
__device__ __forceinline__ bool window_key(const ST& st, int o, int64_t s, int64_t L, int k,
                                           uint64_t& key) {
  if (s + k > L) return false;
  // N flags of chars [o-1, o+k): k+1 <= 33 bits out of a 48-bit window of three u16 words
  int p = o - 1;
  int q = p >> 4, c = p & 15;
  uint64_t x48 = ((uint64_t)st.nbit[q] << 32) | ((uint64_t)st.nbit[q + 1] << 16) |
                 (uint64_t)st.nbit[q + 2];
  uint64_t m = (x48 << (16 + c)) >> (63 - k);          // top k+1 bits
  uint64_t winN = m & ((2ull << (k - 1)) - 1ull);      // low k bits (k <= 32)
  if (winN) return false;
  if (s + k == L && ((m >> k) & 1ull)) return false;
  // 2k code bits of chars [o, o+k)
  int qw = o >> 4, b = (o & 15) * 2;
  uint64_t x = ((uint64_t)st.code[qw] << 32) | st.code[qw + 1];
  uint64_t y = st.code[qw + 2];
  uint64_t t = (x << b) | ((y << b) >> 32);
  key = t >> (64 - 2 * k);
  return true;
}

// Eight consecutive windows at stage offsets o0 .. o0 + 7 (global starts s0 .. s0 + 7), the same
// rule as window_key, from 4 code words and 4 N-flag words read once: 8 LDS reads for 8 windows
// instead of 48.  o0 >= 1 (the stage has HALO chars in front); chars [o0 - 1, o0 + 7 + k) lie
// in the 64 chars from 16 * ((o0 - 1) / 16) for any o0 % 16 and k <= 32.  key(j) and
// valid(j) take static j; only the six words stay live across the windows.
struct Win8 {
  uint64_t hi, lo, nx;                       // code bits of chars 16 q .., N flags of 16 qn ..
  int b, c0, k;
  int64_t s0, L;
  template <class ST>
  __device__ __forceinline__ Win8(const ST& st, int o0, int64_t s0_, int64_t L_, int k_)
      : k(k_), s0(s0_), L(L_) {
    // (words past the stage's end are clamped: the windows of the stage never reach them)
    constexpr int W = ST::kWords - 1;
    const int q = o0 >> 4, qn = (o0 - 1) >> 4;
    b = o0 & 15;
    c0 = (o0 - 1) & 15;
    hi = ((uint64_t)st.code[q] << 32) | st.code[q + 1];
    lo = ((uint64_t)st.code[min(q + 2, W)] << 32) | st.code[min(q + 3, W)];
    nx = ((uint64_t)st.nbit[qn] << 48) | ((uint64_t)st.nbit[qn + 1] << 32) |
         ((uint64_t)st.nbit[min(qn + 2, W)] << 16) | (uint64_t)st.nbit[min(qn + 3, W)];
  }
  __device__ __forceinline__ uint64_t key(int j) const {
    const int sh = 2 * (b + j);              // <= 44: the window's chars start here
    const uint64_t top = sh ? (hi << sh) | (lo >> (64 - sh)) : hi;
    return top >> (64 - 2 * k);
  }
  __device__ __forceinline__ bool valid(int j) const {
    const int64_t s = s0 + j;
    const uint64_t m = (nx << (c0 + j)) >> (63 - k);   // N flags of chars [o - 1, o + k)
    return s + k <= L && !(m & ((2ull << (k - 1)) - 1ull)) && !(s + k == L && ((m >> k) & 1ull));
  }
};

// The key of window j (0-based) from a sequence's global code words (the stage's format, 16
// chars per u32 MSB-first; a, b, c = words j / 16 .. j / 16 + 2): window_key's extraction.
__device__ __forceinline__ uint64_t code_key(uint32_t a, uint32_t b, uint32_t c, int64_t j, int k) {
  const int sh = (int)(j & 15) * 2;
  const uint64_t x = ((uint64_t)a << 32) | b;
  const uint64_t y = c;
  const uint64_t t = (x << sh) | ((y << sh) >> 32);
  return t >> (64 - 2 * k);
}

// ------------------------------------------------------------------ hash table primitives
// Table geometry: nb buckets of capb slots (+ one side slot at nb*capb).  A key's bucket is
// mulhi(h, nb) (high hash bits), its home inside the bucket mulhi32(lo32(h), capb), and linear
// probing wraps inside the bucket -- so a bucket is a self-contained sub-table that one wave
// can build in LDS (partitioned build) and a probe never leaves it.  nb = 1 is a plain
// linear-probing table (the global-atomic build).
__device__ __forceinline__ uint32_t bucket_of(uint64_t h, uint32_t nb) {
  return (uint32_t)__umul64hi(h, (uint64_t)nb);
}
// home slot from the top 16 bits of lo32(h): a non-decreasing function of the 16-bit sort key
// the sorted bucket build orders windows by (V_bucket_sort)
__device__ __forceinline__ uint32_t local_home(uint64_t h, uint32_t capb) {
  return (uint32_t)((((uint64_t)((uint32_t)h >> 16)) * capb) >> 16);
}
__device__ __forceinline__ uint64_t side_slot(Geom g) { return (uint64_t)g.nb * g.capb; }

// Find-or-insert (atomicCAS on the 64-bit key word).  Keys only move EMPTY -> key, so a stale
// plain read can only show EMPTY, which the CAS then corrects.
__device__ __forceinline__ uint32_t table_insert(Slot* __restrict__ T, Geom g, uint64_t key) {
  if (key == EMPTY_KEY) return (uint32_t)side_slot(g);   // side slot (k = 32, all G)
  const uint64_t h = mix64(key);
  const uint64_t b0 = (uint64_t)bucket_of(h, g.nb) * g.capb;
  uint32_t j = local_home(h, g.capb);
  for (;;) {
    const uint64_t i = b0 + j;
    uint64_t cur = T[i].key;
    if (cur == key) return (uint32_t)i;
    if (cur == EMPTY_KEY) {
      uint64_t prev = atomicCAS((unsigned long long*)&T[i].key, (unsigned long long)EMPTY_KEY,
                                (unsigned long long)key);
      if (prev == EMPTY_KEY || prev == key) return (uint32_t)i;
    }
    if (++j == g.capb) j = 0;
  }
}

// One 16-B slot as a probe reads it.  NT: a nontemporal load, for tables far beyond the
// Infinity Cache, whose random slot lines would otherwise evict what the probe reuses (the code
// words, the slot tags) for lines it reads once (launch_query_probe).
template <bool NT = false>
__device__ __forceinline__ uint4 ld_slot(const Slot* p) {
  if constexpr (NT) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}

// A part of an owner-computes build (Geom.nbh != 0) holds buckets [b0, b0 + nb) of a table of
// nbh buckets, indexed from 0: the part's own bucket of hash h, >= g.nb for another part's key.
__device__ __forceinline__ uint32_t part_bucket(uint64_t h, const Geom& g) {
  return bucket_of(h, g.nbh) - g.b0;
}
// whether this part owns `key` (the k = 32 sentinel key ~0 lives in the side slot of the part
// that owns its hash's bucket)
__device__ __forceinline__ bool part_owns(uint64_t key, const Geom& g) {
  return part_bucket(mix64(key), g) < g.nb;
}

// Read-only probe: returns the slot or NONE; count/aux from the same 16-B slot load.  PART: T is
// a part's table (the caller checked part_owns).
template <bool NT = false, bool PART = false>
__device__ __forceinline__ uint32_t table_find(const Slot* __restrict__ T, Geom g, uint64_t key,
                                               uint32_t& count, uint32_t& aux) {
  if (key == EMPTY_KEY) {
    const uint64_t i = side_slot(g);
    uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
    count = v.z; aux = v.w;
    return count ? (uint32_t)i : NONE;
  }
  const uint64_t h = mix64(key);
  const uint64_t b0 = (uint64_t)(PART ? part_bucket(h, g) : bucket_of(h, g.nb)) * g.capb;
  uint32_t j = local_home(h, g.capb);
  for (;;) {
    const uint64_t i = b0 + j;
    uint4 v = ld_slot<NT>(&T[i]);
    uint64_t cur = ((uint64_t)v.y << 32) | v.x;
    if (cur == key) { count = v.z; aux = v.w; return (uint32_t)i; }
    if (cur == EMPTY_KEY) { count = 0; aux = 0; return NONE; }
    if (++j == g.capb) j = 0;
  }
}

// The same probe reading FOUR consecutive slots per round trip (a miss walks its run of
// occupied slots to an empty one: at load 0.67 ~5 slots, one 64-B span instead of 5 dependent
// loads).  Used where misses dominate (the diagonal query path sends only anchors, unpredicted
// windows and misses here).
template <bool NT = false, bool PART = false>
__device__ __forceinline__ uint32_t table_find4(const Slot* __restrict__ T, Geom g, uint64_t key,
                                                uint32_t& count, uint32_t& aux) {
  if (key == EMPTY_KEY) return table_find<NT, PART>(T, g, key, count, aux);
  const uint64_t h = mix64(key);
  const uint64_t b0 = (uint64_t)(PART ? part_bucket(h, g) : bucket_of(h, g.nb)) * g.capb;
  uint32_t j = local_home(h, g.capb);
  for (;;) {
    uint4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t jq = j + q;
      if (jq >= g.capb) jq -= g.capb;
      v[q] = ld_slot<NT>(&T[b0 + jq]);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t cur = ((uint64_t)v[q].y << 32) | v[q].x;
      if (cur == key) {
        count = v[q].z; aux = v[q].w;
        uint32_t jq = j + q;
        if (jq >= g.capb) jq -= g.capb;
        return (uint32_t)(b0 + jq);
      }
      if (cur == EMPTY_KEY) { count = 0; aux = 0; return NONE; }
    }
    j += 4;
    if (j >= g.capb) j -= g.capb;
  }
}

// Slot tags, the diagonal query path's filter for windows that miss (built with the position
// slots, kmhg_kernels.hip k_pos_slots): one byte per table slot, 0 for an empty slot, else the
// low byte of the key's hash (the bucket takes the high word, the home bits 16..31), 0 -> 1.
__device__ __forceinline__ uint8_t slot_tag(uint64_t h) {
  const uint32_t t = (uint32_t)h & 0xFFu;
  return (uint8_t)(t ? t : 1u);
}
// bit q (q < 8) set iff byte q of v is 0, exact for the lowest zero byte (bits above it may be
// spurious); the caller keeps only bits below the first one
__device__ __forceinline__ uint32_t zero_bytes8(uint64_t v) {
  const uint64_t x = (v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull;
  return (uint32_t)(((x >> 7) * 0x0102040810204080ull) >> 56);
}

// table_find through the tags: a miss reads the 16 tags of its home's aligned group (one 16-B
// load from an array 1/16 the table's size) and usually stops at an empty tag without touching
// the table; the table is read only at slots whose tag equals the key's.  Needs g.capb % 16 == 0.
// PART: T and TG are a part's (the caller checked part_owns).
template <bool NT = false, bool PART = false>
__device__ __forceinline__ uint32_t table_find_tag(const Slot* __restrict__ T,
                                                   const uint8_t* __restrict__ TG, Geom g,
                                                   uint64_t key, uint32_t& count, uint32_t& aux) {
  count = 0; aux = 0;
  if (key == EMPTY_KEY) return table_find<NT, PART>(T, g, key, count, aux);
  const uint64_t h = mix64(key);
  const uint64_t b0 = (uint64_t)(PART ? part_bucket(h, g) : bucket_of(h, g.nb)) * g.capb;
  const uint32_t j = local_home(h, g.capb);
  const uint64_t tt = 0x0101010101010101ull * slot_tag(h);
  uint32_t grp = j & ~15u, off = j & 15u;
  for (uint32_t n = 0; n <= g.capb / 16; ++n) {
    const uint4 v = *reinterpret_cast<const uint4*>(TG + b0 + grp);
    uint64_t w0 = ((uint64_t)v.y << 32) | v.x, w1 = ((uint64_t)v.w << 32) | v.z;
    // bytes before the home read as 0xFF: no zero there, so no borrow into the bytes above
    const uint64_t lo0 = off >= 8 ? ~0ull : (off ? ((1ull << (8 * off)) - 1) : 0ull);
    const uint64_t lo1 = off > 8 ? ((1ull << (8 * (off - 8))) - 1) : 0ull;
    w0 |= lo0; w1 |= lo1;
    const uint32_t zm = zero_bytes8(w0) | (zero_bytes8(w1) << 8);
    const uint32_t below = zm ? (1u << (__ffs(zm) - 1)) - 1 : 0xFFFFu;
    uint32_t cand = (zero_bytes8(w0 ^ tt) | (zero_bytes8(w1 ^ tt) << 8)) & below & (0xFFFFu << off);
    while (cand) {                              // tag hits: the full key decides
      const uint32_t q = __ffs(cand) - 1;
      cand &= cand - 1;
      const uint64_t i = b0 + grp + q;
      const uint4 sv = ld_slot<NT>(&T[i]);
      if ((((uint64_t)sv.y << 32) | sv.x) == key) { count = sv.z; aux = sv.w; return (uint32_t)i; }
    }
    if (zm) return NONE;
    grp += 16;
    if (grp >= g.capb) grp = 0;
    off = 0;
  }
  return NONE;
}

// Wave-aggregated atomicAdd on a per-slot u32 counter.  Lanes that hold the same slot are
// grouped behind the first active lane (readfirstlane + ballot); one atomic per group.  The
// loop stops as soon as a group of one appears (i.i.d. data: one iteration), leaving the rest
// to plain per-lane atomics; periodic (tandem-repeat) waves collapse to one atomic per key.
// Returns the old value + this lane's rank inside its group (ranks follow lane order).
__device__ __forceinline__ uint32_t wave_agg_add(uint32_t* base_ptr_of_slot0, bool act,
                                                 uint32_t slot, size_t stride_u32) {
  uint64_t active = __ballot(act);
  uint32_t result = 0;
  bool done = false;
  while (active) {
    int leader = __ffsll((unsigned long long)active) - 1;
    uint32_t lslot = __shfl(slot, leader);
    uint64_t grp = __ballot(act && !done && slot == lslot) & active;
    int gsz = __popcll(grp);
    if (gsz == 1) break;
    uint32_t old = 0;
    if (lane_id() == leader)
      old = atomicAdd(base_ptr_of_slot0 + (size_t)lslot * stride_u32, (uint32_t)gsz);
    old = __shfl(old, leader);
    if ((grp >> lane_id()) & 1ull) {
      result = old + (uint32_t)__popcll(grp & lanemask_lt());
      done = true;
    }
    active &= ~grp;
  }
  if (act && !done) result = atomicAdd(base_ptr_of_slot0 + (size_t)slot * stride_u32, 1u);
  return result;
}


}  // namespace kmhg
