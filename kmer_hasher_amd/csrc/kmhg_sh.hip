// kmhg_sh.hip -- read counting (count.kmers.fq.sh.rp), per-position depth (seq.kmer.depth.sh)
// and the count spectrum (kmer.spec.sh.n) on a GPU counts index of canonical k-mers.
//
// The reference holds these counts in a suffix_hash_n (src/suffix_hash.c:179-285): 2k-bit
// canonical k-mers, a vector of counts_n uint32 counts each.  Here the same map is a counts
// index (kmhg_count.hip: table + U x counts_n count matrix); a FASTQ batch is merged into it by
//   R_kmers<false>  one lane per read runs the reference's k-mer iterator (quality filter
//                   included) and counts the k-mers it accepts
//   (k_scan_u32)    dense output offsets
//   R_kmers<true>   the same walk again, writing min(forward, reverse complement) per k-mer
//   (partitioned build of the key stream -> distinct keys with occurrence counts, merged into
//    the counts index by C_probe / C_append over the batch table's slots, table rebuilt)
// seq.kmer.depth.sh (seq_kmer_counts, src/kmer_reader.c:155-193) is a sequential walk with a
// restart rule; it is restated over the N-free segments of the sequence (D_* below).
#include <hip/hip_runtime.h>
#include "kmhg_common.h"
#include "kmhg_device.h"
#include "kmhg_kernels.h"
#include "kmhg_sh.h"

namespace kmhg {

// ------------------------------------------------------------------ k-mer iterator per read
// Forward byte reader over an 8-B aligned buffer (padded by >= 8 bytes): one 8-B load per
// 8 chars; the iterator only ever moves forward.  (The global-memory walk of long reads.)
struct ByteCursor {
  const uint64_t* base;
  int64_t w;
  uint64_t word;
  __device__ explicit ByteCursor(const uint8_t* b)
      : base(reinterpret_cast<const uint64_t*>(b)), w(-1), word(0) {}
  __device__ __forceinline__ uint32_t at(int64_t p) {
    const int64_t wi = p >> 3;
    if (wi != w) { w = wi; word = base[wi]; }
    return (uint32_t)(word >> ((p & 7) * 8)) & 0xFFu;
  }
};

__device__ __forceinline__ bool is_n(uint32_t c) { return (c | 0x20u) == 'n'; }
__device__ __forceinline__ uint64_t code2(uint32_t c) { return (c >> 1) & 3u; }
__device__ __forceinline__ uint64_t fwd_push(uint64_t f, uint32_t c) { return (f << 2) | code2(c); }
__device__ __forceinline__ uint64_t rev_push(uint64_t r, uint32_t c) {
  return (r >> 2) | (((code2(c) + 2) & 3u) << 62);   // UPDATE_OFFSET_RC, src/kmer_util.h:9
}

// LDS-staged bytes of a workgroup's reads (absolute index p, staged from `base`)
struct LdsBytes {
  const uint8_t* b;
  int64_t base;
  __device__ __forceinline__ uint32_t at(int64_t p) const { return b[p - base]; }
};

// The reference's kmer_iterator (src/kmer_util.c:64-162) for one read [x, e) of the packed batch,
// as a per-base automaton: every loop trip looks at
// exactly one position, so the lanes of a wave stay in step -- the nested restart loops of
// ReadIter serialise a wave whenever any one lane restarts (measured: 4.6x slower).  States:
// SEEK (= kmer_iterator_begin accumulating i < k bases), SKIP (its skip loop), RUN (_next).
// Read rd's range of keys is [cnt[rd], cnt[rd + 1]), sized by its upper bound (k_read_ub): the
// accepted k-mers, then EMPTY_KEY to the end, which the count-only build skips (k <= 31: never a
// real key) -- one walk, no exact count pass.
template <class Acc>
__device__ __forceinline__ void walk_read(Acc s, Acc q, int64_t x, int64_t e, bool hasq, int k,
                                          double min_ll, const double* qll,
                                          const uint32_t* cnt, uint32_t rd, uint64_t* keys) {
  enum : int { SEEK = 0, SKIP = 1, RUN = 2 };
  const uint64_t mask = (1ull << (2 * k)) - 1;
  const int shift = 64 - 2 * k;
  uint64_t* out = keys + cnt[rd];
  uint32_t n = 0;
  int st = SEEK, i = 0;
  uint64_t f = 0, r = 0;
  double kl = 0, pv = 0;                     // SEEK: running sum, last base's term
  double kll = 0, prev = 0;                  // RUN
  while (x < e) {
    const uint32_t c = s.at(x);
    if (c == 0) break;                       // the C string ends
    const double t = hasq ? qll[q.at(x)] : 0.0;
    if (st == SKIP) {
      if (hasq ? (t <= min_ll) : is_n(c)) { ++x; continue; }
      st = SEEK; i = 0; f = 0; r = 0; kl = 0; pv = 0;      // the attempt restarts here
    }
    if (st == SEEK) {
      bool ok;
      if (hasq) { kl = kl + t; ok = kl > min_ll; }
      else ok = !is_n(c);
      if (!ok) { st = SKIP; continue; }      // the skip loop starts at this same base
      f = fwd_push(f, c); r = rev_push(r, c); pv = t; ++x; ++i;
      if (i < k) continue;
      // success: the loop test adds the following base's term before it sees i == k
      kll = kl; prev = pv;
      if (hasq && x < e && s.at(x) != 0) kll = kll + qll[q.at(x)];
      st = RUN;
    } else {                                 // RUN: kmer_iterator_next / _nq_next
      bool restart;
      if (hasq) {
        kll += (t - prev);
        restart = kll < min_ll;
        prev = t;
      } else {
        restart = is_n(c);
      }
      ++x;
      if (restart) { st = SEEK; i = 0; f = 0; r = 0; kl = 0; pv = 0; continue; }
      f = fwd_push(f, c); r = rev_push(r, c);
    }
    const uint64_t a = f & mask, bb = r >> shift;
    out[n++] = a < bb ? a : bb;
  }
  for (uint32_t i = n, ub = cnt[rd + 1] - cnt[rd]; i < ub; ++i) out[i] = EMPTY_KEY;
}

// One wave per RK_READS consecutive reads, one lane per read.  The wave's bases and qualities
// are staged in LDS with 16-B loads (the iterator's byte-serial walk then waits on LDS, not on
// HBM); a wave whose reads span more than `cap` bytes walks them from global memory instead.
constexpr int RK_READS = 64;

__global__ void __launch_bounds__(RK_READS)
k_read_kmers(const uint8_t* __restrict__ seq, const uint8_t* __restrict__ qual,
             const int64_t* __restrict__ off, const uint8_t* __restrict__ hasq, uint32_t n_reads,
             int k, double min_ll, const double* __restrict__ qll_g, uint32_t cap,
             const uint32_t* __restrict__ cnt, uint64_t* __restrict__ keys) {
  extern __shared__ uint4 rk_smem[];
  double* qll = reinterpret_cast<double*>(rk_smem);
  uint8_t* ls = reinterpret_cast<uint8_t*>(rk_smem) + 256 * sizeof(double);
  uint8_t* lq = ls + cap;
  for (int i = threadIdx.x; i < 256; i += RK_READS) qll[i] = qll_g[i];
  const uint32_t r0 = blockIdx.x * RK_READS;
  const uint32_t r1 = min(n_reads, r0 + RK_READS);
  const int64_t base = off[r0] & ~(int64_t)15;
  const int64_t span = off[r1] - base;
  const bool fits = span <= (int64_t)cap;
  if (fits) {
    const uint32_t nw = (uint32_t)((span + 15) >> 4);
    const uint4* gs = reinterpret_cast<const uint4*>(seq + base);
    const uint4* gq = reinterpret_cast<const uint4*>(qual + base);
    uint4* ws = reinterpret_cast<uint4*>(ls);
    uint4* wq = reinterpret_cast<uint4*>(lq);
    for (uint32_t i = threadIdx.x; i < nw; i += RK_READS) {
      const uint4 a = gs[i], b = gq[i];
      ws[i] = a;
      wq[i] = b;
    }
  }
  __syncthreads();
  const uint32_t rd = r0 + threadIdx.x;
  if (rd >= r1) return;
  const int64_t b = off[rd], e = off[rd + 1];
  const bool hq = hasq[rd] != 0;
  if (fits)
    walk_read(LdsBytes{ls, base}, LdsBytes{lq, base}, b, e, hq, k, min_ll, qll, cnt, rd, keys);
  else
    walk_read(ByteCursor(seq), ByteCursor(qual), b, e, hq, k, min_ll, qll, cnt, rd, keys);
}

// Per-read upper bound of the k-mers the iterator can accept: max(0, length - k + 1).
__global__ void __launch_bounds__(BLOCK)
k_read_ub(const int64_t* __restrict__ off, uint32_t n_reads, int k, uint32_t* __restrict__ cnt) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= n_reads) return;
  const int64_t len = off[r + 1] - off[r];
  cnt[r] = len >= k ? (uint32_t)(len - k + 1) : 0u;
}

void launch_read_ub(const int64_t* off, uint32_t n_reads, int k, uint32_t* cnt, hipStream_t s) {
  hipLaunchKernelGGL(k_read_ub, dim3((n_reads + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, off,
                     n_reads, k, cnt);
}

// The largest byte span one k_read_kmers workgroup stages (RK_READS reads from an aligned-down
// start): sizing the LDS staging exactly (not by a mean-length guess with headroom) lets more
// workgroups share a CU -- the walk is latency bound.
__global__ void __launch_bounds__(BLOCK)
k_rk_span(const int64_t* __restrict__ off, uint32_t n_reads, uint32_t* __restrict__ span) {
  const uint32_t w = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t r0 = w * RK_READS;
  if (r0 >= n_reads) return;
  const uint32_t r1 = min(n_reads, r0 + RK_READS);
  const int64_t sp = off[r1] - (off[r0] & ~(int64_t)15);
  atomicMax(span, (uint32_t)min<int64_t>(sp, 0x7FFFFFFF));
}

void launch_rk_span(const int64_t* off, uint32_t n_reads, uint32_t* span, hipStream_t s) {
  const uint32_t nw = (n_reads + RK_READS - 1) / RK_READS;
  hipLaunchKernelGGL(k_rk_span, dim3((nw + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, off, n_reads,
                     span);
}

void launch_read_kmers(const uint8_t* seq, const uint8_t* qual, const int64_t* off,
                       const uint8_t* hasq, uint32_t n_reads, int k, double min_ll,
                       const double* qll, uint32_t cap, const uint32_t* cnt, uint64_t* keys,
                       hipStream_t s) {
  const dim3 grid((n_reads + RK_READS - 1) / RK_READS);
  const size_t smem = 256 * sizeof(double) + 2 * (size_t)cap;
  hipLaunchKernelGGL(k_read_kmers, grid, dim3(RK_READS), smem, s, seq, qual, off, hasq, n_reads, k,
                     min_ll, qll, cap, cnt, keys);
}

// ------------------------------------------------------------------ depth: N-free segments
// seq_kmer_counts walks the sequence once.  An "init" (init_kmer_qual_2) starts at i = 0 and at
// every N met in normal flow: it resets the rolling k-mer, skips N-runs and segments shorter
// than k, and writes the first full window of the segment it lands on at that window's START.
// Normal flow then shifts in one base per step and writes at (end - k), i.e. one position left of
// the window's start -- so the init's write is overwritten unless the segment is exactly k long.
// When the init's window ends exactly at an N, that N-run is skipped WITHOUT a reset and the next
// segment is walked in normal flow with the k bases before the gap still in the register
// ("stale" segment, windows span the gap).  Per segment: stale iff the previous segment was a
// seek segment of length exactly k.  Every output position is written at most once:
//   seek, len > k : base at offset t >= k writes window [i-k+1, i] at i - k
//   seek, len = k : its last base writes window [a, a+k) at a
//   stale         : every base writes the last k bases of (previous k-segment ++ segment) at i - k
//   end           : if the walk ends inside an init that found no window, the partial register
//                   (last segment tried, or nothing after an N) is looked up and written at L - k

__device__ __forceinline__ bool nat(const uint8_t* __restrict__ s, int64_t L, int64_t i) {
  return i >= 0 && i < L && is_n(s[i]);
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* tot) {
  __shared__ uint32_t wsum[BLOCK / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t base = 0, all = 0;
  for (int j = 0; j < BLOCK / 64; ++j) {
    if (j < w) base += wsum[j];
    all += wsum[j];
  }
  __syncthreads();
  if (tot) *tot = all;
  return base + x - v;
}

__global__ void __launch_bounds__(BLOCK)
k_depth_seg_count(const uint8_t* __restrict__ s, int64_t L, uint32_t* __restrict__ tcnt) {
  const int64_t i0 = (int64_t)blockIdx.x * DP_TILE + (int64_t)threadIdx.x * DP_CPT;
  uint32_t c = 0;
  bool prev_n = i0 == 0 ? true : nat(s, L, i0 - 1);
  for (int t = 0; t < DP_CPT; ++t) {
    const int64_t i = i0 + t;
    if (i >= L) break;
    const bool n = is_n(s[i]);
    c += (!n && prev_n);
    prev_n = n;
  }
  uint32_t tot = 0;
  block_excl_scan(c, &tot);
  if (threadIdx.x == 0) tcnt[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK)
k_depth_seg_emit(const uint8_t* __restrict__ s, int64_t L, const uint32_t* __restrict__ tbase,
                 uint32_t* __restrict__ sstart, uint32_t* __restrict__ send) {
  const int64_t i0 = (int64_t)blockIdx.x * DP_TILE + (int64_t)threadIdx.x * DP_CPT;
  uint32_t c = 0;
  {
    bool prev_n = i0 == 0 ? true : nat(s, L, i0 - 1);
    for (int t = 0; t < DP_CPT; ++t) {
      const int64_t i = i0 + t;
      if (i >= L) break;
      const bool n = is_n(s[i]);
      c += (!n && prev_n);
      prev_n = n;
    }
  }
  uint32_t r = tbase[blockIdx.x] + block_excl_scan(c, nullptr);
  bool prev_n = i0 == 0 ? true : nat(s, L, i0 - 1);
  for (int t = 0; t < DP_CPT; ++t) {
    const int64_t i = i0 + t;
    if (i >= L) break;
    const bool n = is_n(s[i]);
    if (!n && prev_n) sstart[r++] = (uint32_t)i;
    if (!n && (i + 1 == L || is_n(s[i + 1]))) send[r - 1] = (uint32_t)(i + 1);
    prev_n = n;
  }
}

// the counts of `key` (zeros when absent) written to out[w * S ...]
__device__ __forceinline__ void depth_write(const Slot* __restrict__ T, Geom g, uint32_t S,
                                            const int32_t* __restrict__ M, uint64_t key,
                                            int32_t* __restrict__ out, int64_t w) {
  uint32_t c = 0, aux = 0;
  // (round 5, A/B in one run: four slots per round trip, table_find4, 0.385 -> 0.443 ms at
  // config 2 -- profiles/r5g_ab_depth.log)
  const uint32_t slot = table_find(T, g, key, c, aux);
  int32_t* o = out + w * S;
  if (slot == NONE) {
    for (uint32_t j = 0; j < S; ++j) o[j] = 0;
  } else if (S == 1) {
    o[0] = (int32_t)aux;                       // source_n = 1: the count sits in the slot
  } else {
    const int32_t* v = M + (aux - S);
    for (uint32_t j = 0; j < S; ++j) o[j] = v[j];
  }
}

// Segment modes (stale flags) by a chained scan of the 2-state automaton over the segment list,
// then the end-of-walk partial write.  One workgroup.
__global__ void __launch_bounds__(BLOCK)
k_depth_modes(const uint8_t* __restrict__ s, int64_t L, int k, const uint32_t* __restrict__ sstart,
              const uint32_t* __restrict__ send, const uint32_t* __restrict__ n_seg,
              uint8_t* __restrict__ stale, const Slot* __restrict__ T, Geom g, uint32_t S,
              const int32_t* __restrict__ M, int32_t* __restrict__ out) {
  __shared__ uint8_t t0[BLOCK], t1[BLOCK], tin[BLOCK];
  const uint32_t m_all = *n_seg;
  const uint32_t chunk = (m_all + BLOCK - 1) / BLOCK;
  const uint32_t a = threadIdx.x * chunk, b = min(m_all, a + chunk);
  // transition of this chunk for input state 0 (seek) and 1 (stale)
  uint32_t x0 = 0, x1 = 1;
  for (uint32_t m = a; m < b; ++m) {
    const bool exact = send[m] - sstart[m] == (uint32_t)k;
    x0 = (x0 == 0 && exact) ? 1u : 0u;
    x1 = (x1 == 0 && exact) ? 1u : 0u;
  }
  t0[threadIdx.x] = (uint8_t)x0;
  t1[threadIdx.x] = (uint8_t)x1;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint8_t st = 0;
    for (int t = 0; t < BLOCK; ++t) { tin[t] = st; st = st ? t1[t] : t0[t]; }
  }
  __syncthreads();
  uint32_t st = tin[threadIdx.x];
  for (uint32_t m = a; m < b; ++m) {
    stale[m] = (uint8_t)st;
    st = (st == 0 && send[m] - sstart[m] == (uint32_t)k) ? 1u : 0u;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  // end of the walk
  if (L - k < 0 || L == 0) return;             // the reference writes before its buffer there
  uint64_t f = 0, r = 0;
  bool partial;
  if (m_all == 0) {
    partial = true;                            // all N: the init's only attempt holds nothing
  } else {
    const uint32_t m = m_all - 1;
    const uint32_t sa = sstart[m], sb = send[m], len = sb - sa;
    const bool last_stale = stale[m] != 0;
    if (!last_stale && len < (uint32_t)k) {
      partial = true;                          // the last segment tried, shorter than k
      for (uint32_t i = sa; i < sb; ++i) { f = fwd_push(f, s[i]); r = rev_push(r, s[i]); }
    } else if (!last_stale && len == (uint32_t)k) {
      partial = false;                         // init succeeded; a trailing N-run is skipped
    } else {
      partial = (int64_t)sb < L;               // normal flow ends at an N: the init finds nothing
    }
  }
  if (!partial) return;
  const uint64_t mask = (1ull << (2 * k)) - 1;
  const uint64_t fa = f & mask, rb = r >> (64 - 2 * k);
  depth_write(T, g, S, M, fa < rb ? fa : rb, out, L - k);
}

// reverse complement of a forward key of k bases: complement = code ^ 2 (A0 C1 T2 G3), then
// the 2-bit groups in reverse order -- equals the reference's rolling UPDATE_OFFSET_RC register
// shifted down by 64 - 2k (src/kmer_util.h:9, src/kmer_reader.c:168-169)
__device__ __forceinline__ uint64_t revcomp(uint64_t f, int k) {
  const uint64_t x = __builtin_bitreverse64(f ^ 0xAAAAAAAAAAAAAAAAull);
  const uint64_t y = ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
  return y >> (64 - 2 * k);
}

constexpr int DP_STAGE_W16 = 22;             // chars [tile - 63.., +352): every window ending in the tile

// One lane per base i of a 256-base tile (the base that ENDS a window).  The tile's chars are
// staged as 2-bit codes in LDS; the window's forward key comes from the stage and its reverse
// complement by bit reversal (no per-lane k-char loop).  The write rule (kmhg_sh.hip header):
// seek segments longer than k write window [i-k+1, i] at i - k from offset k on; a segment of
// exactly k writes its window at its start; stale segments write every base, the first k - 1
// of them (their windows span the N gap) by a short loop over global memory.
__global__ void __launch_bounds__(BLOCK)
k_depth_probe(const uint8_t* __restrict__ s, int64_t L, int k, bool aligned,
              const uint32_t* __restrict__ sstart, const uint32_t* __restrict__ send,
              const uint32_t* __restrict__ n_seg, const uint8_t* __restrict__ stale,
              const Slot* __restrict__ T, Geom g, uint32_t S, const int32_t* __restrict__ M,
              int32_t* __restrict__ out) {
  __shared__ StageN<DP_STAGE_W16> st;
  __shared__ int32_t mrange[2];
  const int64_t t0 = (int64_t)blockIdx.x * BLOCK;
  const int64_t base = (t0 - 48) & ~(int64_t)15;
  stage_tile<false, DP_STAGE_W16>(s, L, base, st, aligned);
  const uint32_t ms = *n_seg;
  if (threadIdx.x < 2 && ms) {                 // segments holding the tile's first / last base
    const int64_t at = threadIdx.x == 0 ? t0 : min(t0 + BLOCK, L) - 1;
    uint32_t lo = 0, hi = ms;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if ((int64_t)sstart[mid] <= at) lo = mid + 1; else hi = mid;
    }
    mrange[threadIdx.x] = (int32_t)lo - 1;
  }
  __syncthreads();
  const int64_t i = t0 + threadIdx.x;
  if (i >= L || !ms) return;
  int32_t m = mrange[0];
  while (m < mrange[1] && (int64_t)sstart[m + 1] <= i) ++m;
  if (m < 0) return;
  const int64_t a = sstart[m], b = send[m];
  if (i >= b) return;                          // an N
  const int64_t off = i - a, len = b - a;
  const bool stl = stale[m] != 0;
  int64_t w;
  if (stl) w = i - k;
  else if (len > k && off >= k) w = i - k;
  else if (len == k && off == k - 1) w = a;
  else return;
  uint64_t f;
  const int64_t from_prev = stl ? (int64_t)k - 1 - off : 0;
  if (from_prev > 0) {                         // window across the gap: previous segment's tail
    f = 0;
    const int64_t pb = send[m - 1];
    for (int64_t j = pb - from_prev; j < pb; ++j) f = fwd_push(f, s[j]);
    for (int64_t j = a; j <= i; ++j) f = fwd_push(f, s[j]);
  } else {
    const int o = (int)(i - k + 1 - base);
    const int qw = o >> 4, bsh = (o & 15) * 2;
    const uint64_t x = ((uint64_t)st.code[qw] << 32) | st.code[qw + 1];
    const uint64_t y = st.code[qw + 2];
    f = ((x << bsh) | ((y << bsh) >> 32)) >> (64 - 2 * k);
  }
  const uint64_t rc = revcomp(f, k);
  depth_write(T, g, S, M, f < rc ? f : rc, out, w);
}

void launch_depth_seg_count(const uint8_t* seq, int64_t L, uint32_t* tcnt, hipStream_t s) {
  hipLaunchKernelGGL(k_depth_seg_count, dim3(depth_tiles(L)), dim3(BLOCK), 0, s, seq, L, tcnt);
}
void launch_depth_seg_emit(const uint8_t* seq, int64_t L, const uint32_t* tbase, uint32_t* sstart,
                           uint32_t* send, hipStream_t s) {
  hipLaunchKernelGGL(k_depth_seg_emit, dim3(depth_tiles(L)), dim3(BLOCK), 0, s, seq, L, tbase,
                     sstart, send);
}
void launch_depth_modes(const uint8_t* seq, int64_t L, int k, const uint32_t* sstart,
                        const uint32_t* send, const uint32_t* n_seg, uint8_t* stale, const Slot* T,
                        Geom g, uint32_t S, const int32_t* M, int32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_depth_modes, dim3(1), dim3(BLOCK), 0, s, seq, L, k, sstart, send, n_seg,
                     stale, T, g, S, M, out);
}
void launch_depth_probe(const uint8_t* seq, int64_t L, int k, const uint32_t* sstart,
                        const uint32_t* send, const uint32_t* n_seg, const uint8_t* stale,
                        const Slot* T, Geom g, uint32_t S, const int32_t* M, int32_t* out,
                        hipStream_t s) {
  const bool aligned = (reinterpret_cast<uintptr_t>(seq) & 15) == 0;
  hipLaunchKernelGGL(k_depth_probe, dim3((unsigned)((L + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                     seq, L, k, aligned, sstart, send, n_seg, stale, T, g, S, M, out);
}

// ------------------------------------------------------------------ spectrum
// sh_count_spectrum_nc (src/suffix_hash.c:338-421): per k-mer, flag bit j = (count_j >=
// source_min_j); for every combination jj it matches (inner: flag == comb, else flag & comb),
// bin min(count_k, max_count) of column (jj, k) gains one.  Bins are u32 (U < 2^32) in LDS per
// workgroup when they fit, flushed with one global atomic per non-zero bin.
constexpr uint32_t SPEC_LDS_BINS = 8192;

__global__ void __launch_bounds__(BLOCK)
k_spectrum(const int32_t* __restrict__ M, uint64_t U, uint32_t S, uint32_t max_count,
           const uint32_t* __restrict__ comb, const uint32_t* __restrict__ inner, uint32_t comb_n,
           const uint32_t* __restrict__ smin, uint32_t* __restrict__ bins) {
  __shared__ uint32_t lb[SPEC_LDS_BINS];
  const uint64_t nbins = (uint64_t)(max_count + 1) * comb_n * S;
  const bool use_lds = nbins <= SPEC_LDS_BINS;
  if (use_lds) {
    for (uint32_t i = threadIdx.x; i < nbins; i += BLOCK) lb[i] = 0;
    __syncthreads();
  }
  for (uint64_t r = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; r < U;
       r += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t* v = reinterpret_cast<const uint32_t*>(M + r * S);
    uint32_t vals[4];
    uint32_t flag = 0;
    for (uint32_t j = 0; j < S; ++j) {
      vals[j] = v[j];
      flag |= (uint32_t)(vals[j] >= smin[j]) << j;
    }
    for (uint32_t jj = 0; jj < comb_n; ++jj) {
      if (!((inner[jj] && flag == comb[jj]) || (!inner[jj] && (flag & comb[jj]) > 0))) continue;
      for (uint32_t kk = 0; kk < S; ++kk) {
        const uint32_t c = vals[kk] < max_count ? vals[kk] : max_count;
        const uint64_t bin = (uint64_t)c * (comb_n * S) + jj * S + kk;
        if (use_lds) atomicAdd(&lb[bin], 1u);
        else atomicAdd(&bins[bin], 1u);
      }
    }
  }
  if (use_lds) {
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nbins; i += BLOCK)
      if (lb[i]) atomicAdd(&bins[i], lb[i]);
  }
}

void launch_spectrum(const int32_t* M, uint64_t U, uint32_t S, uint32_t max_count,
                     const uint32_t* comb, const uint32_t* inner, uint32_t comb_n,
                     const uint32_t* smin, uint32_t* bins, hipStream_t s) {
  uint64_t g = (U + BLOCK - 1) / BLOCK;
  if (g > 2048) g = 2048;
  if (g == 0) g = 1;
  hipLaunchKernelGGL(k_spectrum, dim3((unsigned)g), dim3(BLOCK), 0, s, M, U, S, max_count, comb,
                     inner, comb_n, smin, bins);
}

}  // namespace kmhg

namespace kmhg {

// Fallback of a batch table whose partitioned build overflowed a bucket: global find-or-insert
// and an atomic count per key occurrence (nb = 1 table).
__global__ void __launch_bounds__(BLOCK)
k_key_count_insert(const uint64_t* __restrict__ keys, uint64_t n, Slot* __restrict__ T, Geom g) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t key = keys[i];
    if (key == EMPTY_KEY) continue;              // padding (suffix-hash k <= 31: never a key)
    const uint32_t slot = table_insert(T, g, key);
    atomicAdd(&T[slot].count, 1u);
  }
}

void launch_key_count_insert(const uint64_t* keys, uint64_t n, Slot* T, Geom g, hipStream_t s) {
  uint64_t gr = (n + BLOCK - 1) / BLOCK;
  if (gr > 16384) gr = 16384;
  if (gr == 0) gr = 1;
  hipLaunchKernelGGL(k_key_count_insert, dim3((unsigned)gr), dim3(BLOCK), 0, s, keys, n, T, g);
}

}  // namespace kmhg
