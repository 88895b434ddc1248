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
// Forward byte reader over an 8-B aligned buffer (padded by >= 8 bytes): one dword pair load
// per 8 chars; the iterator only ever moves forward.
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

// The reference's kmer_iterator (src/kmer_util.c:64-162) for one read [b, e) of the packed
// batch, its tail recursion unrolled.  With qualities the window's running log-likelihood is
// kept exactly as the reference accumulates it (double adds in the same order: bit-identical).
struct ReadIter {
  ByteCursor s, q;
  int64_t p, e;
  int k;
  bool hasq;
  uint64_t f, r;
  double kll, prev, min_ll;
  const double* qll;

  __device__ bool end(int64_t x) { return x >= e || s.at(x) == 0; }

  __device__ bool begin_nq(int64_t x) {           // kmer_iterator_nq_begin
    for (;;) {
      uint64_t ff = 0, rr = 0;
      int i = 0;
      while (!end(x) && !is_n(s.at(x)) && i < k) {
        const uint32_t c = s.at(x);
        ff = fwd_push(ff, c); rr = rev_push(rr, c); ++x; ++i;
      }
      if (i == k) { f = ff; r = rr; p = x; return true; }
      while (!end(x) && is_n(s.at(x))) ++x;
      if (end(x)) return false;
    }
  }
  __device__ bool begin_q(int64_t x) {            // kmer_iterator_begin
    for (;;) {
      uint64_t ff = 0, rr = 0;
      double kl = 0, pv = 0;
      int i = 0;
      // the next base's term is added before i < k is tested (a k + 1-th term mid-read)
      while (!end(x) && ((kl = kl + qll[q.at(x)]) > min_ll) && i < k) {
        const uint32_t c = s.at(x);
        ff = fwd_push(ff, c); rr = rev_push(rr, c);
        pv = qll[q.at(x)];
        ++x; ++i;
      }
      if (i == k) { f = ff; r = rr; p = x; prev = pv; kll = kl; return true; }
      while (!end(x) && qll[q.at(x)] <= min_ll) ++x;
      if (end(x)) return false;
    }
  }
  __device__ bool begin() { return hasq ? begin_q(p) : begin_nq(p); }
  __device__ bool next() {                        // kmer_iterator_next / _nq_next
    if (end(p)) return false;
    const uint32_t c = s.at(p);
    if (!hasq) {
      if (is_n(c)) return begin_nq(p + 1);
    } else {
      const double t = qll[q.at(p)];
      kll += (t - prev);
      if (kll < min_ll) return begin_q(p + 1);
      prev = t;
    }
    f = fwd_push(f, c); r = rev_push(r, c);
    ++p;
    return true;
  }
};

template <bool EMIT>
__global__ void __launch_bounds__(BLOCK)
k_read_kmers(const uint8_t* __restrict__ seq, const uint8_t* __restrict__ qual,
             const int64_t* __restrict__ off, const uint8_t* __restrict__ hasq, uint32_t n_reads,
             int k, double min_ll, const double* __restrict__ qll_g, uint32_t* __restrict__ cnt,
             uint64_t* __restrict__ keys) {
  __shared__ double qll[256];
  qll[threadIdx.x] = qll_g[threadIdx.x];
  __syncthreads();
  const uint32_t rd = blockIdx.x * BLOCK + threadIdx.x;
  if (rd >= n_reads) return;
  ReadIter it{ByteCursor(seq), ByteCursor(qual), off[rd], off[rd + 1], k, hasq[rd] != 0,
              0, 0, 0, 0, min_ll, qll};
  const uint64_t mask = (1ull << (2 * k)) - 1;
  const int shift = 64 - 2 * k;
  uint32_t n = 0;
  uint64_t* out = EMIT ? keys + cnt[rd] : nullptr;
  bool ok = it.begin();
  while (ok) {
    if (EMIT) {
      const uint64_t a = it.f & mask, b = it.r >> shift;
      out[n] = a < b ? a : b;
    }
    ++n;
    ok = it.next();
  }
  if (!EMIT) cnt[rd] = n;
}

void launch_read_kmers(const uint8_t* seq, const uint8_t* qual, const int64_t* off,
                       const uint8_t* hasq, uint32_t n_reads, int k, double min_ll,
                       const double* qll, uint32_t* cnt, uint64_t* keys, bool emit,
                       hipStream_t s) {
  const dim3 grid((n_reads + BLOCK - 1) / BLOCK);
  if (emit)
    hipLaunchKernelGGL(k_read_kmers<true>, grid, dim3(BLOCK), 0, s, seq, qual, off, hasq, n_reads,
                       k, min_ll, qll, cnt, keys);
  else
    hipLaunchKernelGGL(k_read_kmers<false>, grid, dim3(BLOCK), 0, s, seq, qual, off, hasq,
                       n_reads, k, min_ll, qll, cnt, keys);
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

// One lane per DP_CPT consecutive bases: the base's segment (binary search once, then walk), its
// write rule, the rolling canonical key, the probe, the write.
__global__ void __launch_bounds__(BLOCK)
k_depth_probe(const uint8_t* __restrict__ s, int64_t L, int k,
              const uint32_t* __restrict__ sstart, const uint32_t* __restrict__ send,
              const uint32_t* __restrict__ n_seg, const uint8_t* __restrict__ stale,
              const Slot* __restrict__ T, Geom g, uint32_t S, const int32_t* __restrict__ M,
              int32_t* __restrict__ out) {
  const int64_t i0 = (int64_t)blockIdx.x * DP_TILE + (int64_t)threadIdx.x * DP_CPT;
  if (i0 >= L) return;
  const uint32_t ms = *n_seg;
  if (!ms) return;
  // last segment starting at or before i0
  uint32_t lo = 0, hi = ms;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((int64_t)sstart[mid] <= i0) lo = mid + 1; else hi = mid;
  }
  int64_t m = (int64_t)lo - 1;
  const uint64_t mask = (1ull << (2 * k)) - 1;
  const int shift = 64 - 2 * k;
  uint64_t f = 0, r = 0;
  int64_t have_at = -2;                        // the register holds the window ending here
  for (int t = 0; t < DP_CPT; ++t) {
    const int64_t i = i0 + t;
    if (i >= L) break;
    while (m + 1 < (int64_t)ms && (int64_t)sstart[m + 1] <= i) ++m;
    if (m < 0) continue;
    const int64_t a = sstart[m], b = send[m];
    if (i >= b) continue;                      // an N
    const int64_t off = i - a, len = b - a;
    const bool st = stale[m] != 0;
    int64_t w;
    if (st) w = i - k;
    else if (len > k && off >= k) w = i - k;
    else if (len == k && off == k - 1) w = a;
    else continue;
    if (have_at == i - 1) {
      const uint32_t c = s[i];
      f = fwd_push(f, c); r = rev_push(r, c);
    } else {                                   // (re)load the k stream bases ending at i
      f = 0; r = 0;
      const int64_t from_prev = st ? (int64_t)k - 1 - off : 0;   // > 0 only across the gap
      if (from_prev > 0) {
        const int64_t pb = send[m - 1];
        for (int64_t j = pb - from_prev; j < pb; ++j) { f = fwd_push(f, s[j]); r = rev_push(r, s[j]); }
        for (int64_t j = a; j <= i; ++j) { f = fwd_push(f, s[j]); r = rev_push(r, s[j]); }
      } else {
        for (int64_t j = i - k + 1; j <= i; ++j) { f = fwd_push(f, s[j]); r = rev_push(r, s[j]); }
      }
    }
    have_at = i;
    const uint64_t fa = f & mask, rb = r >> shift;
    depth_write(T, g, S, M, fa < rb ? fa : rb, out, w);
  }
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
  hipLaunchKernelGGL(k_depth_probe, dim3(depth_tiles(L)), dim3(BLOCK), 0, s, seq, L, k, sstart,
                     send, n_seg, stale, T, g, S, M, out);
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
    const uint32_t slot = table_insert(T, g, keys[i]);
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
