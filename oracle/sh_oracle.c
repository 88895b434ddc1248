/*
 * oracle/sh_oracle.c -- TEST INFRASTRUCTURE ONLY (linked into liboracle.so with kmer_oracle.c).
 *
 * Clean-room CPU restatement of the reference's read-counting path (count.kmers.fq.sh.rp ->
 * suffix_hash_n) and of seq.kmer.depth.sh, written from the behaviour of lmjakt/kmer_hasheR.
 * Pinned against the reference's own compiled counting core (oracle/_ref/libkmh_ref_sh.so,
 * see ref_sh_harness.c) by tests/test_sh_oracle.py and the vectors in tests/golden/.
 *
 *   orc_qll        the phred -> log-likelihood table q_to_ll (src/Q_to_log_likelihood.h): -708
 *                  below '"', else log(1 - 10^(-(q - 33) / 10)) rounded to 15 significant
 *                  digits (the reference pasted R's printout); equality with the header's 256
 *                  doubles is checked by tests/golden/make_sh_golden.py
 *   orc_read_kmers the k-mer iterator of one read (kmer_iterator_begin / _next and the _nq_
 *                  variants, src/kmer_util.c:64-162) as used by kmer_reader_read
 *                  (src/kmer_reader.c:41-76): emits min(forward, reverse complement) of every
 *                  accepted window, in iteration order
 *   orc_depth      seq_kmer_counts (src/kmer_reader.c:155-193) with init_kmer_qual_2 / skip_n
 *                  (src/kmer_util.c:4-8, 34-52) over a sorted (key, counts) table
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define SH_IS_N(c) ((((unsigned char)(c)) | 0x20) == 'n')
#define SH_CODE(c) ((((uint64_t)(unsigned char)(c)) >> 1) & 3u)
/* forward: append the base's code at the low end; reverse complement: complement ((code + 2)
 * mod 4 swaps A<->T, C<->G in the A0 C1 T2 G3 code) enters at the top (src/kmer_util.h:8-9) */
#define SH_FWD(f, c) (((f) << 2) | SH_CODE(c))
#define SH_REV(r, c) (((r) >> 2) | (((SH_CODE(c) + 2) & 3u) << 62))

void orc_qll(double *out) {
  for (int q = 0; q < 256; ++q) {
    if (q < 34) { out[q] = -708.0; continue; }
    char buf[64];
    snprintf(buf, sizeof buf, "%.15g", log(1.0 - pow(10.0, -(double)(q - 33) / 10.0)));
    out[q] = strtod(buf, 0);
  }
}

typedef struct {
  const unsigned char *s, *q;
  long len, p;
  int k;
  uint64_t f, r;
  double kll, prev, min_ll;
  const double *qll;
} orc_it;

static int it_end(const orc_it *it, long p) { return p >= it->len || it->s[p] == 0; }

/* kmer_iterator_nq_begin, its recursion unrolled into a loop */
static int it_begin_nq(orc_it *it, long p) {
  for (;;) {
    uint64_t f = 0, r = 0;
    int i = 0;
    while (!it_end(it, p) && !SH_IS_N(it->s[p]) && i < it->k) {
      f = SH_FWD(f, it->s[p]); r = SH_REV(r, it->s[p]); ++p; ++i;
    }
    if (i == it->k) { it->f = f; it->r = r; it->p = p; return 1; }
    while (!it_end(it, p) && SH_IS_N(it->s[p])) ++p;
    if (it_end(it, p)) return 0;
  }
}

/* kmer_iterator_begin with qualities.  The loop condition adds the next base's log-likelihood
 * before it tests i < k, so a window that is not at the read's end carries k + 1 terms. */
static int it_begin_q(orc_it *it, long p) {
  for (;;) {
    uint64_t f = 0, r = 0;
    double kll = 0, prev = 0;
    int i = 0;
    while (!it_end(it, p) && ((kll = kll + it->qll[it->q[p]]) > it->min_ll) && i < it->k) {
      f = SH_FWD(f, it->s[p]); r = SH_REV(r, it->s[p]);
      prev = it->qll[it->q[p]];
      ++p; ++i;
    }
    if (i == it->k) { it->f = f; it->r = r; it->p = p; it->prev = prev; it->kll = kll; return 1; }
    while (!it_end(it, p) && it->qll[it->q[p]] <= it->min_ll) ++p;
    if (it_end(it, p)) return 0;
  }
}

static int it_next(orc_it *it) {
  if (it_end(it, it->p)) return 0;
  const long p = it->p;
  if (!it->q) {
    if (SH_IS_N(it->s[p])) return it_begin_nq(it, p + 1);
  } else {
    it->kll += (it->qll[it->q[p]] - it->prev);
    if (it->kll < it->min_ll) return it_begin_q(it, p + 1);
    it->prev = it->qll[it->q[p]];
  }
  it->f = SH_FWD(it->f, it->s[p]);
  it->r = SH_REV(it->r, it->s[p]);
  it->p = p + 1;
  return 1;
}

/* Canonical k-mers of one read (qual = NULL for a FASTA record).  min_q_param is params[2] of
 * count.kmers.fq.sh.rp: the threshold is q_to_ll['!' + min_q_param] (src/kmer_hash.c:821).
 * Returns the number written to out (capacity len - k + 1). */
long orc_read_kmers(const unsigned char *seq, const unsigned char *qual, long len, int k,
                    int min_q_param, uint64_t *out) {
  static double qll[256];
  static int ready = 0;
  if (!ready) { orc_qll(qll); ready = 1; }
  if (k < 1 || k > 31 || len <= k) return 0;
  orc_it it = {seq, qual, len, 0, k, 0, 0, 0, 0, 0, qll};
  it.min_ll = qll[(unsigned char)('!' + (unsigned char)min_q_param)];
  const uint64_t mask = ((uint64_t)1 << (2 * k)) - 1;
  const int shift = 64 - 2 * k;
  long n = 0;
  int ok = qual ? it_begin_q(&it, 0) : it_begin_nq(&it, 0);
  while (ok) {
    const uint64_t a = it.f & mask, b = it.r >> shift;
    out[n++] = a < b ? a : b;
    ok = it_next(&it);
  }
  return n;
}

static long find_key(const uint64_t *keys, long U, uint64_t key) {
  long lo = 0, hi = U;
  while (lo < hi) {
    long mid = (lo + hi) / 2;
    if (keys[mid] < key) lo = mid + 1; else hi = mid;
  }
  return (lo < U && keys[lo] == key) ? lo : -1;
}

/* seq_kmer_counts: out is cn x L int32 (column-major).  Positions never written hold INT_MIN
 * (R's NA); a key absent from the table writes zeros.  keys[] ascending. */
int orc_depth(const uint64_t *keys, const int32_t *counts, long U, int cn, const char *seq,
              long L, int k, int32_t *out) {
  for (long i = 0; i < L * cn; ++i) out[i] = INT_MIN;
  const uint64_t mask = ((uint64_t)1 << (2 * k)) - 1;
  const int shift = 64 - 2 * k;
  uint64_t f = 0, r = 0;
#define END(x) ((x) >= L || seq[(x)] == 0)
#define WRITE(at)                                                                   \
  do {                                                                              \
    const long w_ = (long)(at);                                                     \
    const uint64_t a_ = f & mask, b_ = r >> shift, key_ = a_ < b_ ? a_ : b_;        \
    if (w_ >= 0) {                                                                  \
      const long h_ = find_key(keys, U, key_);                                      \
      for (int j_ = 0; j_ < cn; ++j_) out[w_ * cn + j_] = h_ < 0 ? 0 : counts[h_ * cn + j_]; \
    }                                                                               \
  } while (0)
  long i = 0;
  while (!END(i)) {
    if (i == 0 || SH_IS_N(seq[i])) {
      /* init_kmer_qual_2 without qualities */
      long j = 0;
      while (!END(i)) {
        f = 0; r = 0;
        for (j = 0; j < k && !END(i + j) && !SH_IS_N(seq[i + j]); ++j) {
          f = SH_FWD(f, seq[i + j]); r = SH_REV(r, seq[i + j]);
        }
        if (END(i + j) || j == k) break;
        i += j;
        while (!END(i) && SH_IS_N(seq[i])) ++i;
        j = 0;
      }
      i += j;
      WRITE(i - k);
      if (END(i)) break;
      if (SH_IS_N(seq[i])) {
        while (!END(i) && SH_IS_N(seq[i])) ++i;
        continue;
      }
    }
    f = SH_FWD(f, seq[i]); r = SH_REV(r, seq[i]);
    WRITE(i - k);
    ++i;
  }
#undef WRITE
#undef END
  return 1;
}
