/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never the measured path).
 *
 * A tiny R-free driver over the *reference's own* index core, compiled from the sources
 * where they lie under /root/reference/src (see oracle/Makefile; output goes to oracle/_ref/).
 * R is not installed in this image, so src/kmer_hash.c (which needs Rinternals.h) cannot be
 * compiled; the three .Call wrappers of the hot path are restated here without the R API:
 *
 *   ref_build      <- make_kmer_h_index      (reference src/kmer_hash.c:506-540)
 *   ref_positions  <- kmer_positions         (reference src/kmer_hash.c:1054-1147)
 *   ref_query      <- sequence_kmer_positions(reference src/kmer_hash.c:1151-1172)
 *   ref_free_index <- finalise_khash_ptr     (reference src/kmer_hash.c:56-66)
 *   decode_kmer    <- kmer_seq               (reference src/kmer_hash.c:123-133)
 *   ref_count      <- count_kmers            (reference src/kmer_hash.c:548-591)
 *                     + seq_to_counts :220-251, kmer_count_insert :185-208 (also in
 *                     kmer_hash.c, so restated here over the compiled khash/kvec/init_kmer)
 *
 * The heavy lifting (seq_to_hash, seq_kmer_positions, sort_kmer_pos, clear_kmer_h and the
 * khash/kvec containers) is the reference's compiled code, linked in unchanged.
 * Outputs are malloc'd flat arrays laid out exactly as the R matrices' column-major data.
 */
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "kmer_pos.h"
#include "kmer_util.h"

/* 2-bit code -> base, the decode table of kmer_hash.c:21 */
static const char REF_NUC[4] = {'A', 'C', 'T', 'G'};

static void decode_kmer(char *out, int k, uint64_t key) {
  out[k] = 0;
  for (int c = k - 1; c >= 0; --c) { out[c] = REF_NUC[key & 3]; key >>= 2; }
}

/* error codes mirror the R error() branches of make_kmer_h_index */
#define REF_EK 1   /* k must be a positive integer less than 1+MAX_K */
#define REF_EL 2   /* the length of the sequence must be at least k */

void *ref_build(const char *seq, int k, int do_sort, long *kmer_count, int *err) {
  *err = 0;
  if (k < 1 || k > MAX_K) { *err = REF_EK; return 0; }
  if ((long)strlen(seq) <= k) { *err = REF_EL; return 0; }
  khash_ptr *p = calloc(1, sizeof(khash_ptr));
  p->k = k;
  p->hash = kh_init(kmer_h);
  p->kmer_count = seq_to_hash(seq, k, p->hash);
  if (do_sort) sort_kmer_pos(p);
  if (kmer_count) *kmer_count = (long)p->kmer_count;
  return p;
}

long ref_size(void *h) { return (long)kh_size(((khash_ptr *)h)->hash); }

void ref_free_index(void *h) {
  khash_ptr *p = (khash_ptr *)h;
  if (!p) return;
  if (p->hash) { clear_kmer_h(p->hash); p->hash = 0; }
  free(p);
}

void ref_free(void *x) { free(x); }

typedef struct {
  long n_kmers;  char *kmers;   /* n_kmers strings of k+1 bytes (NUL-terminated) */
  long n_pos;    int  *pos;     /* 2 x n_pos   column-major (i, pos)            */
  long n_pairs;  int  *pairs;   /* 3 x n_pairs column-major (i, x, y)           */
  long n_counts; int  *counts;  /* n_counts                                     */
} ref_pos_result;

/* Bucket walk of kmer_positions: opt bits 1 kmer / 2 pos / 4 pair.pos / 8 count.
 * i is the 1-based rank of the bucket among existing buckets (khash order). */
int ref_positions(void *h, unsigned opt, ref_pos_result *r) {
  khash_ptr *p = (khash_ptr *)h;
  khash_t(kmer_h) *hash = p->hash;
  int k = p->k;
  memset(r, 0, sizeof(*r));
  long U = (long)kh_size(hash), npos = 0, npair = 0;
  /* pre-size: one sweep for totals */
  for (khiter_t it = kh_begin(hash); it != kh_end(hash); ++it) {
    if (!kh_exist(hash, it)) continue;
    long n = (long)kh_val(hash, it).v.n;
    npos += n; npair += n * (n - 1) / 2;
  }
  if (opt & 1) r->kmers = malloc((size_t)U * (k + 1) + 1);
  if (opt & 2) r->pos = malloc(sizeof(int) * 2 * (size_t)npos + 4);
  if (opt & 4) r->pairs = malloc(sizeof(int) * 3 * (size_t)npair + 4);
  if (opt & 8) r->counts = malloc(sizeof(int) * (size_t)U + 4);
  long i = 0, a = 0, b = 0;
  for (khiter_t it = kh_begin(hash); it != kh_end(hash); ++it) {
    if (!kh_exist(hash, it)) continue;
    kmer_pos_t kv = kh_val(hash, it);
    if (opt & 1) decode_kmer(r->kmers + (size_t)i * (k + 1), k, kv.kmer);
    if (opt & 8) r->counts[i] = (int)kv.v.n;
    ++i;
    for (size_t j = 0; j < kv.v.n; ++j) {
      if (opt & 2) { r->pos[a++] = (int)i; r->pos[a++] = kv.v.a[j]; }
      if (opt & 4)
        for (size_t m = j + 1; m < kv.v.n; ++m) {
          r->pairs[b++] = (int)i; r->pairs[b++] = kv.v.a[j]; r->pairs[b++] = kv.v.a[m];
        }
    }
  }
  if (opt & 1) r->n_kmers = U;
  if (opt & 2) r->n_pos = npos;
  if (opt & 4) r->n_pairs = npair;
  if (opt & 8) r->n_counts = U;
  return 0;
}

/* The same bucket walk, streamed in chunks so a full-size pair.pos (config 4: ~7e8 rows, 8 GB)
 * can be digested without materialising it.  opt = 2 (pos rows, 2 ints) or 4 (pair rows, 3
 * ints).  st[0..4] = {bucket, label i of that bucket, j, m, entered}: zero it before the first
 * call.  Writes at most cap rows into out and returns the number written (0 = walk finished). */
long ref_rows_chunk(void *h, unsigned opt, long *st, int *out, long cap) {
  khash_t(kmer_h) *hash = ((khash_ptr *)h)->hash;
  long it = st[0], i = st[1], j = st[2], m = st[3], entered = st[4], b = 0;
  while (it < (long)kh_end(hash) && b < cap) {
    if (!kh_exist(hash, (khiter_t)it)) { ++it; continue; }
    const kmer_pos_t *kv = &kh_val(hash, (khiter_t)it);
    long n = (long)kv->v.n;
    if (!entered) { ++i; j = 0; m = 1; entered = 1; }
    if (opt == 2) {
      for (; j < n && b < cap; ++j, ++b) { out[2 * b] = (int)i; out[2 * b + 1] = kv->v.a[j]; }
      if (j >= n) { ++it; entered = 0; }
    } else {
      while (j < n && b < cap) {
        for (; m < n && b < cap; ++m, ++b) {
          out[3 * b] = (int)i; out[3 * b + 1] = kv->v.a[j]; out[3 * b + 2] = kv->v.a[m];
        }
        if (m >= n) { ++j; m = j + 1; }
      }
      if (j >= n) { ++it; entered = 0; }
    }
  }
  st[0] = it; st[1] = i; st[2] = j; st[3] = m; st[4] = entered;
  return b;
}

/* sum C(n,2), max n and N over the live buckets (sizes of the streamed walk) */
void ref_totals(void *h, long *n_pos, long *n_pairs, long *max_n) {
  khash_t(kmer_h) *hash = ((khash_ptr *)h)->hash;
  long np = 0, pp = 0, mx = 0;
  for (khiter_t it = kh_begin(hash); it != kh_end(hash); ++it) {
    if (!kh_exist(hash, it)) continue;
    long n = (long)kh_val(hash, it).v.n;
    np += n; pp += n * (n - 1) / 2; if (n > mx) mx = n;
  }
  *n_pos = np; *n_pairs = pp; *max_n = mx;
}

/* seq.kmer.pos: returns 2 x n rows (i_end, j_start), column-major, as the R matrix data. */
int ref_query(void *h, const char *seq, int k, long *n_rows, int **rows) {
  if ((long)strlen(seq) <= k || k > 31) return 3;
  kmer_ppos pp = seq_kmer_positions(((khash_ptr *)h)->hash, seq, k);
  *n_rows = (long)(pp.n / 2);
  *rows = pp.a;  /* caller frees with ref_free */
  return 0;
}

/* ---------------------------------------------------------------- count.kmers
 * Per-source counts: a key's kvec holds source_n ints, one per source, and a window adds one
 * to slot `source`.  Returns 1 for a new key, 0 for a known one, -1 when source >= source_n
 * (the reference warning()s and the caller gives up on that sequence). */
static int count_one(khash_t(kmer_h) *hash, uint64_t key, size_t source, size_t source_n) {
  if (source >= source_n) return -1;
  int is_new = 0, ret = 0;
  khiter_t it = kh_get(kmer_h, hash, key);
  if (it == kh_end(hash)) {
    it = kh_put(kmer_h, hash, key, &ret);
    if (it == kh_end(hash)) return -1;
    kmer_pos_t *e = &kh_val(hash, it);
    e->kmer = key;
    e->v.a = calloc(source_n, sizeof(int));
    e->v.n = e->v.m = source_n;
    is_new = 1;
  }
  kh_val(hash, it).v.a[source] += 1;
  return is_new;
}

/* the window walk of seq_to_counts: the same visit order as seq_to_hash (init_kmer restarts
 * after N runs; a restart that reaches the end of the string counts nothing) */
static int count_seq(const char *seq, int k, khash_t(kmer_h) *hash, size_t source,
                     size_t source_n) {
  const uint64_t mask = k < 32 ? (((uint64_t)1) << (2 * k)) - 1 : ~(uint64_t)0;
  uint64_t off = 0;
  size_t i = 0;
  int added = 0, r;
  while (seq[i]) {
    i = init_kmer(seq, i, &off, k);
    if (!seq[i]) break;
    if ((r = count_one(hash, off & mask, source, source_n)) < 0) return r;
    added += r;
    for (; seq[i] && LC(seq[i]) != 'n'; ++i) {
      off = UPDATE_OFFSET(off, seq[i]);
      if ((r = count_one(hash, off & mask, source, source_n)) < 0) return r;
      added += r;
    }
  }
  return added;
}

#define REF_ESRC 4  /* source_n must be larger than 1 and larger than source */
#define REF_EKMM 5  /* mismatch between specified k and that given in the external pointer */

/* h == NULL: a new counts pointer.  Sequences of length <= k are skipped. */
void *ref_count(void *h, const char **seqs, int n, int k, int source, int source_n, int *err) {
  *err = 0;
  if (k < 1 || k > MAX_K) { *err = REF_EK; return 0; }
  if (source_n < 1 || source >= source_n) { *err = REF_ESRC; return 0; }
  khash_ptr *p = (khash_ptr *)h;
  if (!p) {
    p = calloc(1, sizeof(khash_ptr));
    p->k = k;
    p->hash = kh_init(kmer_h);
  }
  if (p->k != k) { *err = REF_EKMM; return h; }
  for (int s = 0; s < n; ++s) {
    if ((long)strlen(seqs[s]) <= k) continue;
    int added = count_seq(seqs[s], k, p->hash, (size_t)source, (size_t)source_n);
    if (added > 0) p->kmer_count += (size_t)added;
  }
  return p;
}

long ref_kmer_count(void *h) { return (long)((khash_ptr *)h)->kmer_count; }
