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

/* seq.kmer.pos: returns 2 x n rows (i_end, j_start), column-major, as the R matrix data. */
int ref_query(void *h, const char *seq, int k, long *n_rows, int **rows) {
  if ((long)strlen(seq) <= k || k > 31) return 3;
  kmer_ppos pp = seq_kmer_positions(((khash_ptr *)h)->hash, seq, k);
  *n_rows = (long)(pp.n / 2);
  *rows = pp.a;  /* caller frees with ref_free */
  return 0;
}
