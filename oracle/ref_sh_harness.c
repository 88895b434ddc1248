/*
 * oracle/ref_sh_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never the measured path).
 *
 * R-free driver over the reference's own k-mer counting core (src/suffix_hash.c,
 * src/kmer_reader.c, src/kmer_util.c, src/thread_queue.c + klib's kseq/khash, zlib, pthreads),
 * compiled from the sources where they lie under /root/reference/src by oracle/Makefile into
 * oracle/_ref/libkmh_ref_sh.so.  The .Call wrappers live in src/kmer_hash.c, which needs R
 * headers, so they are restated here:
 *
 *   ref_sh_count_fastq <- count_kmers_fastq_sh_rp  (reference src/kmer_hash.c:810-857)
 *                         init_kmer_reader_pool / _sh + join (src/kmer_reader.c:78-147)
 *   ref_sh_depth       <- seq_kmer_depth_sh        (reference src/kmer_hash.c:859-879)
 *                         seq_kmer_counts           (src/kmer_reader.c:155-193), unchanged
 *   ref_sh_spectrum    <- kmer_spectrum_suffix_hash_n (src/kmer_hash.c:1010-1039)
 *                         sh_count_spectrum_nc      (src/suffix_hash.c:338-421), unchanged
 *   ref_sh_dump        walks every prefix table (khash iteration) -> (key, counts) rows
 *   ref_sh_free        <- finalise_suffix_hash_n_ptr (src/kmer_hash.c:85-95)
 */
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include "kmer_util.h"
#include "kmer_reader.h"

/* count_kmers_fastq_sh_rp with the R argument checks already done by the caller; sh_in = NULL
 * creates a new suffix_hash_n.  Returns the (possibly new) suffix_hash_n. */
void *ref_sh_count_fastq(void *sh_in, const char *path, int k, int prefix_bits, int min_q,
                         int thread_n, long max_reads, int source_n, int source) {
  kmer_reader_pool krp;
  unsigned char mq = (unsigned char)('!' + (unsigned char)min_q);
  size_t max_mem = (size_t)1 << 30;
  suffix_hash_n *sh = (suffix_hash_n *)sh_in;
  if (!sh)
    sh = init_kmer_reader_pool(&krp, path, k, (uint32_t)prefix_bits, max_mem, (uint32_t)thread_n,
                               mq, (size_t)max_reads, (uint32_t)source_n, (uint32_t)source);
  else
    sh = init_kmer_reader_pool_sh(&krp, path, k, sh, max_mem, (uint32_t)thread_n, mq,
                                  (size_t)max_reads, (uint32_t)source);
  join_kmer_reader_pool(&krp);
  free_kmer_reader_pool(&krp);
  return sh;
}

int ref_sh_counts_n(void *h) { return (int)((suffix_hash_n *)h)->counts_n; }

/* number of distinct k-mers held */
long ref_sh_size(void *h) {
  suffix_hash_n *sh = (suffix_hash_n *)h;
  long n = 0;
  for (size_t i = 0; i < sh->prefix_n; ++i) {
    if (!sh->prefixes[i]) continue;
    /* every khash_t(kcount*) starts with n_buckets, size, ... (klib's struct layout) */
    n += (long)((khash_t(kcount) *)sh->prefixes[i])->size;
  }
  return n;
}

/* (key, counts[counts_n]) of every k-mer, prefix tables in order, khash bucket order inside */
long ref_sh_dump(void *h, uint64_t *keys, int32_t *counts) {
  suffix_hash_n *sh = (suffix_hash_n *)h;
  const int cn = (int)sh->counts_n;
  long r = 0;
  for (size_t i = 0; i < sh->prefix_n; ++i) {
    void *hp = sh->prefixes[i];
    if (!hp) continue;
    khint_t nb = ((khash_t(kcount) *)hp)->n_buckets;
    for (khint_t b = 0; b < nb; ++b) {
      const uint32_t *val = 0;
      uint32_t suffix = 0;
      switch (cn) {
        case 1: { khash_t(kcount) *t = hp; if (!kh_exist(t, b)) continue;
                  suffix = kh_key(t, b); val = &kh_value(t, b); break; }
        case 2: { khash_t(kcount_2) *t = hp; if (!kh_exist(t, b)) continue;
                  suffix = kh_key(t, b); val = kh_value(t, b).n; break; }
        case 3: { khash_t(kcount_3) *t = hp; if (!kh_exist(t, b)) continue;
                  suffix = kh_key(t, b); val = kh_value(t, b).n; break; }
        default: { khash_t(kcount_4) *t = hp; if (!kh_exist(t, b)) continue;
                   suffix = kh_key(t, b); val = kh_value(t, b).n; break; }
      }
      keys[r] = ((uint64_t)i << sh->suffix_bits) | suffix;
      for (int j = 0; j < cn; ++j) counts[r * cn + j] = (int32_t)val[j];
      ++r;
    }
  }
  return r;
}

/* seq_kmer_depth_sh: counts is counts_n x seq_l int32 (column-major, R layout) */
int ref_sh_depth(void *h, const char *seq, long seq_l, int k, int32_t *counts) {
  suffix_hash_n *sh = (suffix_hash_n *)h;
  return seq_kmer_counts(seq, (size_t)seq_l, counts, sh, k);
}

/* kmer_spectrum_suffix_hash_n: counts is (comb_n * counts_n) x (max_count + 1) doubles */
int ref_sh_spectrum(void *h, int max_count, const int32_t *comb, const int32_t *comb_inner,
                    int comb_n, const int32_t *source_min, double *counts) {
  suffix_hash_n *sh = (suffix_hash_n *)h;
  uint32_t counts_l = (uint32_t)(max_count + 1);
  memset(counts, 0, sizeof(double) * (size_t)comb_n * sh->counts_n * counts_l);
  return sh_count_spectrum_nc(sh, counts, (uint32_t)comb_n * sh->counts_n * counts_l,
                              (uint32_t)max_count, (uint32_t *)comb, (uint32_t *)comb_inner,
                              (uint32_t)comb_n, (uint32_t *)source_min);
}

void ref_sh_free(void *h) {
  suffix_hash_n *sh = (suffix_hash_n *)h;
  if (!sh) return;
  free_suffix_hash_n(sh);
  free(sh);
}
