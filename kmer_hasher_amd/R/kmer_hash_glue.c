/*
 * kmer_hash_glue.c -- R .Call bridge over the libkmhgpu C-ABI (include/kmhgpu.h).
 *
 * Drop-in for the index and read-counting halves of the reference's src/kmer_hash.c: the .Call
 * symbols with the same arities (registration as in src/kmer_hash.c:1205-1224), the same
 * argument validation and error() texts, the same externalptr tag "kmer_hash_250930"
 * (src/kmer_hash.c:22) and return shapes:
 *
 *   make_kmer_h_index(seq, k, do_sort)      src/kmer_hash.c:506-540   -> EXTPTRSXP
 *   kmer_positions(ptr, opt_flag)           src/kmer_hash.c:1054-1147 -> named VECSXP[4]
 *   sequence_kmer_positions(ptr, seq, k)    src/kmer_hash.c:1151-1172 -> INTSXP 2 x H
 *   kmer_pair_pos(ptr_a, ptr_b)             src/kmer_hash.c:1174-1203 -> INTSXP 2 x M (fixed)
 *   count_kmers(hash_ptr, params, seq)      src/kmer_hash.c:548-591   -> EXTPTRSXP (counts)
 *   count_kmers_fastq_sh_rp(ptr, params, f) src/kmer_hash.c:810-857   -> EXTPTRSXP (suffix_hash_n)
 *   seq_kmer_depth_sh(ptr, seq, k)          src/kmer_hash.c:859-879   -> INTSXP counts_n x L
 *   kmer_spectrum_suffix_hash_n(ptr, ...)   src/kmer_hash.c:1010-1039 -> REALSXP
 *
 * Differences, all deliberate: the finaliser frees the whole payload (the reference leaks the
 * 32-B khash_ptr, src/kmer_hash.c:56-66); a freed pointer is detected instead of dereferenced;
 * result sizes are checked against R's int ncol before allocMatrix (the reference overflows at
 * 2^31 pair rows, README.md:80-89).  Results are written by the GPU library straight into the
 * R-allocated INTSXP buffers (one D2H copy, no kvec temporaries).
 *
 * Build (R headers required; R is not installed in the development image, so this file is
 * compiled by R CMD SHLIB on the user's machine -- see INTEGRATION.md):
 *   R CMD SHLIB -o kmer_hash.so kmer_hash_glue.c -I../../include -L.. -lkmhgpu \
 *       -Wl,-rpath,'$ORIGIN/..'
 */
#include <R.h>
#include <Rinternals.h>
#include <R_ext/Rdynload.h>
#include <limits.h>
#include <stdlib.h>
#include <string.h>

#include "kmhgpu.h"

static const char *kmer_hash_tag = "kmer_hash_250930";
static const char *pos_fields[4] = {"kmer", "pos", "pair.pos", "count"};

static void finalise_gpu_index(SEXP ptr_r) {
  kmhg_index *idx = (kmhg_index *)R_ExternalPtrAddr(ptr_r);
  if (idx) {
    kmhg_free(idx);
    R_ClearExternalPtr(ptr_r);
  }
}

/* extract_khash_ptr, src/kmer_hash.c:491-503 (same messages) */
static kmhg_index *gpu_index_of(SEXP ptr_r) {
  if (TYPEOF(ptr_r) != EXTPTRSXP) error("ptr_r should be an external pointer");
  SEXP tag = R_ExternalPtrTag(ptr_r);
  if (TYPEOF(tag) != STRSXP || length(tag) != 1 || strcmp(CHAR(STRING_ELT(tag, 0)), kmer_hash_tag))
    error("External pointer has incorrect tag");
  kmhg_index *idx = (kmhg_index *)R_ExternalPtrAddr(ptr_r);
  if (!idx) error("external pointer has been finalised");
  return idx;
}

SEXP make_kmer_h_index(SEXP seq_r, SEXP k_r, SEXP sort_pos_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r should be a character vector of length at least one");
  if (TYPEOF(k_r) != INTSXP || length(k_r) < 1)
    error("k_r must be an integer vector of length at least one");
  if (TYPEOF(sort_pos_r) != INTSXP || length(k_r) < 1)
    error("sort_pos_r must be an integer vector of length at least one");
  int k = INTEGER(k_r)[0];
  int do_sort = asInteger(sort_pos_r);
  SEXP s = STRING_ELT(seq_r, 0);
  kmhg_index *idx = NULL;
  int rc = kmhg_build(CHAR(s), (size_t)length(s), k, do_sort, &idx);
  if (rc != KMHG_OK) error("%s", kmhg_last_error());
  SEXP tag = PROTECT(allocVector(STRSXP, 1));
  SET_STRING_ELT(tag, 0, mkChar(kmer_hash_tag));
  SEXP ptr = PROTECT(R_MakeExternalPtr(idx, tag, R_NilValue));
  R_RegisterCFinalizerEx(ptr, finalise_gpu_index, TRUE);
  UNPROTECT(2);
  return ptr;
}

SEXP kmer_positions(SEXP ptr_r, SEXP opt_flag_r) {
  kmhg_index *idx = gpu_index_of(ptr_r);
  if (TYPEOF(opt_flag_r) != INTSXP || length(opt_flag_r) != 1)
    error("opt_flag_r should be an integer vector of length 1");
  uint32_t opt = (uint32_t)asInteger(opt_flag_r);
  int64_t nk = 0, np = 0, npp = 0, nc = 0;
  if (kmhg_positions_size(idx, opt, &nk, &np, &npp, &nc) != KMHG_OK)
    error("%s", kmhg_last_error());
  if (np > INT_MAX || npp > INT_MAX || nk > INT_MAX)
    error("result has more than 2^31-1 columns (R matrix limit)");
  kmhg_info info;
  kmhg_index_info(idx, &info);
  SEXP ret = PROTECT(allocVector(VECSXP, 4));
  SEXP nm = PROTECT(allocVector(STRSXP, 4));
  for (int i = 0; i < 4; ++i) SET_STRING_ELT(nm, i, mkChar(pos_fields[i]));
  setAttrib(ret, R_NamesSymbol, nm);
  int *pos = NULL, *pairs = NULL, *counts = NULL;
  char *kmers = NULL;
  if (opt & KMHG_OPT_POS) {
    SET_VECTOR_ELT(ret, 1, allocMatrix(INTSXP, 2, (int)np));
    pos = INTEGER(VECTOR_ELT(ret, 1));
  }
  if (opt & KMHG_OPT_PAIRS) {
    SET_VECTOR_ELT(ret, 2, allocMatrix(INTSXP, 3, (int)npp));
    pairs = INTEGER(VECTOR_ELT(ret, 2));
  }
  if (opt & KMHG_OPT_COUNT) {
    SET_VECTOR_ELT(ret, 3, allocVector(INTSXP, (R_xlen_t)nc));
    counts = INTEGER(VECTOR_ELT(ret, 3));
  }
  if ((opt & KMHG_OPT_KMER) && nk) kmers = (char *)R_alloc((size_t)nk, info.k + 1);
  if (kmhg_positions_fill(idx, opt, kmers, pos, pairs, counts) != KMHG_OK)
    error("%s", kmhg_last_error());
  if (opt & KMHG_OPT_KMER) {
    SET_VECTOR_ELT(ret, 0, allocVector(STRSXP, (R_xlen_t)nk));
    SEXP kr = VECTOR_ELT(ret, 0);
    for (int64_t i = 0; i < nk; ++i)
      SET_STRING_ELT(kr, (R_xlen_t)i, mkChar(kmers + (size_t)i * (info.k + 1)));
  }
  UNPROTECT(2);
  return ret;
}

/* With KMHG_DEVICES=d0,d1,... in the environment, kmhg_query_run splits the query over those
 * GPUs (index replicas peer-copied once, rows filled straight into the R matrix by
 * kmhg_query_fill at each device's row offset): same signature, same result. */
SEXP sequence_kmer_positions(SEXP ptr_r, SEXP seq_r, SEXP k_r) {
  kmhg_index *idx = gpu_index_of(ptr_r);
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) != 1) error("seq_r should be a single sequence");
  if (TYPEOF(k_r) != INTSXP || length(k_r) != 1) error("k should be an integer of length 1");
  int k = INTEGER(k_r)[0];
  SEXP s = STRING_ELT(seq_r, 0);
  kmhg_query *q = NULL;
  int64_t h = 0;
  if (kmhg_query_run(idx, CHAR(s), (size_t)length(s), k, &q, &h) != KMHG_OK)
    error("%s", kmhg_last_error());
  if (h > INT_MAX) {
    kmhg_query_free(q);
    error("result has more than 2^31-1 columns (R matrix limit)");
  }
  SEXP ret = PROTECT(allocMatrix(INTSXP, 2, (int)h));
  int rc = h ? kmhg_query_fill(q, INTEGER(ret)) : KMHG_OK;
  kmhg_query_free(q);
  if (rc != KMHG_OK) error("%s", kmhg_last_error());
  UNPROTECT(1);
  return ret;
}

/* kmer_pair_pos, src/kmer_hash.c:1174-1203 (called by kmer.pairs, kmer_hash.R:30-34): rows
 * (a, b) for the k-mers both indices hold.  The reference walks empty buckets and reads past
 * the end of b's flags (test.R:330 "This crashes"); kmhg_pairs_run defines the intended result
 * and refuses indices of different k. */
SEXP kmer_pair_pos(SEXP ptr_a, SEXP ptr_b) {
  kmhg_index *a = gpu_index_of(ptr_a);
  kmhg_index *b = gpu_index_of(ptr_b);
  kmhg_query *q = NULL;
  int64_t h = 0;
  if (kmhg_pairs_run(a, b, &q, &h) != KMHG_OK) error("%s", kmhg_last_error());
  if (h > INT_MAX) {
    kmhg_query_free(q);
    error("result has more than 2^31-1 columns (R matrix limit)");
  }
  SEXP ret = PROTECT(allocMatrix(INTSXP, 2, (int)h));
  int rc = h ? kmhg_query_fill(q, INTEGER(ret)) : KMHG_OK;
  kmhg_query_free(q);
  if (rc != KMHG_OK) error("%s", kmhg_last_error());
  UNPROTECT(1);
  return ret;
}

/* count_kmers, src/kmer_hash.c:548-591 (count.kmers, kmer_hash.R:43-46): per-source counts of
 * every k-mer of a character vector, added to hash_ptr_r or to a new counts pointer (same tag,
 * so kmer.pos / seq.kmer.pos read it, test.R:340-343).  Validation order and texts as the
 * reference; kmhg_count also refuses a position index and a different source_n, where the
 * reference would write past the end of a k-mer's vector. */
SEXP count_kmers(SEXP hash_ptr_r, SEXP params_r, SEXP seq_r) {
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) < 1)
    error("seq_r should be a character vector of length at least one");
  if (TYPEOF(params_r) != INTSXP || length(params_r) != 3)
    error("k_r must be an integer vector of length 3");
  const int *params = INTEGER(params_r);
  const int k = params[0], source = params[1], source_n = params[2];
  if (k < 1 || k > 32) error("k must be a positive integer less than 1+MAX_K");
  if (source_n < 1 || source >= source_n)
    error("source_n must be larger than 1 and larger than source");
  kmhg_index *idx = NULL;
  if (hash_ptr_r != R_NilValue) {
    if (TYPEOF(hash_ptr_r) != EXTPTRSXP) error("failed to extract kmer_hash from external pointer");
    SEXP tag = R_ExternalPtrTag(hash_ptr_r);
    if (TYPEOF(tag) != STRSXP || length(tag) != 1 ||
        strcmp(CHAR(STRING_ELT(tag, 0)), kmer_hash_tag))
      error("failed to extract kmer_hash from external pointer");
    idx = (kmhg_index *)R_ExternalPtrAddr(hash_ptr_r);
    if (!idx) error("failed to extract kmer_hash from external pointer");
  }
  const R_xlen_t n = XLENGTH(seq_r);
  const char **seqs = (const char **)R_alloc((size_t)n, sizeof(char *));
  size_t *lens = (size_t *)R_alloc((size_t)n, sizeof(size_t));
  for (R_xlen_t i = 0; i < n; ++i) {
    SEXP e = STRING_ELT(seq_r, i);
    seqs[i] = CHAR(e);
    lens[i] = (size_t)length(e);
  }
  kmhg_index *out = idx;
  if (kmhg_count(&out, seqs, lens, (int64_t)n, k, source, source_n) != KMHG_OK)
    error("%s", kmhg_last_error());
  if (source < 0) warning("source (%d) equal to or larger than source_n (%d)", source, source_n);
  if (idx) return hash_ptr_r;
  SEXP tag = PROTECT(allocVector(STRSXP, 1));
  SET_STRING_ELT(tag, 0, mkChar(kmer_hash_tag));
  SEXP ptr = PROTECT(R_MakeExternalPtr(out, tag, R_NilValue));
  R_RegisterCFinalizerEx(ptr, finalise_gpu_index, TRUE);
  UNPROTECT(2);
  return ptr;
}

/* ---- suffix_hash_n (read counting) ------------------------------------------------------
 * Same tag as the reference's suffix hashes (src/kmer_hash.c:25), so pointers made here are
 * refused by kmer.pos exactly as the reference refuses a suffix_hash_n. */
static const char *suffix_hash_n_tag = "suffix_hash_n_250930";

/* extract_ext_ptr(ptr, suffix_hash_n_tag), src/kmer_hash.c:41-52: NULL for anything else */
static kmhg_index *gpu_sh_of(SEXP ptr_r) {
  if (TYPEOF(ptr_r) != EXTPTRSXP) return NULL;
  SEXP tag = R_ExternalPtrTag(ptr_r);
  if (TYPEOF(tag) != STRSXP || length(tag) != 1 ||
      strcmp(CHAR(STRING_ELT(tag, 0)), suffix_hash_n_tag))
    return NULL;
  return (kmhg_index *)R_ExternalPtrAddr(ptr_r);
}

static int gpu_sh_sources(kmhg_index *sh) {
  kmhg_info info;
  if (kmhg_index_info(sh, &info) != KMHG_OK) error("%s", kmhg_last_error());
  return info.sources;
}

/* count_kmers_fastq_sh_rp, src/kmer_hash.c:810-857 (count.kmers.fq.sh.rp, kmer_hash.R:70-73):
 * params = (k, prefix_bits, min_q, thread_n, max_reads, max_mem, source_n, source); the
 * canonical k-mers of the FASTA/FASTQ file the quality iterator accepts, counted on the GPU
 * into entry `source` of a new or the given suffix hash.  Validation order and texts as the
 * reference (kmhg_sh_count_fastq repeats the k / source checks). */
SEXP count_kmers_fastq_sh_rp(SEXP hash_ptr_r, SEXP params_r, SEXP fq_file_r) {
  if (TYPEOF(fq_file_r) != STRSXP || length(fq_file_r) != 1)
    error("fq_file should be a character vector of length at least one");
  if (TYPEOF(params_r) != INTSXP || length(params_r) != 8)
    error("k_r must be an integer vector of length 6 (k, prefix_bits, min_q, thread_n, "
          "max_reads, max_mem, source_n, source");
  const char *fq_file = CHAR(STRING_ELT(fq_file_r, 0));
  kmhg_index *sh = gpu_sh_of(hash_ptr_r);
  kmhg_index *out = sh;
  if (kmhg_sh_count_fastq(&out, fq_file, (const int32_t *)INTEGER(params_r)) != KMHG_OK)
    error("%s", kmhg_last_error());
  if (sh) return hash_ptr_r;
  SEXP tag = PROTECT(allocVector(STRSXP, 1));
  SET_STRING_ELT(tag, 0, mkChar(suffix_hash_n_tag));
  SEXP ptr = PROTECT(R_MakeExternalPtr(out, tag, R_NilValue));
  R_RegisterCFinalizerEx(ptr, finalise_gpu_index, TRUE);
  UNPROTECT(2);
  return ptr;
}

/* seq_kmer_depth_sh, src/kmer_hash.c:859-879 (seq.kmer.depth.sh, kmer_hash.R:75-78):
 * counts_n x L int matrix of the canonical k-mer counts along seq, written by the GPU. */
SEXP seq_kmer_depth_sh(SEXP hash_ptr_r, SEXP seq_r, SEXP k_r) {
  kmhg_index *sh = gpu_sh_of(hash_ptr_r);
  if (!sh) error("unable to obtain suffix_hash_n from external pointer");
  if (TYPEOF(k_r) != INTSXP || length(k_r) != 1) error("k_r should be a single integer");
  const int k = asInteger(k_r);
  if (TYPEOF(seq_r) != STRSXP || length(seq_r) != 1)
    error("seq_r should be a character vector of length 1");
  SEXP s = STRING_ELT(seq_r, 0);
  const size_t L = (size_t)length(s);
  SEXP counts_r = PROTECT(allocMatrix(INTSXP, gpu_sh_sources(sh), (int)L));
  if (kmhg_sh_depth(sh, CHAR(s), L, k, INTEGER(counts_r)) != KMHG_OK) {
    UNPROTECT(1);
    error("Receieved error from seq_kmer_counts");
  }
  UNPROTECT(1);
  return counts_r;
}

/* kmer_spectrum_suffix_hash_n, src/kmer_hash.c:1010-1039 (kmer.spec.sh.n, kmer_hash.R:88-91) */
SEXP kmer_spectrum_suffix_hash_n(SEXP hash_ptr_r, SEXP max_count_r, SEXP comb_r,
                                 SEXP comb_inner_r, SEXP source_min_r) {
  kmhg_index *sh = gpu_sh_of(hash_ptr_r);
  if (!sh) error("unable to obtain suffix_hash_n from external pointer");
  if (TYPEOF(max_count_r) != INTSXP || length(max_count_r) != 1)
    error("max_count_r should be a single integer");
  if (TYPEOF(comb_r) != INTSXP || length(comb_r) < 1)
    error("comb_r should be an integer vector of length > 0");
  if (TYPEOF(comb_inner_r) != INTSXP || length(comb_inner_r) != length(comb_r))
    error("comb_inner_r should be an integer vector of the same length as comb_r");
  const int S = gpu_sh_sources(sh);
  if (TYPEOF(source_min_r) != INTSXP || length(source_min_r) != S)
    error("source_min_r should be an integer vector of length sh->counts_n");
  const int max_count = asInteger(max_count_r);
  if (max_count < 0) error("max_count must be >= 0");
  const int comb_n = length(comb_r);
  SEXP counts_r = PROTECT(allocMatrix(REALSXP, comb_n * S, max_count + 1));
  int status = 1;
  if (kmhg_sh_spectrum(sh, max_count, INTEGER(comb_r), INTEGER(comb_inner_r), comb_n,
                       INTEGER(source_min_r), S, REAL(counts_r), &status) != KMHG_OK) {
    UNPROTECT(1);
    error("%s", kmhg_last_error());
  }
  if (status < 0) Rprintf("sh_count_spectrum_nc returned an error: %d\n", status);
  UNPROTECT(1);
  return counts_r;
}

/* Not in the reference: choose the kmer.pos k-mer order of an index, "first" (first
 * occurrence, the default) or "khash" (the reference's own bucket order, byte-identical
 * output).  KMHG_ROW_ORDER=khash in the environment sets the default for new indices. */
SEXP kmer_row_order(SEXP ptr_r, SEXP order_r) {
  kmhg_index *idx = gpu_index_of(ptr_r);
  if (TYPEOF(order_r) != STRSXP || length(order_r) != 1)
    error("order should be \"first\" or \"khash\"");
  const char *o = CHAR(STRING_ELT(order_r, 0));
  int code = !strcmp(o, "khash") ? KMHG_ORDER_KHASH : (!strcmp(o, "first") ? KMHG_ORDER_FIRST : -1);
  if (code < 0) error("order should be \"first\" or \"khash\"");
  if (kmhg_set_row_order(idx, code) != KMHG_OK) error("%s", kmhg_last_error());
  return R_NilValue;
}

static const R_CallMethodDef gpu_call_methods[] = {
    {"make_kmer_h_index", (DL_FUNC)&make_kmer_h_index, 3},
    {"kmer_positions", (DL_FUNC)&kmer_positions, 2},
    {"sequence_kmer_positions", (DL_FUNC)&sequence_kmer_positions, 3},
    {"kmer_pair_pos", (DL_FUNC)&kmer_pair_pos, 2},
    {"count_kmers", (DL_FUNC)&count_kmers, 3},
    {"count_kmers_fastq_sh_rp", (DL_FUNC)&count_kmers_fastq_sh_rp, 3},
    {"seq_kmer_depth_sh", (DL_FUNC)&seq_kmer_depth_sh, 3},
    {"kmer_spectrum_suffix_hash_n", (DL_FUNC)&kmer_spectrum_suffix_hash_n, 5},
    {"kmer_row_order", (DL_FUNC)&kmer_row_order, 2},
    {NULL, NULL, 0}};

void R_init_kmer_hash(DllInfo *info) { R_registerRoutines(info, NULL, gpu_call_methods, NULL, NULL); }
