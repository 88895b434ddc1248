/*
 * kmhgpu.h -- C-ABI of the MI355X k-mer position index (libkmhgpu.so).
 *
 * Drop-in boundary for the hot path of lmjakt/kmer_hasheR.  Plain pointers and sizes only; no
 * torch or HIP types in the signatures (streams are passed as `void*` = hipStream_t, NULL = the
 * HIP null stream; host-pointer entry points run on a library-owned stream and return synced).  Every function returns KMHG_OK (0) or an error code; the message is
 * in kmhg_last_error() (thread-local).  Where the reference raises an R error() the message is
 * the reference's own text.
 *
 * Reference interfaces replaced (paths relative to the reference checkout):
 *   kmhg_build / kmhg_build_device
 *        <- .Call("make_kmer_h_index", seq, k, do.sort)      src/kmer_hash.c:506-540
 *           (+ seq_to_hash, src/kmer_pos.c:66-98; sort_kmer_pos, src/kmer_pos.c:21-33)
 *   kmhg_free
 *        <- finalise_khash_ptr (externalptr finaliser)       src/kmer_hash.c:56-66
 *           (+ clear_kmer_h, src/kmer_pos.c:10-19)
 *   kmhg_positions_size / kmhg_positions_fill / kmhg_positions_fill_device
 *        <- .Call("kmer_positions", ptr, opt.flag)           src/kmer_hash.c:1054-1147
 *           (+ kmer_seq decode, src/kmer_hash.c:123-133)
 *   kmhg_query_run / kmhg_query_run_device / kmhg_query_fill / kmhg_query_rows_device
 *        <- .Call("sequence_kmer_positions", ptr, seq, k)    src/kmer_hash.c:1151-1172
 *           (+ seq_kmer_positions, src/kmer_pos.c:110-136)
 *   kmhg_count / kmhg_count_device
 *        <- .Call("count_kmers", hash.ptr, params, seq)       src/kmer_hash.c:548-591
 *   kmhg_build_device_part / kmhg_part_info / kmhg_part_export
 *        <- the owner-computes partition of the reader pool  src/kmer_reader.c:28-39, 101-108
 *           (multi-GPU make.kmer.hash; no single reference entry point)
 *   KMHG_DEVICES=d0,d1,... (environment): kmhg_query_run splits seq.kmer.pos over those devices
 *           (index peer-copied once per device, rows copied straight into the caller's buffer)
 *   registration of the three symbols with arities 3/2/3    src/kmer_hash.c:1205-1224
 *           is done by the R glue (kmer_hasher_amd/R/kmer_hash_glue.c) over this ABI.
 *
 * Output layouts are the R matrices' column-major data, exactly what the reference memcpy's:
 *   pos      2 x N int32   (i, pos)      i = 1-based k-mer index, pos = 1-based window start
 *   pair.pos 3 x P int32   (i, x, y)     x < y, j-outer / k-inner inside a k-mer
 *   count    N_kmers int32
 *   kmer     N_kmers strings of k chars, each followed by a NUL (stride k+1)
 *   query    2 x H int32   (i, j)        i = 1-based END of the query window, j = index pos
 * K-mer order (the `i` labels): by default distinct k-mers ranked by first occurrence; the sets,
 * counts, position lists and pairs per k-mer equal the reference's, and seq.kmer.pos rows are
 * identical including order (DESIGN.md "Parity").  With KMHG_ORDER_KHASH (kmhg_set_row_order, or
 * KMHG_ROW_ORDER=khash in the environment when the index is built) kmer.pos is labelled in the
 * reference's own khash bucket order, i.e. byte-identical to its output.
 */
#ifndef KMHGPU_H
#define KMHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KMHG_OK 0
#define KMHG_EINVAL 1     /* argument rejected (message = the reference's R error text) */
#define KMHG_ENOMEM 2     /* device or host allocation failed */
#define KMHG_EDEVICE 3    /* HIP runtime error */
#define KMHG_EOVERFLOW 4  /* result exceeds int32 / R matrix limits */

/* opt.flag bits of kmer.pos (src/kmer_hash.c:17; src/kmer_pos.h:8-12) */
#define KMHG_OPT_KMER 1u
#define KMHG_OPT_POS 2u
#define KMHG_OPT_PAIRS 4u
#define KMHG_OPT_COUNT 8u

/* kmer.pos k-mer (row) order */
#define KMHG_ORDER_FIRST 0   /* ranked by first occurrence (default) */
#define KMHG_ORDER_KHASH 1   /* the reference's khash 0.2.8 bucket order, src/kmer_hash.c:1096-1124 */

typedef struct kmhg_index kmhg_index;
typedef struct kmhg_query kmhg_query;

typedef struct {
  int32_t k;             /* index k-mer length */
  int32_t device;        /* HIP device ordinal holding the index */
  int64_t seq_len;       /* L */
  int64_t n_kmers;       /* distinct k-mers (kh_size) */
  int64_t n_positions;   /* windows indexed (rows of kmer.pos $pos) */
  int64_t n_pairs;       /* sum C(n,2) (rows of kmer.pos $pair.pos) */
  int64_t max_count;     /* largest position list */
  int64_t table_slots;   /* hash-table capacity */
  int64_t device_bytes;  /* device memory held by the index */
  int32_t sources;       /* counts index (count.kmers): source_n; 0 for a position index */
  int32_t kind;          /* 0 position index, 1 counts index, 2 suffix hash (canonical counts) */
  int64_t kmer_count;    /* khash_ptr.kmer_count: distinct k-mers added (both kinds) */
  int32_t build;         /* KMHG_BUILD_*: how the table was built (0 = imported / assembled) */
  int32_t fallback;      /* 1: a partitioned build was rebuilt with the global-atomic build (a
                            bucket's LDS table overflowed or its stream failed the order check) */
} kmhg_info;

/* kmhg_info.build */
#define KMHG_BUILD_GLOBAL 1              /* global-atomic insert (KMHG_BUILD=v1, or the fallback) */
#define KMHG_BUILD_PARTITIONED 2         /* radix partition + per-bucket LDS tables (default) */
#define KMHG_BUILD_PARTITIONED_BALLOT 3  /* the same with ballot ranks: the device failed the
                                            LDS lane-order self-check */

const char *kmhg_last_error(void);
int kmhg_version(void);

/* make.kmer.hash.  seq: host chars, L = its length (the sequence ends at L or at the first NUL,
 * as a C string does).  Errors: "k must be a positive integer less than 1+MAX_K",
 * "the length of the sequence must be at least k".  do_sort is accepted for API identity; the
 * engine always stores positions ascending, which is what sort_kmer_pos would produce. */
int kmhg_build(const char *seq, size_t L, int k, int do_sort, kmhg_index **out);
/* Same, for a device-resident sequence (no NULs assumed) on `stream`.  Asynchronous: it returns
 * once the build is queued, so back-to-back builds pipeline host and device work.  The first
 * call that reads the index (info, kmer.pos, a query, export, kmhg_index_wait) waits for it;
 * until then `d_seq` must stay valid and unmodified (the overflow fallback re-reads it).
 * kmhg_free of an index never used does not wait. */
int kmhg_build_device(const void *d_seq, size_t L, int k, int do_sort, void *stream,
                      kmhg_index **out);
/* Wait for an asynchronous build to finish (no-op for a finished index). */
int kmhg_index_wait(kmhg_index *idx);
int kmhg_free(kmhg_index *idx);
int kmhg_index_info(const kmhg_index *idx, kmhg_info *info);

/* Row order of later kmer.pos calls on this index (KMHG_ORDER_*).  The khash order is replayed
 * on the host from the distinct keys (src/khash.h:230-348 semantics), once per index. */
int kmhg_set_row_order(kmhg_index *idx, int order);
int kmhg_get_row_order(const kmhg_index *idx, int *order);
/* The host replay itself: order[r] = index (into keys) of the r-th live khash bucket after
 * kh_put of the n distinct keys in the given order.  Host-only, no device work. */
int kmhg_khash_order(const uint64_t *keys, int64_t n, uint32_t *order);

/* kmer.pos, two-phase: sizes first so the caller (R's allocMatrix) can allocate, then fill.
 * Unset opt bits give 0 sizes and the corresponding pointers may be NULL. */
int kmhg_positions_size(kmhg_index *idx, uint32_t opt, int64_t *n_kmers, int64_t *n_pos_rows,
                        int64_t *n_pair_rows, int64_t *n_counts);
int kmhg_positions_fill(kmhg_index *idx, uint32_t opt, char *kmers, int32_t *pos,
                        int32_t *pairs, int32_t *counts);
int kmhg_positions_fill_device(kmhg_index *idx, uint32_t opt, char *d_kmers, int32_t *d_pos,
                               int32_t *d_pairs, int32_t *d_counts, void *stream);

/* seq.kmer.pos.  Errors: "the sequence should be longer than k and k should not be longer than
 * 31" (also for k < 1, where the reference's behaviour is undefined). */
int kmhg_query_run(kmhg_index *idx, const char *seq, size_t L, int k, kmhg_query **q,
                   int64_t *n_rows);
int kmhg_query_run_device(kmhg_index *idx, const void *d_seq, size_t L, int k, void *stream,
                          kmhg_query **q, int64_t *n_rows);
/* Windows [w_begin, w_end) (0-based window starts, w_end <= L - k + 1) of a device-resident
 * query: the unit of the multi-GPU query shard.  Window validity still sees the whole sequence
 * (the char before a window, the true sequence end), so consecutive ranges concatenate to the
 * unsharded result row for row. */
int kmhg_query_run_device_range(kmhg_index *idx, const void *d_seq, size_t L, int k,
                                int64_t w_begin, int64_t w_end, void *stream, kmhg_query **q,
                                int64_t *n_rows);
/* The same range query with its rows left as diagonal runs (the format of kmhg_rows_runs, the
 * sharded gather's): made from the query's per-window records, the rows are never written.
 * *n_runs >= 0: the query holds n_runs runs (kmhg_query_runs_device, 3 int32 each; rows
 * through kmhg_runs_expand); *n_runs = -1: runs would not be smaller and it holds the rows as
 * kmhg_query_run_device_range's do.  The rows / fill / copy entries refuse a runs query. */
int kmhg_query_run_device_range_runs(kmhg_index *idx, const void *d_seq, size_t L, int k,
                                     int64_t w_begin, int64_t w_end, void *stream,
                                     kmhg_query **q, int64_t *n_rows, int64_t *n_runs);
int kmhg_query_runs_device(kmhg_query *q, const int32_t **d_runs);   /* owned by q */
/* seq.kmer.pos over a PART of an owner-computes build (kmhg_build_device_part), without
 * assembling the parts: every window of the query is hashed and only the windows whose k-mer
 * this part owns are probed, so the rows are those windows' rows, in window order.  With one
 * such query per part (one per rank), kmhg_merge_part_rows on the root interleaves them into
 * exactly the unsharded seq.kmer.pos rows (src/kmer_pos.c:110-136 behind
 * src/kmer_hash.c:1151-1172; the partition is the reference reader pool's,
 * src/kmer_reader.c:28-39).  kmhg_query_tile_offsets writes the query's n_tiles + 1 per-tile row
 * offsets (tiles of 2048 windows; [n_tiles] = n_rows) to device memory on `stream`. */
int kmhg_query_run_device_part(kmhg_index *part, const void *d_seq, size_t L, int k,
                               void *stream, kmhg_query **q, int64_t *n_rows);
int kmhg_query_tile_offsets(kmhg_query *q, uint64_t *d_out, int64_t *n_tiles, void *stream);
/* The root's merge: n_parts segments of (i, j) rows in device memory, part r's at
 * d_rows + 2 * d_seg_base[r] int32, with its tile offsets at d_tile_off + r * (n_tiles + 1);
 * writes the sum of their rows to d_out ordered by window end i, then j, on `stream`. */
int kmhg_merge_part_rows(const void *d_rows, const uint64_t *d_seg_base,
                         const uint64_t *d_tile_off, int n_parts, int64_t n_tiles, int k,
                         int64_t w0, void *d_out, void *stream);
/* A device sequence as it crosses xGMI (C1 scatter / broadcast of the multi-GPU query and of
 * the owner-computes build): what the reference reads of a char -- its 2-bit code (c >> 1) & 3
 * and its N test, src/kmer_pos.c:81-83 -- as 16 chars per u32 code word and u16 N-flag word
 * (ceil(L / 16) of each; 6 B per 16 chars).  kmhg_seq_unpack writes chars [a, b) back ("ACTG"
 * by code, or 'N', which every entry point reads as the original) from the words held at
 * d_code / d_nbit starting with word `word0` (<= a / 16), on `stream`. */
int kmhg_seq_pack(const void *d_seq, int64_t L, uint32_t *d_code, uint16_t *d_nbit,
                  void *stream);
int kmhg_seq_unpack(const uint32_t *d_code, const uint16_t *d_nbit, int64_t word0, int64_t a,
                    int64_t b, void *d_seq, void *stream);
/* The sharded query's row gather format (src/kmer_pos.c:110-136's rows, moved between ranks):
 * n_rows (i, j) int32 rows in device memory as diagonal runs -- maximal stretches of rows
 * (i, j), (i + 1, j + 1), ... -- each run 3 int32 {its first row's index, i, j}.
 * kmhg_rows_runs counts the runs (*n_runs; it waits for `stream`) and writes them to d_runs when
 * *n_runs <= cap_runs (else nothing: the caller sends rows); kmhg_runs_expand writes the n_rows
 * rows back to d_rows on `stream`.  n_rows < 2^31. */
/* n_rows (i, j) rows in device memory into host memory (2 * n_rows int32, e.g. an R matrix or
 * one rank's slice of a node-shared matrix), as kmhg_query_fill copies a query's rows: from
 * 512 K rows on as diagonal runs over PCIe, expanded by host threads.  Synchronous. */
int kmhg_rows_to_host(const void *d_rows, int64_t n_rows, int32_t *rows, void *stream);
int kmhg_rows_runs(const void *d_rows, int64_t n_rows, void *d_runs, int64_t cap_runs,
                   int64_t *n_runs, void *stream);
int kmhg_runs_expand(const void *d_runs, int64_t n_runs, int64_t n_rows, void *d_rows,
                     void *stream);
int kmhg_query_fill(kmhg_query *q, int32_t *rows);               /* host, 2 * n_rows int32 */
int kmhg_query_rows_device(kmhg_query *q, const int32_t **d_rows); /* owned by q */
/* Device-to-device copy of the 2 x n_rows int32 rows into caller memory on `stream`. */
int kmhg_query_copy_device(kmhg_query *q, void *d_dst, void *stream);
int kmhg_query_free(kmhg_query *q);

/* kmer.pairs <- .Call("kmer_pair_pos", ptr_a, ptr_b)           src/kmer_hash.c:1174-1203
 * Rows (a, b) = (position in index a, position in index b) for every k-mer both indices hold:
 * a's k-mers in a's kmer.pos row order (kmhg_set_row_order), a's positions outer, b's inner;
 * the result is a query handle holding 2 x n_rows int32, read like a seq.kmer.pos result.
 * Defined where the reference is broken: only a's live k-mers are visited (the reference reads
 * empty buckets and calls kh_exist(b, kh_end(b)), src/kmer_hash.c:1182-1185; test.R:330 "This
 * crashes"), and both indices must have the same k ("the two indices must have the same k"). */
int kmhg_pairs_run(kmhg_index *a, kmhg_index *b, kmhg_query **q, int64_t *n_rows);
int kmhg_pairs_run_device(kmhg_index *a, kmhg_index *b, void *stream, kmhg_query **q,
                          int64_t *n_rows);

/* count.kmers <- .Call("count_kmers", hash.ptr, c(k, source, source_n), seq)
 *                                                            src/kmer_hash.c:548-591
 *        (+ seq_to_counts :220-251, kmer_count_insert :185-208)
 * Per-source k-mer counts: every valid window (the window walk of make.kmer.hash) of every
 * sequence adds one to entry `source` of its k-mer's vector of source_n ints.  *idx == NULL
 * makes a new counts index, else the counts are added to *idx (same k and source_n).  Sequences
 * of length <= k are skipped; windows never span two sequences.  A negative source counts
 * nothing (the reference warns for every window).  Errors, in the reference's order and words:
 * "seq_r should be a character vector of length at least one", "k must be a positive integer
 * less than 1+MAX_K", "source_n must be larger than 1 and larger than source", "mismatch between
 * specified k and that given in the external pointer"; and, where the reference would write
 * out of bounds, a position index or a different source_n is refused.
 * A counts index reads like a position index whose "positions" are the count vectors, as the
 * reference's kmer_positions / sequence_kmer_positions read them: kmer.pos gives count = source_n
 * per k-mer and pos rows (i, count_s) for s = 0..source_n-1, seq.kmer.pos rows (i, count_s);
 * k-mers are ranked by first insertion, or in khash order (kmhg_set_row_order). */
int kmhg_count(kmhg_index **idx, const char *const *seqs, const size_t *lens, int64_t n_seqs,
               int k, int source, int source_n);
/* One device-resident sequence on `stream` (synchronous). */
int kmhg_count_device(kmhg_index **idx, const void *d_seq, size_t L, int k, int source,
                      int source_n, void *stream);

/* ---- read counting: the suffix_hash_n path (SURVEY.md §8 f next-4, depth half) -------------
 * A suffix hash is a counts index of CANONICAL k-mers (min of forward and reverse complement,
 * info.kind = 2, info.sources = counts_n), the reference's suffix_hash_n (src/suffix_hash.c).
 *
 * count.kmers.fq.sh.rp <- .Call("count_kmers_fastq_sh_rp", hash.ptr, params, fq.file)
 *                                                       src/kmer_hash.c:810-857
 *        (+ init_kmer_reader_pool(_sh) / kmer_reader_read src/kmer_reader.c:41-147, the k-mer
 *         iterator src/kmer_util.c:64-162, sh_n_add_kmer src/suffix_hash.c:179-285)
 * params = (k, prefix_bits, min_q, thread_n, max_reads, max_mem, source_n, source).  Reads the
 * FASTA/FASTQ file (plain or gzip) as the reference's kseq does, the first max_reads records
 * (negative: all), skips records of length <= k, and adds one to entry `source` of every
 * canonical k-mer the quality iterator accepts (threshold q_to_ll['!' + min_q]; FASTA records
 * only break at N).  *sh == NULL makes a new suffix hash of source_n counts; into an existing one
 * a different k or a source >= its counts_n prints the reference's message and counts nothing.
 * prefix_bits, thread_n and max_mem do not change the counts.  Errors (reference order and
 * words): "k must be a positive integer less than 1+MAX_K", "Source_n must be in the range
 * 1 - 4", "source_i must be less than source_n"; deviations on the reference's undefined paths:
 * k = 32 and (k < 16, prefix_bits > 2k) are refused. */
int kmhg_sh_count_fastq(kmhg_index **sh, const char *path, const int32_t params[8]);

/* The host reader alone (kseq semantics): records up to max_reads, those longer than k kept,
 * packed as bases / qualities (0 for FASTA records) / offsets[n+1] / has_qual[n]. */
typedef struct kmhg_reads kmhg_reads;
int kmhg_fastx_read(const char *path, int64_t max_reads, int k, kmhg_reads **out);
int kmhg_reads_info(const kmhg_reads *r, int64_t *n_records, int64_t *n_reads, int64_t *n_bases);
int kmhg_reads_copy(const kmhg_reads *r, uint8_t *seq, uint8_t *qual, int64_t *offsets,
                    uint8_t *has_qual);
int kmhg_reads_free(kmhg_reads *r);
/* Count reads already read (same params as kmhg_sh_count_fastq; max_reads is not applied). */
int kmhg_sh_count_reads(kmhg_index **sh, const kmhg_reads *r, const int32_t params[8]);
/* Device-resident packed reads on `stream`: d_seq / d_qual 16-byte aligned with >= 16 readable
 * bytes past the last read, d_offsets[n_reads + 1] (int64), d_has_qual[n_reads]. */
int kmhg_sh_count_reads_device(kmhg_index **sh, const void *d_seq, const void *d_qual,
                               const int64_t *d_offsets, const uint8_t *d_has_qual,
                               int64_t n_reads, const int32_t params[8], void *stream);

/* Diagnostics of the last batch counted into a suffix hash (no reference counterpart): the HLL
 * estimate of its distinct canonical k-mers, the bucket spread its count-only build chose
 * (stream entries per LDS sub-table / 1024), and the path taken: 1 = built at that spread,
 * 2 = a sub-table overflowed and the batch was rebuilt at spread 1, 3 = global find-or-insert. */
int kmhg_sh_last_batch(const kmhg_index *sh, double *distinct_est, int *spread, int *path);

/* seq.kmer.depth.sh <- .Call("seq_kmer_depth_sh", hash.ptr, seq, k)  src/kmer_hash.c:859-879
 *        (+ seq_kmer_counts src/kmer_reader.c:155-193)
 * counts = counts_n x L int32 (R column-major): the counts of the canonical k-mer the reference's
 * walk writes at each position (its write lands at window start - 1 in normal flow, at the start
 * for an init window; see kmhg_sh.hip), zeros for k-mers absent from the hash, INT_MIN (NA)
 * where nothing is written.  Errors: "unable to obtain suffix_hash_n from external pointer",
 * "Receieved error from seq_kmer_counts" (k differs from the hash's); L < k writes nothing at
 * L - k (the reference writes before its buffer). */
int kmhg_sh_depth(kmhg_index *sh, const char *seq, size_t L, int k, int32_t *counts);
int kmhg_sh_depth_device(kmhg_index *sh, const void *d_seq, size_t L, int k, int32_t *d_counts,
                         void *stream);

/* kmer.spec.sh.n <- .Call("kmer_spectrum_suffix_hash_n", ptr, max.count, comb, comb.inner,
 *                          source.min)          src/kmer_hash.c:1010-1039
 *        (+ sh_count_spectrum_nc src/suffix_hash.c:338-421)
 * counts = (comb_n * counts_n) x (max_count + 1) doubles (R column-major).  *status = 1, or the
 * reference's code -3 (comb_inner not 0/1) / -4 (comb >= 2^counts_n) with all counts zero. */
int kmhg_sh_spectrum(kmhg_index *sh, int max_count, const int32_t *comb,
                     const int32_t *comb_inner, int comb_n, const int32_t *source_min,
                     int n_source_min, double *counts, int *status);

/* Rows of a counts index or suffix hash: keys[U] and counts[U * sources] in row order. */
int kmhg_counts_export(kmhg_index *idx, uint64_t *keys, int32_t *counts);

/* Index replication for the multi-GPU query (the index is broadcast once over RCCL/xGMI by the
 * caller): the device image is the hash table (16-B slots {key, count, end}) + the positions +
 * (codes_bytes > 0) the index sequence's 2-bit code words and N flags that the diagonal
 * query path verifies against (0.5 B per window; NULL / 0 = table probes only); export copies
 * it into caller device buffers, import rebuilds an index on the current device. */
typedef struct {
  int64_t table_bytes, positions_bytes, codes_bytes;
} kmhg_image_sizes;
int kmhg_image_sizes_get(const kmhg_index *idx, kmhg_image_sizes *sz, int64_t header[8]);
int kmhg_image_export(const kmhg_index *idx, void *d_table, void *d_positions, void *d_codes,
                      void *stream);
int kmhg_image_import(const int64_t header[8], const void *d_table, const void *d_positions,
                      const void *d_codes, void *stream, kmhg_index **out);

/* Owner-computes multi-GPU build (the reference's own partition pattern, every
 * reader thread inserting only the k-mers it owns, src/kmer_reader.c:28-39): part `part` of
 * `n_parts` walks every window of the (broadcast) sequence but keeps only the k-mers whose hash
 * bucket lies in its contiguous range [b0, b0 + nb) of the whole table's buckets, so each k-mer
 * is built on exactly one device, its positions ascending, with no all-to-all.  The parts,
 * concatenated in bucket order (positions in part order, list ends rebased by each part's first
 * position index), ARE the single-device index: the caller gathers them (RCCL) and imports the
 * result with kmhg_image_import.  A part index refuses queries and readout.
 *   info = {b0, nb, nb_total, slots per bucket, positions N, distinct k-mers U, pairs P, max n,
 *           owns the side slot (key ~0 at k = 32) 0/1, code block bytes}
 *   export: d_table <- its nb x capb slots with count >= 2 list ends + pos_base; d_side_slot <-
 *   its side slot (16 B; meaningful when it owns it); d_positions <- its N int32 positions;
 *   d_codes <- the sequence's code block (every part computes the same one).  Synchronous. */
int kmhg_build_device_part(const void *d_seq, size_t L, int k, int part, int n_parts,
                           void *stream, kmhg_index **out);
int kmhg_part_info(kmhg_index *idx, int64_t info[10]);
int kmhg_part_export(kmhg_index *idx, int64_t pos_base, void *d_table, void *d_side_slot,
                     void *d_positions, void *d_codes, void *stream);

/* Device self-check of the property the radix passes' stable ranks rest on: the lanes of one
 * returning LDS add that hit the same address receive old values in increasing lane order
 * (kmhg_build_v2.hip V_scatter; the bucket kernels also verify every bucket's stream order and
 * fall back).  Writes the same-digit lane pairs found out of order and the pairs checked. */
int kmhg_check_lds_lane_order(uint64_t *out_of_order, uint64_t *checked);

/* Per-kernel HIP-event timing (KMHG_TIMING=1 also enables it).  The report is JSON:
 * {"kernel": [launches, total_ms], ...}; events are recorded on the kernels' own stream. */
int kmhg_timing_enable(int on);
int kmhg_timing_select(const char *kernel);   /* record only this kernel (NULL = all) */
int kmhg_timing_reset(void);
int kmhg_timing_report(char *buf, size_t cap);

/* Device memory pool (caching allocator). */
int kmhg_pool_trim(void);
int64_t kmhg_pool_cached_bytes(void);

#ifdef __cplusplus
}
#endif
#endif /* KMHGPU_H */
