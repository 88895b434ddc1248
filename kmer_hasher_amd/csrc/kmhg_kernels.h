// kmhg_kernels.h -- launch wrappers of the HIP kernels (host side of kmhg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "kmhg_common.h"

namespace kmhg {

constexpr uint32_t LARGE_MIN = 64;     // keys with >= this many positions sort per workgroup
// partitioned build (kmhg_build_v2.hip)
// group buckets: mean windows per bucket and LDS sub-table slots (load 2/3).  Variant builds
// (A/B, `make variant`) may set -DKMHG_BW_WG=2048 -DKMHG_CAPW=3072 -DKMHG_BUCKET_WGS=4.
#ifndef KMHG_BW_WG
#define KMHG_BW_WG 1024
#endif
#ifndef KMHG_CAPW
#define KMHG_CAPW 1536
#endif
#ifndef KMHG_BUCKET_WGS
#define KMHG_BUCKET_WGS 8      // workgroups per CU the compact LDS table allows (1,536 slots)
#endif
constexpr uint32_t V2_BW_WG = KMHG_BW_WG;
constexpr uint32_t V2_CAPW = KMHG_CAPW;  // slots per group bucket (LDS sub-table of one workgroup)
constexpr uint32_t V2_SLOT_BITS_WG = V2_CAPW >= 2048 ? 12 : 11;
static_assert(V2_CAPW < (1u << V2_SLOT_BITS_WG), "slot index bits");
constexpr uint32_t V2_MAXR = 640;      // LDS digit arrays of the histogram / bounds kernels
constexpr uint32_t V2_MAXR_IL = 320;   // max radix of one partition pass (the scatter's LDS)
constexpr uint32_t SORT_CHUNK = 4096;  // LDS bitonic chunk (16 KiB)

struct BuildMeta {              // written by the build kernels, read once by the host
  uint64_t n_kmers;             // U
  uint64_t n_positions;         // N
  uint64_t n_pairs;             // P = sum C(n, 2)
  uint32_t max_count;           // max n
  uint32_t n_small;             // keys with 2 <= n < LARGE_MIN
  uint32_t n_large;             // keys with n >= LARGE_MIN
  uint32_t overflow;            // partitioned build: a bucket's LDS sub-table filled up
  uint32_t blocks_done;         // V_stats arrival counter (last block publishes to the host)
  double distinct_est;          // count-only builds: V_hll's estimate of the distinct keys
};

struct ReadMeta {               // canonical-order readout preparation
  uint64_t n_keys, n_rows, n_multi, n_pairs;
};

void launch_table_init(Slot* T, uint64_t n, hipStream_t s);
// dst[i] = src[i] with aux += base where count >= 2 (a part's list ends in the whole index)
void launch_part_rebase(const Slot* src, Slot* dst, uint64_t n, uint32_t base, hipStream_t s);
void launch_build_insert(const uint8_t* seq, int64_t L, int k, Slot* T, Geom g,
                         uint32_t* win_slot, int64_t Nw, bool aligned, hipStream_t s);
void launch_build_compact(Slot* T, uint64_t nslots, uint64_t* status, uint32_t* ticket,
                          uint64_t* ukeys, uint32_t* counts, uint32_t* offsets,
                          uint32_t* small_ids, uint32_t* large_ids, BuildMeta* meta,
                          hipStream_t s);
void launch_build_scatter(const uint32_t* win_slot, int64_t Nw, Slot* T, int32_t* positions,
                          hipStream_t s);
void launch_sort_small(const uint32_t* small_ids, const BuildMeta* meta, const uint32_t* counts,
                       const uint32_t* offsets, int32_t* positions, hipStream_t s);
void launch_sort_large(const uint32_t* large_ids, const BuildMeta* meta, const uint32_t* counts,
                       const uint32_t* offsets, int32_t* positions, int32_t* tmp, hipStream_t s);
void launch_inline_singles(Slot* T, uint64_t nslots, const int32_t* positions, hipStream_t s);
// The diagonal query path's view of the INDEX sequence.  The build (V_hist0) keeps its 2-bit
// codes, 16 chars per u32 MSB-first (char c in word c / 16, the LDS stage's format), and its N
// flags, 16 chars per u16 (same order); the first diagonal query derives `uniq` from them and
// the table (V_diag_valid, V_diag_prep): one bit per index window j (0-based, u32 word j / 32,
// bit j % 32) set iff window j is indexed and its key occurs once -- so a set bit says "window
// j's key has count 1 and its slot's aux is j + 1".
struct DiagIdx {
  const uint32_t* code;
  const uint32_t* uniq;
  int64_t nA;            // index windows (L - k + 1)
};
// ceil(Nw / PTILE) partition tiles; PTILE / 16 code (and N-flag) words each, + the words the
// last windows reach into
inline uint64_t diag_tiles(int64_t Nw) { return (uint64_t)((Nw + PTILE - 1) / PTILE); }
inline uint64_t diag_code_words(int64_t Nw) { return diag_tiles(Nw) * (PTILE / 16) + 4; }
inline uint64_t diag_uniq_words(int64_t Nw) { return diag_tiles(Nw) * (PTILE / 32); }   // u32
// the block, in u64 words: code words (u32), N-flag words (u16), uniq words (u32)
inline uint64_t diag_block_words(int64_t Nw) {
  return diag_code_words(Nw) / 2 + diag_code_words(Nw) / 4 + diag_uniq_words(Nw) / 2;
}
struct DiagBlock {
  uint32_t* code;
  uint16_t* nbit;
  uint32_t* uniq;
};
inline DiagBlock diag_block(uint64_t* p, int64_t Nw) {
  uint32_t* c = reinterpret_cast<uint32_t*>(p);
  const uint64_t cw = diag_code_words(Nw);
  return DiagBlock{c, reinterpret_cast<uint16_t*>(c + cw), c + cw + cw / 2};
}
// X.code == nullptr: table probes only.  TG (optional, with X, g.capb % 16 == 0): slot tags for
// the windows the diagonal path does not resolve
void launch_query_probe(const uint8_t* seq, int64_t L, int kq, const Slot* T, Geom g,
                        uint32_t* qrec, uint2* qmulti, int64_t w0, int64_t w1, bool aligned,
                        uint64_t* tile_rows,
                        hipStream_t s, DiagIdx X = DiagIdx{nullptr, nullptr, 0},
                        const uint8_t* TG = nullptr, uint32_t* ecount = nullptr);
// Once per index, before its first diagonal query: `uniq` = the indexed windows (from the N
// flags: the reference's window rule), then TG[i] = slot_tag of slot i (0 empty), all nslots
// slots, and the `uniq` bits of every position of a key seen more than once cleared
void launch_diag_prep(const uint16_t* nbit, int64_t L, int k, uint32_t* uniq, const Slot* T,
                      uint64_t nslots, const int32_t* positions, uint8_t* TG, hipStream_t s);
// An index whose build already wrote the slot tags and set the repeated keys' window bits in
// the uniq words (V_bucket_wg, TAGS): uniq = the indexed windows AND NOT those bits
void launch_diag_valid(const uint16_t* nbit, int64_t L, int k, uint32_t* uniq, bool multi_in,
                       hipStream_t s);
void launch_scan_tiles_u64(uint64_t* a, uint32_t n, uint64_t* total, hipStream_t s);
// the owner-routed query's merge (kmhg_merge_part_rows): n_parts rank segments of rows (rank r's
// at rows + seg_base[r]) with their per-tile offsets tile_off[r * (nt + 1) + t] -> out, ordered
// by window as the unsharded query (one workgroup per query tile of TILE windows from w0)
void launch_merge_part_rows(const int2* rows, const uint64_t* seg_base, const uint64_t* tile_off,
                            uint32_t n_parts, uint32_t nt, int kq, int64_t w0, int2* out,
                            hipStream_t s);
void launch_fill_u64(uint64_t* p, uint64_t v, hipStream_t s);
// a range query's rows as diagonal runs straight from its per-window records: run starts per
// query tile (scanned like the rows' tile totals), then the runs at their tile offsets
void launch_qruns_count(const uint32_t* qrec, const uint2* qmulti, uint64_t Nw,
                        uint64_t* tile_cnt, hipStream_t s);
void launch_qruns_emit(const uint32_t* qrec, const uint2* qmulti, const int32_t* positions,
                       uint64_t Nw, int64_t w0, int kq, const uint64_t* tile_row0,
                       const uint64_t* tile_run0, uint64_t n_runs, int32_t* runs, hipStream_t s);
// a sequence as 2-bit codes + N flags, 16 chars per u32 / u16 word (kmhg_seq_pack /
// kmhg_seq_unpack: C1 transfers); unpack writes chars [a, b) from the words held from w0 on
void launch_seq_pack(const uint8_t* seq, int64_t L, uint32_t* code, uint16_t* nbit,
                     hipStream_t s);
void launch_seq_unpack(const uint32_t* code, const uint16_t* nbit, uint64_t w0, int64_t a,
                       int64_t b, uint8_t* seq, hipStream_t s);
// diagonal runs of query rows (the sharded query's gather format, kmhg_rows_runs /
// kmhg_runs_expand): run starts per TILE rows; the starts as {row, i, j} at the scanned tile
// offsets; and back to rows (`cover`: one u32 per output tile, scratch)
void launch_runs_count(const int2* rows, uint64_t n, uint64_t* tile_cnt, hipStream_t s);
void launch_runs_emit(const int2* rows, uint64_t n, const uint64_t* tile_off, int32_t* runs,
                      hipStream_t s);
void launch_runs_expand(const int32_t* runs, uint64_t n_runs, uint64_t n, uint32_t* cover,
                        int2* out, hipStream_t s);
// exclusive u64 scan in place, *total <- sum: one workgroup up to SCAN1_MAX entries, else
// reduce-then-scan with `scratch` = scan_u64_scratch(n) u64
// (round 4: one workgroup up to 64 K / 256 K totals instead -- config 3 query 185 -> 162 Gbp/s,
// config 5 92.5 -> 82.4; profiles/rd4ak_*)
constexpr uint64_t SCAN1_MAX = 16384;
inline uint64_t scan_u64_scratch(uint64_t n) { return (n + TILE - 1) / TILE + 1; }
void launch_scan_u64(uint64_t* a, uint64_t n, uint64_t* total, uint64_t* scratch, hipStream_t s);
// rows >= cap are dropped (the caller re-runs the emit into an exact buffer if the total exceeds
// cap).  Two kernels: Q_emit1 writes the tiles whose windows have <= 1 hit and lists the others
// in elist (nt entries; *ecount zeroed by the probe), Q_emit writes the listed tiles.  A re-emit
// passes append = false (the list is already complete).
void launch_query_emit(const uint32_t* qrec, const uint2* qmulti, int64_t Nw, int64_t w0, int kq,
                       const int32_t* positions, const uint64_t* tile_row0, int2* out,
                       uint64_t cap, uint32_t* elist, uint32_t* ecount, bool append,
                       hipStream_t s);
// F = L entries {slot, count} preset to slot NONE
void launch_read_first(const Slot* T, uint64_t nslots, const int32_t* positions, uint2* F,
                       hipStream_t s);
// rinfo[c] = {count, aux} of row c's slot, so the readout kernels below read rows in order
// instead of gathering T[perm[c]] (only the k-mer strings need the slot itself)
void launch_read_order(const uint2* F, int64_t L, const Slot* T, uint64_t* st_a, uint64_t* st_b,
                       uint64_t* st_c, uint32_t* ticket, uint32_t* perm, uint32_t* canon_off,
                       uint32_t* pkeys, uint64_t* pair_off, uint2* rinfo, ReadMeta* rmeta,
                       hipStream_t s);
void launch_read_keys(const uint32_t* perm, const uint2* rinfo, uint32_t U, const Slot* T, int k,
                      int32_t* out_counts, char* out_kmers, hipStream_t s);
void launch_gather_keys(const uint32_t* perm, uint32_t U, const Slot* T, uint64_t* out_keys,
                        hipStream_t s);
void launch_read_pos(const uint2* rinfo, const uint32_t* canon_off, uint32_t U, uint64_t nrows,
                     const int32_t* positions, uint32_t* tile_key, int2* out, hipStream_t s);
uint32_t read_pos_tiles(uint64_t nrows);     // tile_key holds read_pos_tiles(nrows) + 1 u32
void launch_read_pairs(const uint32_t* pkeys, const uint64_t* pair_off, uint32_t M,
                       uint64_t nrows, const uint2* rinfo, const int32_t* positions,
                       uint32_t* tile_key, int32_t* out, hipStream_t s);
uint32_t read_pairs_tiles(uint64_t nrows);   // tile_key holds read_pairs_tiles(nrows) + 1 u32
// radix digit of a bucket id: floor(b / div) mod R via magic multipliers (see digit_of)
struct Digit {
  uint64_t mdiv;   // ceil(2^64 / div), 0 for div = 1
  uint64_t mR;     // ceil(2^64 / R), 0 for R = 1
  uint32_t R;
  int nbits;       // bits to name a digit 0..R-1
};
inline uint64_t magic64(uint32_t d) {   // ceil(2^64 / d) for d >= 2
  return d <= 1 ? 0 : (uint64_t)(~0ull / d) + 1;
}
inline Digit make_digit(uint32_t div, uint32_t R) {
  Digit d;
  d.mdiv = magic64(div);
  d.mR = magic64(R);
  d.R = R;
  d.nbits = 0;
  while ((1u << d.nbits) < R) ++d.nbits;
  return d;
}
// Radix passes run over tiles of PTILE windows; histograms are [digit][tile] (ntiles columns),
// and the persistent scatter grids give every XCD one contiguous tile range (xcd_remap).
// V_hist0 also zeroes the look-back words of the scan that follows (n_status u64) and `meta`
// code / nbit (optional, position indices: the diagonal query path, DiagBlock): the sequence's
// 2-bit code words and N-flag words
void launch_v2_hist0(const uint8_t* seq, int64_t L, int k, int64_t Nw, Geom g, Digit D,
                     uint32_t* hist, uint32_t ntiles, uint64_t* scan_status, uint32_t n_status,
                     BuildMeta* meta, hipStream_t s, uint32_t* code = nullptr,
                     uint16_t* nbit = nullptr, uint32_t* bids = nullptr,
                     uint64_t* ckeys = nullptr, uint32_t* cpos = nullptr,
                     uint32_t* tcnt = nullptr);
// ckeys (a part build, key streams): instead of the histogram, the part's windows compacted
// per tile, (key, position) at [t * PTILE, t * PTILE + tcnt[t]) in window order (ckeys / cpos
// hold Nw + PTILE entries); after a scan of tcnt (offsets, total in n_total) launch_part_dense
// packs them into dk / dp
void launch_part_dense(const uint64_t* ck, const uint32_t* cp, const uint32_t* off,
                       uint32_t ntiles, const uint32_t* n_total, uint64_t* dk, uint32_t* dp,
                       hipStream_t s, bool aos = false);
// The scatter passes' outputs hold n_max + PTILE elements: lanes past a tile's end store into the
// pad at [pad, pad + BLOCK) so every lane issues the same stores (see k_v2_scatter).
// exclusive scan of a u32 array; status = tiles_for(n) + 1 u64, zeroed by the histogram kernel
// launched before it; total <- sum.  Single-pass look-back (8192-entry tiles beyond 64 2048-entry
// tiles).
void launch_scan_u32(uint32_t* a, uint64_t n, uint64_t* status, uint32_t* total, hipStream_t s);
// hll_rows (count-only builds, first pass): the histogram workgroups also sketch the distinct
// keys (HyperLogLog, HLL_REGS registers, 1/64 key-space sample) into one 256-B row each (ntiles
// rows, HLL_REGS / 4 u32); launch_v2_hll reduces the rows (through hll_regs = HLL_PART_WORDS u32
// of partial rows) and writes the distinct-key estimate to *host_est (pinned host memory)
constexpr uint32_t HLL_REGS = 256;
constexpr uint32_t HLL_PART_WORDS = 256 * 64 + 1;
void launch_v2_hist(const uint64_t* keys, const uint32_t* n_ptr, Geom g, Digit D, uint32_t* hist,
                    uint32_t ntiles, uint64_t* scan_status, uint32_t n_status, hipStream_t s,
                    uint32_t* hll_rows = nullptr, uint32_t* hll_regs = nullptr,
                    uint32_t* save_col0 = nullptr, bool skip_empty = false,
                    bool padded = false, bool aos = false, int sh8 = 0);
// one level of the bucket starts from the histograms (the unfused form of BoundsFuse): one
// workgroup per lo value (div of them); kprev = pass p's input keys, lo_start = S_(p-1) (pass 0's
// column 0 saved by launch_v2_hist's save_col0 for p = 1; nullptr for one pass); start[c / spread]
// for c < nlim that are multiples of spread, start[nlim / spread] = n
// bprev (bucket-id streams): the pass's input bucket ids instead of kprev
void launch_v2_bounds_lo(const uint64_t* kprev, const uint32_t* n_ptr, Geom g, Digit Dlast,
                         uint32_t div, const uint32_t* hist, uint32_t C, const uint32_t* lo_start,
                         uint32_t spread, uint32_t* start, uint32_t nlim, hipStream_t s,
                         const uint32_t* bprev = nullptr, bool aos = false, int sh8 = 0);
// segb (Pack8) from pass 0's scanned histogram: R x (nseg + 1) entries, tps = tiles per segment
void launch_seg_bounds(const uint32_t* hist, uint32_t ntiles, uint32_t R, uint32_t nseg,
                       uint32_t tps, const uint32_t* n_valid, uint32_t* segb, hipStream_t s);
// also copies *n_valid (launch it after the pass's scan) to *host_n
void launch_v2_hll(const uint32_t* hll_rows, uint32_t n_rows, uint32_t* hll_regs, double* host_est,
                   const uint32_t* n_valid, uint64_t* host_n, hipStream_t s);
// One level of V_bounds_lo folded into radix pass p >= 1: its inputs -- the pass's input
// stream, its scanned histogram, the starts of the input's combined lower digits (S_(p-1)) --
// are complete before the pass starts, and its output (S_p: the bucket starts for the last pass)
// is read only by the next level or the bucket kernel, so the pass's workgroups each compute
// the starts of a few lower-digit values before their tiles (no launch, no key pass).
// start == nullptr: not fused.
// A radix pass's digit stream (DS): out[i] = the next pass's digit of output element i (u16,
// or u8 in out8 for a radix <= 256; n + PTILE entries), which the next pass's histogram reads
// (launch_v2_hist_digits) instead of the keys: 1-2 B per element instead of 8 or 12.
struct DigitOut {
  uint16_t* out;
  Digit Dn;
  uint8_t* out8 = nullptr;
};
constexpr DigitOut kNoDigits{nullptr, Digit{}, nullptr};
void launch_v2_hist_digits(const void* digits, bool u8, const uint32_t* n_ptr, Geom g, Digit D,
                           uint32_t* hist, uint32_t ntiles, uint64_t* scan_status,
                           uint32_t n_status, hipStream_t s, uint32_t* save_col0 = nullptr);
// Packed 8-B elements of a small-k key stream (the first pass of a two-pass build with 2k <= 52,
// i.e. k <= 26: the engine needs sh >= 12): the high 2k bits hold the key, the low sh = 64 - 2k bits the window's index inside its segment
// of 2^sh windows.  The segment comes back from the element's place in the stream: pass 0 writes
// digit d's elements tile by tile, so segment s of digit d starts at the scanned histogram entry
// of (d, s * 2^sh / PTILE) -- segb[d * (nseg + 1) + s], nseg + 1 entries per digit.
struct Pack8 {
  int sh;                      // 0: no packed stream
  const uint32_t* segb;
  uint32_t nseg;
  Digit d0;                    // pass 0's digit
};
struct BoundsFuse {
  const uint64_t* kprev;       // the pass's input (keys, or bucket ids with bid = 1)
  const uint32_t* lo_start;    // S_(p-1): starts of the input's combined lower digits
  uint32_t* start;             // S_p
  Digit Dlast;                 // the pass's own digit
  uint32_t div, spread;        // div = R^p lower-digit values
  int bid;                     // 0 u64 keys, 1 u32 bucket ids, 2 packed 12-B (key, pos) elements,
                               // 3 packed 8-B (key << sh | window) elements
  uint32_t nlim;               // entries of S_p: nb for the last pass, R^(p+1) before
  int sh = 0;                  // bid 3: the element's key is e >> sh
};
// the sequence must be 16-B aligned (the engine copies an unaligned input)
void launch_v2_scatter_seq(const uint8_t* seq, int64_t L, int k, int64_t Nw, Geom g, Digit D,
                           const uint32_t* hist, uint32_t ntiles, uint64_t* kout, uint32_t* pout,
                           uint32_t pad, hipStream_t s, bool aos = false,
                           const Pack8* pk = nullptr, const DigitOut* ds = nullptr);
// first pass over a caller's key stream of n_keys keys (>= 1): positions are e + 1; nopos:
// keys only (count-only builds), pout unused; skip_empty: EMPTY_KEY entries are not keys (padded
// read k-mer streams, k <= 31)
void launch_v2_scatter_keys0(const uint64_t* kin, uint64_t n_keys, const uint32_t* n_ptr, Geom g,
                             Digit D, const uint32_t* hist, uint32_t ntiles, uint64_t* kout,
                             uint32_t* pout, uint32_t pad, bool nopos, bool skip_empty,
                             hipStream_t s);
void launch_v2_scatter_nopos(const uint64_t* kin, const uint32_t* n_ptr, Geom g, Digit D,
                             const uint32_t* hist, uint32_t ntiles, uint64_t* kout, uint32_t pad,
                             hipStream_t s, const BoundsFuse* bf = nullptr);
void launch_v2_scatter(const uint64_t* kin, const uint32_t* pin, const uint32_t* n_ptr, Geom g,
                       Digit D, const uint32_t* hist, uint32_t ntiles, uint64_t* kout, uint32_t* pout,
                       uint32_t pad, hipStream_t s, const BoundsFuse* bf = nullptr,
                       bool aos = false, bool aos_in = true, const Pack8* pk = nullptr,
                       const DigitOut* ds = nullptr);
// Packed key streams (aos): position builds on key streams carry each window as ONE 12-B
// element {key lo, key hi, pos} (kout holds n + PTILE of them; pout unused), so a tile's digit
// run is one contiguous write; aos_in: the input is packed too (else kin / pin arrays).
// Bucket-id streams (position builds that keep the sequence's code words): V_hist0 stores
// every window's bucket id (`bids`, Nw u32, ~0 = not indexed), the radix passes carry (bucket
// id u32, pos u32) and the last pass writes positions only (bout = nullptr); the bucket kernel
// cuts the keys from the code words.  Histograms without hashing.
void launch_v2_scatter_bid0(const uint32_t* bids, int64_t Nw, Geom g, Digit D,
                            const uint32_t* hist, uint32_t ntiles, uint32_t* bout, uint32_t* pout,
                            uint32_t pad, hipStream_t s, const DigitOut* ds = nullptr);
void launch_v2_scatter_bid(const uint32_t* bin, const uint32_t* pin, const uint32_t* n_ptr,
                           Geom g, Digit D, const uint32_t* hist, uint32_t ntiles, uint32_t* bout,
                           uint32_t* pout, uint32_t pad, hipStream_t s,
                           const BoundsFuse* bf = nullptr, const DigitOut* ds = nullptr);
void launch_v2_hist_bid(const uint32_t* bids, const uint32_t* n_ptr, Geom g, Digit D,
                        uint32_t* hist, uint32_t ntiles, uint64_t* scan_status, uint32_t n_status,
                        hipStream_t s, uint32_t* save_col0 = nullptr);
struct BucketStats {           // per-bucket partials of the build statistics
  uint32_t n_kmers, max_count;
  uint64_t n_pairs;
};
// count_only: occurrence counts only (no positions written; slot aux unspecified)
// code (bucket-id streams): keys unused, each window's key cut from the code words at its pos
void launch_v2_bucket_wg(const uint64_t* keys, const uint32_t* pos, const uint32_t* start, Geom g,
                         Slot* T, int32_t* positions, BucketStats* bstats, BuildMeta* meta,
                         bool count_only, hipStream_t s, const uint32_t* n_ptr, uint32_t nw,
                         const uint32_t* code = nullptr, int k = 0, bool aos = false,
                         uint8_t* TG = nullptr, uint32_t* rep = nullptr);
// TG / rep (key-stream position builds): the build also writes the diagonal path's slot tags and
// sets the repeated keys' window bits in rep (zeroed by the caller); the first query then runs
// launch_diag_valid(..., multi_in = true) instead of launch_diag_prep
// ballot_ranks(): the current device fails the LDS lane-order self-check (or KMHG_TEST_BALLOT):
// the radix passes and the bucket kernel then rank with ballots (kmhg_engine.cpp)
bool ballot_ranks();
void launch_lane_order_check(unsigned long long* res, hipStream_t s, int blocks = 1024);
void launch_v2_test_disorder(uint32_t* pos, uint32_t* start, const uint32_t* n_ptr, int mode,
                             hipStream_t s, uint32_t stride = 1);
void launch_v2_stats(const BucketStats* bstats, uint32_t nb, const uint32_t* n_valid,
                     BuildMeta* meta, BuildMeta* host_meta, hipStream_t s);

// kmer.pairs (kmhg_join.hip)
void launch_join_probe(const uint32_t* perm_a, uint32_t Ua, const Slot* Ta, const Slot* Tb, Geom gb,
                       uint4* jinfo, uint64_t* tile_rows, hipStream_t s);
void launch_join_emit(const uint4* jinfo, uint32_t Ua, const int32_t* pos_a, const int32_t* pos_b,
                      const uint64_t* tile_row0, int2* out, hipStream_t s);

// count.kmers (kmhg_count.hip)
void launch_count_probe(const uint32_t* perm_b, uint32_t Ub, const Slot* Tb, const Slot* Tc,
                        Geom gc, const uint32_t* slot_row, uint32_t S, uint32_t source,
                        int32_t* M, uint32_t* newf, hipStream_t s);
// rord (count.kmers; nullptr for a suffix hash): new row's order key = base + its key's first
// position in the batch (bpos: the batch's position lists) - 1
void launch_count_append(const uint32_t* perm_b, uint32_t Ub, const Slot* Tb,
                         const uint32_t* rank, const uint32_t* n_new, uint32_t U0, uint32_t S,
                         uint32_t source, uint64_t* ckeys, int32_t* M, const int32_t* bpos,
                         uint64_t* rord, uint64_t base, hipStream_t s);
void launch_count_insert(const uint64_t* ckeys, uint32_t U, Slot* T, Geom g, uint32_t S,
                         const int32_t* M, uint32_t* slot_row, uint32_t* row_slot,
                         hipStream_t s);
// first-insertion order of a count.kmers index's rows: F = n u32 preset to NONE, n > every
// order key; `status` = ceil(n / TILE) zeroed look-back words, `ticket` a zeroed u32; rorder[i] =
// the row read out i-th.  C_gather copies the rows out in that order.
void launch_rows_place(const uint64_t* rord, uint32_t U, uint32_t* F, hipStream_t s);
void launch_rows_order(const uint32_t* F, int64_t n, uint64_t* status, uint32_t* ticket,
                       uint32_t* rorder, hipStream_t s);
// rorder by a radix sort of the U (order key, row) pairs instead (O(U) scratch: keys_out U u64,
// rows_in U u32, temp rows_sort_temp_bytes(U, bits)); bits covers every order key
hipError_t rows_sort_temp_bytes(uint32_t U, int bits, size_t* bytes);
hipError_t launch_rows_sort(const uint64_t* rord, uint32_t U, int bits, uint64_t* keys_out,
                      uint32_t* rows_in, uint32_t* rorder, void* temp, size_t temp_bytes,
                      hipStream_t s);
void launch_rows_gather(const uint32_t* rorder, const uint64_t* ckeys, const int32_t* M,
                        uint32_t U, uint32_t S, uint64_t* okeys, int32_t* oM, hipStream_t s);
// first batch into a new counts index / suffix hash: rows in slot order; `status` =
// count_walk_tiles zeroed look-back words, `ticket` a zeroed u32; rord (count.kmers; nullptr for a
// suffix hash): each row's order key, base + its first position in the batch (bpos) - 1
uint64_t count_walk_tiles(uint64_t nslots);   // look-back words launch_count_walk needs
// the same walk with bucket-aligned tiles (a batch from the partitioned build, bstats = its
// per-bucket statistics): C_wcount writes count_walk_b_tiles(nb) tile counts to tc (and zeroes
// *err), k_scan_u32 turns them into offsets (nt + 1 entries, [nt] = total), C_walk_b writes the
// rows and raises *err if a tile's occupied slots disagree with the statistics
uint32_t count_walk_b_tiles(uint32_t nb);
void launch_walk_counts(const BucketStats* bs, const Slot* T, Geom g, uint32_t* tc, uint32_t nt,
                        uint32_t* err, hipStream_t s);
void launch_count_walk_b(Slot* T, Geom g, const uint32_t* tbase, uint32_t nt, uint32_t S,
                         uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                         uint32_t* row_slot, const int32_t* bpos, uint64_t* rord, uint64_t base,
                         uint32_t* err, hipStream_t s);
void launch_count_walk(Slot* T, uint64_t nslots, uint64_t* status, uint32_t* ticket, uint32_t S,
                       uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                       uint32_t* row_slot, const int32_t* bpos, uint64_t* rord, uint64_t base,
                       hipStream_t s);
void launch_count_fix(Slot* T, uint64_t nslots, uint32_t S, const int32_t* M, uint32_t* slot_row,
                      uint32_t* row_slot, hipStream_t s);
// rorder: the rows in readout order (nullptr: the row order itself)
void launch_count_canon(const uint32_t* rorder, const uint32_t* row_slot, const int32_t* M,
                        uint32_t U, uint32_t S, uint32_t* perm, uint32_t* canon_off,
                        uint32_t* pkeys, uint64_t* pair_off, uint2* rinfo, hipStream_t s);

#ifdef KMHG_STAMPS
void set_stamp_buffer(uint64_t* p);
#endif

inline uint32_t tiles_for(uint64_t n) { return (uint32_t)((n + TILE - 1) / TILE); }

}  // namespace kmhg
