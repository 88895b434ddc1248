// kmhg_sh.h -- launch wrappers of kmhg_sh.hip (read counting, depth, spectrum).
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include "kmhg_common.h"

namespace kmhg {

constexpr int DP_CPT = 16;                   // depth: chars per lane
constexpr int DP_TILE = BLOCK * DP_CPT;      // depth: chars per workgroup
inline uint32_t depth_tiles(int64_t L) { return (uint32_t)((L + DP_TILE - 1) / DP_TILE); }

// one lane per read of a packed batch: seq / qual bytes (16-B aligned, >= 16 B of padding),
// read r = [off[r], off[r+1]), hasq[r] = 0 for a FASTA record.  cnt = exclusive offsets of the
// per-read UPPER bounds (launch_read_ub + scan, n_reads + 1 entries): keys[cnt[r] + t] =
// canonical k-mer t accepted from read r, EMPTY_KEY after the last (the count-only build skips
// it).  cap = LDS bytes per stream staged per wave of 64 reads (read_kmers_cap_span).
void launch_read_kmers(const uint8_t* seq, const uint8_t* qual, const int64_t* off,
                       const uint8_t* hasq, uint32_t n_reads, int k, double min_ll,
                       const double* qll, uint32_t cap, const uint32_t* cnt, uint64_t* keys,
                       hipStream_t s);
// cnt[r] = max(0, length of read r - k + 1)
void launch_read_ub(const int64_t* off, uint32_t n_reads, int k, uint32_t* cnt, hipStream_t s);
// staging capacity for a batch of mean read length `mean_len`: 1.5x the mean span of a wave,
// 16-B multiple, at most 28 KiB per stream (4+ waves per CU)
// *span = the largest byte span a k_read_kmers workgroup stages (atomicMax; zero it first)
void launch_rk_span(const int64_t* off, uint32_t n_reads, uint32_t* span, hipStream_t s);
// LDS bytes per staged stream: the measured span, capped (a workgroup whose reads do not fit
// walks them from global memory)
inline uint32_t read_kmers_cap_span(uint32_t span) {
  uint32_t c = span < 1024 ? 1024 : span;
  if (c > 28672) c = 28672;
  return (c + 15) & ~15u;
}
// depth: tcnt = depth_tiles(L) u32 (segment starts per tile, scanned in place by the caller),
// sstart / send = segment bounds, n_seg = number of segments, stale = per-segment flag
void launch_depth_seg_count(const uint8_t* seq, int64_t L, uint32_t* tcnt, hipStream_t s);
void launch_depth_seg_emit(const uint8_t* seq, int64_t L, const uint32_t* tbase, uint32_t* sstart,
                           uint32_t* send, hipStream_t s);
void launch_depth_modes(const uint8_t* seq, int64_t L, int k, const uint32_t* sstart,
                        const uint32_t* send, const uint32_t* n_seg, uint8_t* stale, const Slot* T,
                        Geom g, uint32_t S, const int32_t* M, int32_t* out, hipStream_t s);
void launch_depth_probe(const uint8_t* seq, int64_t L, int k, const uint32_t* sstart,
                        const uint32_t* send, const uint32_t* n_seg, const uint8_t* stale,
                        const Slot* T, Geom g, uint32_t S, const int32_t* M, int32_t* out,
                        hipStream_t s);

// batch-table fallback (a bucket of the partitioned build overflowed): T initialised empty
void launch_key_count_insert(const uint64_t* keys, uint64_t n, Slot* T, Geom g, hipStream_t s);

// spectrum bins: (max_count + 1) x comb_n x S u32, zeroed by the caller
void launch_spectrum(const int32_t* M, uint64_t U, uint32_t S, uint32_t max_count,
                     const uint32_t* comb, const uint32_t* inner, uint32_t comb_n,
                     const uint32_t* smin, uint32_t* bins, hipStream_t s);

}  // namespace kmhg
