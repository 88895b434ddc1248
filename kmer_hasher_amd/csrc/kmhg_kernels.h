// kmhg_kernels.h -- launch wrappers of the HIP kernels (host side of kmhg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "kmhg_common.h"

namespace kmhg {

constexpr uint32_t LARGE_MIN = 64;     // keys with >= this many positions sort per workgroup
constexpr uint32_t SORT_CHUNK = 4096;  // LDS bitonic chunk (16 KiB)

struct BuildMeta {              // written by the build kernels, read once by the host
  uint64_t n_kmers;             // U
  uint64_t n_positions;         // N
  uint64_t n_pairs;             // P = sum C(n, 2)
  uint32_t max_count;           // max n
  uint32_t n_small;             // keys with 2 <= n < LARGE_MIN
  uint32_t n_large;             // keys with n >= LARGE_MIN
  uint32_t pad_;
};

struct ReadMeta {               // canonical-order readout preparation
  uint64_t n_keys, n_rows, n_multi, n_pairs;
};

void launch_table_init(Slot* T, uint64_t n, hipStream_t s);
void launch_build_insert(const uint8_t* seq, int64_t L, int k, Slot* T, uint64_t cap,
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
void launch_query_probe(const uint8_t* seq, int64_t L, int kq, const Slot* T, uint64_t cap,
                        uint2* qinfo, int64_t w0, int64_t w1, bool aligned, uint64_t* status,
                        uint32_t* ticket, uint64_t* tile_row0, uint64_t* total_rows,
                        hipStream_t s);
void launch_query_emit(const uint2* qinfo, int64_t Nw, int64_t w0, int kq,
                       const int32_t* positions, const uint64_t* tile_row0, int2* out,
                       hipStream_t s);
void launch_read_first(const uint32_t* offsets, const int32_t* positions, uint32_t U, uint32_t* F,
                       hipStream_t s);
void launch_read_order(const uint32_t* F, int64_t L, const uint32_t* counts, uint64_t* st_a,
                       uint64_t* st_b, uint64_t* st_c, uint32_t* ticket, uint32_t* perm,
                       uint32_t* canon_off, uint32_t* pkeys, uint64_t* pair_off,
                       ReadMeta* rmeta, hipStream_t s);
void launch_read_keys(const uint32_t* perm, uint32_t U, const uint64_t* ukeys,
                      const uint32_t* counts, int k, int32_t* out_counts, char* out_kmers,
                      hipStream_t s);
void launch_read_pos(const uint32_t* perm, const uint32_t* canon_off, uint32_t U, uint64_t nrows,
                     const uint32_t* offsets, const int32_t* positions, int2* out, hipStream_t s);
void launch_read_pairs(const uint32_t* pkeys, const uint64_t* pair_off, uint32_t M,
                       uint64_t nrows, const uint32_t* perm, const uint32_t* counts,
                       const uint32_t* offsets, const int32_t* positions, int32_t* out,
                       hipStream_t s);

inline uint32_t tiles_for(uint64_t n) { return (uint32_t)((n + TILE - 1) / TILE); }

}  // namespace kmhg
