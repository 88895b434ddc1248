// kmhg_khash.h -- host-only: the khash 0.2.8 bucket-order replay behind KMHG_ORDER_KHASH.
// Plain C++ (no HIP), so the sanitizer harness (tools/asan/) builds it with
// -fsanitize=address,undefined beside the FASTA/FASTQ reader.
#pragma once
#include <cstdint>
#include <utility>
#include <vector>

namespace kmhg {

// khash 0.2.8 bucket-order replay (the reference's row order, src/kmer_hash.c:1096-1124).
// The reference only ever calls kh_get (read-only) and kh_put on NEW keys, so its final table
// depends only on the distinct keys in first-insertion order = our first-occurrence order.  This
// replays kh_put's sizing (4 buckets minimum; when occupancy reaches (int)(0.77 nb + 0.5) the
// table is resized to the next power of two above nb, src/khash.h:307-317), its probe sequence
// (i + ++step) & mask from hash (u32)(key>>33 ^ key ^ key<<11) (src/khash.h:385), and kh_resize's
// in-place rehash, which moves elements by kick-out in old-bucket order (src/khash.h:244-306).
// Returns order[r] = first-occurrence id of the r-th live bucket.
inline std::vector<uint32_t> khash_bucket_order(const std::vector<uint64_t>& keys) {
  enum : uint8_t { LIVE = 0, MOVED = 1, EMPTY = 2 };
  auto hash = [](uint64_t k) { return (uint32_t)((k >> 33) ^ k ^ (k << 11)); };
  uint32_t nb = 0, size = 0, upper = 0;
  std::vector<uint8_t> st;
  std::vector<uint64_t> key;
  std::vector<uint32_t> val;
  auto resize = [&](uint32_t want) {
    uint32_t nnb = 4;
    while (nnb < want) nnb <<= 1;
    if (size >= (uint32_t)(nnb * 0.77 + 0.5)) return;   // too small: unchanged
    std::vector<uint8_t> nst(nnb, EMPTY);
    if (nnb > nb) { key.resize(nnb); val.resize(nnb); }
    const uint32_t nmask = nnb - 1;
    for (uint32_t j = 0; j < nb; ++j) {
      if (st[j] != LIVE) continue;
      uint64_t k = key[j];
      uint32_t v = val[j];
      st[j] = MOVED;
      for (;;) {                            // kick-out: displace a not-yet-moved element
        uint32_t i = hash(k) & nmask, step = 0;
        while (nst[i] != EMPTY) i = (i + (++step)) & nmask;
        nst[i] = LIVE;
        if (i < nb && st[i] == LIVE) {
          std::swap(k, key[i]);
          std::swap(v, val[i]);
          st[i] = MOVED;
        } else {
          key[i] = k;
          val[i] = v;
          break;
        }
      }
    }
    st.swap(nst);
    nb = nnb;
    upper = (uint32_t)(nb * 0.77 + 0.5);
  };
  for (uint32_t u = 0; u < (uint32_t)keys.size(); ++u) {
    if (size >= upper) resize(nb + 1);      // no deletions: n_occupied == size
    const uint32_t mask = nb - 1;
    uint32_t i = hash(keys[u]) & mask, step = 0;
    while (st[i] != EMPTY) i = (i + (++step)) & mask;   // distinct keys: never a match
    key[i] = keys[u];
    val[i] = u;
    st[i] = LIVE;
    ++size;
  }
  std::vector<uint32_t> order;
  order.reserve(size);
  for (uint32_t j = 0; j < nb; ++j)
    if (st[j] == LIVE) order.push_back(val[j]);
  return order;
}

}  // namespace kmhg
