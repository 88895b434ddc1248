// tools/asan/host_check.cpp -- the host-side C/C++ of the engine and of the oracle under
// AddressSanitizer + UndefinedBehaviorSanitizer (the reference itself was built
// with fortify / stack protection, src/debug.sh:17-23).  Built by tools/asan/Makefile, driven by
// tests/test_asan_host.py (CPU only).  What runs here is exactly the source the product and the
// checker compile: kmhg_fastx.h (the FASTA/FASTQ reader that parses untrusted input),
// kmhg_khash.h (the khash row-order replay), oracle/kmer_oracle.c and oracle/sh_oracle.c.
//
//   host_check fastx <path> <max_records>   one line per record: R <len> <has_qual> <fnv seq>
//                                           <fnv qual>, then E <last return code>
//   host_check khash <n> <seed>             replay n random distinct keys with kmhg_khash.h and
//                                           the oracle's orc_khash_order; "ok <fnv>" if equal
//   host_check index <path> <k>             orc_index_build + orc_query (self) of the file's
//                                           bytes: U N P maxn H <wsum rows>
//   host_check reads <path> <k> <min_q>     orc_read_kmers of every record: n <wsum keys>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <type_traits>
#include <vector>

#include "../../kmer_hasher_amd/csrc/kmhg_fastx.h"
#include "../../kmer_hasher_amd/csrc/kmhg_khash.h"

extern "C" {
long orc_windows(const char* seq, long L, int k, uint64_t* keys, int32_t* s, int32_t* e);
long orc_index_build(const char* seq, long L, int k, uint64_t* ukeys, int32_t* counts,
                     int64_t* offsets, int32_t* positions, long* n_out, int64_t* pairs_out,
                     int32_t* maxn);
int64_t orc_query(const uint64_t* ukeys, const int32_t* counts, const int64_t* offsets,
                  const int32_t* positions, long U, const char* seq, long L, int kq,
                  int32_t* rows);
long orc_khash_order(const uint64_t* keys, long U, int64_t* order_out);
long orc_read_kmers(const unsigned char* seq, const unsigned char* qual, long len, int k,
                    int min_q, uint64_t* out);
}

static uint64_t fnv(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// order-sensitive digest of an int array, vectorizable on the Python side:
// sum_i x_i * (i * 0x9E3779B97F4A7C15 + 1) mod 2^64 (x_i as unsigned 64-bit)
template <class T>
static uint64_t wsum(const T* x, size_t n) {
  uint64_t h = 0;
  for (size_t i = 0; i < n; ++i)
    h += (uint64_t)(std::make_unsigned_t<T>)x[i] * ((uint64_t)i * 0x9E3779B97F4A7C15ull + 1);
  return h;
}

static std::string slurp(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  std::string s;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
  fclose(f);
  return s;
}

static int cmd_fastx(const char* path, long max_records) {
  kmhg::FastxReader rd(path);
  if (!rd.ok()) { printf("E open\n"); return 0; }
  std::string sq, ql;
  bool hq = false;
  int rc = 0;
  for (long i = 0; i < max_records; ++i) {
    rc = rd.read(sq, ql, hq);
    if (rc < 0) break;
    printf("R %zu %d %016" PRIx64 " %016" PRIx64 "\n", sq.size(), hq ? 1 : 0,
           fnv(sq.data(), sq.size()), fnv(ql.data(), ql.size()));
  }
  printf("E %d\n", rc);
  return 0;
}

static uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static int cmd_khash(long n, uint64_t seed) {
  std::vector<uint64_t> keys;
  std::set<uint64_t> seen;
  uint64_t x = seed;
  while ((long)keys.size() < n) {
    // structured keys (2-bit DNA codes of k <= 31 plus a few near-duplicates) and random ones
    uint64_t v = splitmix(x);
    if (keys.size() % 3 == 0) v &= (1ull << 42) - 1;
    if (keys.size() % 7 == 1 && !keys.empty()) v = keys.back() ^ 1;
    if (seen.insert(v).second) keys.push_back(v);
  }
  const std::vector<uint32_t> a = kmhg::khash_bucket_order(keys);
  std::vector<int64_t> b((size_t)n + 1);
  const long m = orc_khash_order(keys.data(), n, b.data());
  if (m != (long)a.size()) { printf("size %ld %zu\n", m, a.size()); return 1; }
  for (long i = 0; i < m; ++i)
    if ((int64_t)a[(size_t)i] != b[(size_t)i]) { printf("diff at %ld\n", i); return 1; }
  printf("ok %016" PRIx64 "\n", fnv(a.data(), a.size() * 4));
  return 0;
}

static int cmd_index(const char* path, int k) {
  const std::string s = slurp(path);
  const long L = (long)s.size();
  std::vector<uint64_t> keys((size_t)L + 1);
  std::vector<int32_t> counts((size_t)L + 1), pos((size_t)L + 1);
  std::vector<int64_t> offs((size_t)L + 2);
  long N = 0;
  int64_t P = 0;
  int32_t mx = 0;
  const long U = orc_index_build(s.data(), L, k, keys.data(), counts.data(), offs.data(),
                                 pos.data(), &N, &P, &mx);
  if (U < 0) return 1;
  const int kq = k > 31 ? 31 : k;
  int64_t H = 0;
  uint64_t h = 0;
  if (L > kq) {
    H = orc_query(keys.data(), counts.data(), offs.data(), pos.data(), U, s.data(), L, kq,
                  nullptr);
    std::vector<int32_t> rows((size_t)(2 * H + 1));
    orc_query(keys.data(), counts.data(), offs.data(), pos.data(), U, s.data(), L, kq,
              rows.data());
    h = wsum(rows.data(), (size_t)(2 * H));
  }
  printf("%ld %ld %" PRId64 " %d %" PRId64 " %016" PRIx64 "\n", U, N, P, mx, H, h);
  return 0;
}

static int cmd_reads(const char* path, int k, int min_q) {
  kmhg::FastxReader rd(path);
  if (!rd.ok()) return 1;
  std::string sq, ql;
  bool hq = false;
  uint64_t h = 0;
  long n = 0;
  std::vector<uint64_t> all;
  while (rd.read(sq, ql, hq) >= 0) {
    if ((long)sq.size() <= k) continue;
    std::vector<uint64_t> out(sq.size() - k + 1);
    const long m = orc_read_kmers((const unsigned char*)sq.data(),
                                  hq ? (const unsigned char*)ql.data() : nullptr,
                                  (long)sq.size(), k, min_q, out.data());
    all.insert(all.end(), out.begin(), out.begin() + m);
    n += m;
  }
  h = wsum(all.data(), all.size());
  printf("%ld %016" PRIx64 "\n", n, h);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: see the file header\n"); return 2; }
  const std::string c = argv[1];
  if (c == "fastx" && argc == 4) return cmd_fastx(argv[2], atol(argv[3]));
  if (c == "khash" && argc == 4) return cmd_khash(atol(argv[2]), strtoull(argv[3], nullptr, 10));
  if (c == "index" && argc == 4) return cmd_index(argv[2], atoi(argv[3]));
  if (c == "reads" && argc == 5) return cmd_reads(argv[2], atoi(argv[3]), atoi(argv[4]));
  fprintf(stderr, "bad arguments\n");
  return 2;
}
