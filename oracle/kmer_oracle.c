/*
 * oracle/kmer_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's k-mer position-index hot path, written clean-room from
 * the behaviour of lmjakt/kmer_hasheR (no reference source is copied).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this; the product path
 * (kmer_hasher_amd/libkmhgpu.so) never does.
 *
 * Parity is pinned against the reference itself: oracle/_ref/libkmh_ref.so is the reference's
 * own src/kmer_pos.c + src/kmer_util.c + klib compiled by oracle/Makefile, and
 * tests/golden/ holds vectors generated from it (tests/golden/make_golden.py).
 *
 * What each function restates (reference file:line):
 *   orc_windows      window walk of seq_to_hash / seq_kmer_positions
 *                    (src/kmer_pos.c:66-98, 110-136) with init_kmer / skip_n
 *                    (src/kmer_util.c:4-8, 18-32) and UPDATE_OFFSET / LC (src/kmer_util.h:8,10)
 *   orc_index_build  the khash<u64, kvec<int>> build (src/kmer_pos.c:36-50), emitted in the
 *                    canonical order "distinct keys ranked by first position"
 *   orc_query        seq_kmer_positions + pair_positions_push (src/kmer_pos.c:101-136)
 *   orc_pairs        the pair.pos loop of kmer_positions (src/kmer_hash.c:1113-1121)
 *   orc_khash_order  the bucket order khash 0.2.8 gives the same distinct keys
 *                    (src/khash.h:230-348; hash kh_int64_hash_func at src/khash.h:385),
 *                    i.e. the row order of kmer_positions' bucket walk (src/kmer_hash.c:1096)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define IS_N(c) ((((unsigned char)(c)) | 0x20) == 'n')
#define CODE(c) ((((unsigned char)(c)) >> 1) & 3u)

/* Sequential restatement of the reference walk.  The sequence ends at L or at the first NUL.
 * A window [s, s+k) is visited when it holds no N; the FIRST window of every N-free run is
 * skipped when it ends exactly at the end of the sequence (init_kmer returns the past-the-end
 * index and the caller breaks on seq[i]==0).  For each visited window it writes the masked key
 * and the 1-based start (index build, kmer_pos.c:84,91: i+1-k) and the 1-based end (query,
 * kmer_pos.c:127,132: i).  Returns the number of windows. */
long orc_windows(const char *seq, long L, int k, uint64_t *keys, int32_t *start1, int32_t *end1) {
  uint64_t mask = k < 32 ? (((uint64_t)1) << (2 * k)) - 1 : ~(uint64_t)0;
  long n = 0, i = 0;
  for (long t = 0; t < L; ++t) if (!seq[t]) { L = t; break; }
  while (i < L) {
    /* init: find the next k consecutive non-N bases */
    uint64_t code = 0;
    long j = 0;
    for (;;) {
      if (i >= L) return n;
      code = 0;
      for (j = 0; j < k && i + j < L && !IS_N(seq[i + j]); ++j) code = (code << 2) | CODE(seq[i + j]);
      if (i + j >= L || j == k) break;
      i += j;                                   /* at an N: skip the run */
      while (i < L && IS_N(seq[i])) ++i;
    }
    i += j;                                     /* past-the-end of the first window */
    if (i >= L) return n;                       /* the end-drop quirk */
    keys[n] = code & mask; start1[n] = (int32_t)(i + 1 - k); end1[n] = (int32_t)i; ++n;
    while (i < L && !IS_N(seq[i])) {
      code = (code << 2) | CODE(seq[i]);
      ++i;
      keys[n] = code & mask; start1[n] = (int32_t)(i + 1 - k); end1[n] = (int32_t)i; ++n;
    }
  }
  return n;
}

/* ---- a plain key -> id map (linear probing, splitmix64 finaliser) ---- */
typedef struct { uint64_t *keys; int64_t *ids; uint64_t mask; } omap;

static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31;
  return x;
}
static int omap_init(omap *m, long n) {
  uint64_t cap = 16; while (cap < (uint64_t)(2 * n + 16)) cap <<= 1;
  m->keys = malloc(cap * sizeof(uint64_t)); m->ids = malloc(cap * sizeof(int64_t));
  if (!m->keys || !m->ids) return -1;
  memset(m->ids, 0xff, cap * sizeof(int64_t));
  m->mask = cap - 1;
  return 0;
}
static void omap_free(omap *m) { free(m->keys); free(m->ids); }
/* returns slot; *fresh = 1 if the key was inserted now */
static uint64_t omap_slot(omap *m, uint64_t key, int *fresh) {
  uint64_t s = mix64(key) & m->mask;
  for (;;) {
    if (m->ids[s] < 0) { m->keys[s] = key; *fresh = 1; return s; }
    if (m->keys[s] == key) { *fresh = 0; return s; }
    s = (s + 1) & m->mask;
  }
}
static int64_t omap_get(const omap *m, uint64_t key) {
  uint64_t s = mix64(key) & m->mask;
  for (;;) {
    if (m->ids[s] < 0) return -1;
    if (m->keys[s] == key) return m->ids[s];
    s = (s + 1) & m->mask;
  }
}

/* Canonical index (CSR).  ids rank distinct keys by first position, positions ascend.
 *   ukeys[U], counts[U], offsets[U+1], positions[N]   (caller allocates L-sized buffers)
 * Returns U, or -1 on allocation failure.  *n_out = N, *pairs_out = sum C(n,2), *maxn = max n. */
long orc_index_build(const char *seq, long L, int k, uint64_t *ukeys, int32_t *counts,
                     int64_t *offsets, int32_t *positions, long *n_out, int64_t *pairs_out,
                     int32_t *maxn) {
  uint64_t *wk = malloc(sizeof(uint64_t) * (size_t)(L + 1));
  int32_t *ws = malloc(sizeof(int32_t) * (size_t)(L + 1));
  int32_t *we = malloc(sizeof(int32_t) * (size_t)(L + 1));
  int64_t *wid = malloc(sizeof(int64_t) * (size_t)(L + 1));
  if (!wk || !ws || !we || !wid) return -1;
  long N = orc_windows(seq, L, k, wk, ws, we);
  omap m;
  if (omap_init(&m, N) < 0) return -1;
  long U = 0;
  for (long w = 0; w < N; ++w) {
    int fresh;
    uint64_t s = omap_slot(&m, wk[w], &fresh);
    if (fresh) { m.ids[s] = U; ukeys[U] = wk[w]; counts[U] = 0; ++U; }
    wid[w] = m.ids[s];
    counts[wid[w]]++;
  }
  int64_t acc = 0, pairs = 0; int32_t mx = 0;
  for (long u = 0; u < U; ++u) {
    offsets[u] = acc; acc += counts[u];
    pairs += (int64_t)counts[u] * (counts[u] - 1) / 2;
    if (counts[u] > mx) mx = counts[u];
  }
  offsets[U] = acc;
  int64_t *cur = malloc(sizeof(int64_t) * (size_t)(U + 1));
  memcpy(cur, offsets, sizeof(int64_t) * (size_t)U);
  for (long w = 0; w < N; ++w) positions[cur[wid[w]]++] = ws[w];
  free(cur); free(wk); free(ws); free(we); free(wid); omap_free(&m);
  *n_out = N; *pairs_out = pairs; *maxn = mx;
  return U;
}

/* seq.kmer.pos against a canonical index.  Two calls: rows == NULL returns the row count;
 * otherwise fills 2 x H (i_end, j_start) interleaved, rows ordered by i then j. */
int64_t orc_query(const uint64_t *ukeys, const int32_t *counts, const int64_t *offsets,
                  const int32_t *positions, long U, const char *seq, long L, int kq,
                  int32_t *rows) {
  omap m;
  if (omap_init(&m, U) < 0) return -1;
  for (long u = 0; u < U; ++u) { int f; uint64_t s = omap_slot(&m, ukeys[u], &f); m.ids[s] = u; }
  uint64_t *wk = malloc(sizeof(uint64_t) * (size_t)(L + 1));
  int32_t *ws = malloc(sizeof(int32_t) * (size_t)(L + 1));
  int32_t *we = malloc(sizeof(int32_t) * (size_t)(L + 1));
  long N = orc_windows(seq, L, kq, wk, ws, we);
  int64_t h = 0;
  for (long w = 0; w < N; ++w) {
    int64_t id = omap_get(&m, wk[w]);
    if (id < 0) continue;
    if (rows)
      for (int64_t e = offsets[id]; e < offsets[id] + counts[id]; ++e) {
        rows[2 * h] = we[w]; rows[2 * h + 1] = positions[e]; ++h;
      }
    else h += counts[id];
  }
  free(wk); free(ws); free(we); omap_free(&m);
  return h;
}

/* pair.pos rows (i, x, y) for a CSR given in some key order; i = 1 + order index.
 * order[r] = the key id printed as row-group r (NULL = identity). */
int64_t orc_pairs(const int32_t *counts, const int64_t *offsets, const int32_t *positions, long U,
                  const int64_t *order, int32_t *out) {
  int64_t b = 0;
  for (long r = 0; r < U; ++r) {
    long u = order ? (long)order[r] : r;
    const int32_t *a = positions + offsets[u];
    for (int32_t j = 0; j < counts[u]; ++j)
      for (int32_t q = j + 1; q < counts[u]; ++q) {
        out[b++] = (int32_t)(r + 1); out[b++] = a[j]; out[b++] = a[q];
      }
  }
  return b / 3;
}

/* ---- khash 0.2.8 bucket-order replay ----
 * kh_get does not change the table, so the final layout depends only on the sequence of
 * NEW keys, i.e. the distinct keys in first-occurrence order.  This replays kh_put's sizing
 * (4 buckets minimum, power-of-two growth when occupancy reaches (int)(0.77*n+0.5)),
 * triangular probing ((i + ++step) & mask) and the in-place "kick-out" rehash, then walks the
 * buckets in index order.  order_out[r] = id of the r-th existing bucket. */
static uint32_t kh64_hash(uint64_t key) { return (uint32_t)((key >> 33) ^ key ^ (key << 11)); }

typedef struct { uint32_t nb, size, upper; uint8_t *st; int64_t *val; uint64_t *key; } khrep;
/* st: 2 = empty, 1 = deleted (used transiently by the rehash), 0 = live */

static int khrep_grow(khrep *h, uint32_t want) {
  uint32_t nb = 4;
  while (nb < want) nb <<= 1;
  if (h->size >= (uint32_t)(nb * 0.77 + 0.5)) return 0;
  uint8_t *nst = malloc(nb);
  if (!nst) return -1;
  memset(nst, 2, nb);
  if (nb > h->nb) {
    h->key = realloc(h->key, sizeof(uint64_t) * nb);
    h->val = realloc(h->val, sizeof(int64_t) * nb);
  }
  uint32_t nmask = nb - 1;
  for (uint32_t j = 0; j < h->nb; ++j) {
    if (h->st[j] != 0) continue;
    uint64_t k = h->key[j]; int64_t v = h->val[j];
    h->st[j] = 1;
    for (;;) {
      uint32_t i = kh64_hash(k) & nmask, step = 0;
      while (nst[i] != 2) i = (i + (++step)) & nmask;
      nst[i] = 0;
      if (i < h->nb && h->st[i] == 0) {      /* displace a not-yet-moved element */
        uint64_t tk = h->key[i]; int64_t tv = h->val[i];
        h->key[i] = k; h->val[i] = v; k = tk; v = tv;
        h->st[i] = 1;
      } else { h->key[i] = k; h->val[i] = v; break; }
    }
  }
  free(h->st);
  h->st = nst; h->nb = nb; h->upper = (uint32_t)(nb * 0.77 + 0.5);
  return 0;
}

long orc_khash_order(const uint64_t *keys_first_order, long U, int64_t *order_out) {
  khrep h = {0, 0, 0, NULL, NULL, NULL};
  h.st = malloc(1);
  for (long u = 0; u < U; ++u) {
    if (h.size >= h.upper) {               /* no deletions, so n_occupied == size */
      if (khrep_grow(&h, h.nb + 1) < 0) return -1;
    }
    uint32_t mask = h.nb - 1, i = kh64_hash(keys_first_order[u]) & mask, step = 0;
    while (h.st[i] != 2) i = (i + (++step)) & mask;   /* keys are distinct: no match case */
    h.key[i] = keys_first_order[u]; h.val[i] = u; h.st[i] = 0; ++h.size;
  }
  long r = 0;
  for (uint32_t j = 0; j < h.nb; ++j) if (h.st[j] == 0) order_out[r++] = h.val[j];
  free(h.st); free(h.key); free(h.val);
  return r;
}
