"""MI355X-native k-mer position index: the make.kmer.hash / kmer.pos / seq.kmer.pos hot path
of lmjakt/kmer_hasheR as hand-written HIP (gfx950) kernels behind a C-ABI (include/kmhgpu.h).

    from kmer_hasher_amd import make_kmer_hash, kmer_pos, seq_kmer_pos
"""
from .api import (FIELDS, KMER_HASH_TAG, ExtPtr, KmerHashError, count_kmers, kmer_pairs,
                  kmer_pos, make_kmer_hash, seq_kmer_pos, set_row_order)

__all__ = ["make_kmer_hash", "kmer_pos", "seq_kmer_pos", "kmer_pairs", "count_kmers",
           "set_row_order", "ExtPtr",
           "KmerHashError", "KMER_HASH_TAG", "FIELDS"]
