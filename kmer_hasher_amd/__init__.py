"""MI355X-native k-mer position index: the make.kmer.hash / kmer.pos / seq.kmer.pos hot path
of lmjakt/kmer_hasheR as hand-written HIP (gfx950) kernels behind a C-ABI (include/kmhgpu.h),
plus the counting rows next to it (count.kmers, count.kmers.fq.sh.rp, seq.kmer.depth.sh,
kmer.spec.sh.n).

    from kmer_hasher_amd import make_kmer_hash, kmer_pos, seq_kmer_pos
"""
from .api import (FIELDS, KMER_HASH_TAG, SUFFIX_HASH_N_TAG, ExtPtr, KmerHashError, count_kmers,
                  count_kmers_fq_sh_rp, counts_table, kmer_pairs, kmer_pos, kmer_spec_sh_n,
                  make_kmer_hash, seq_kmer_depth_sh, seq_kmer_pos, set_row_order)

__all__ = ["make_kmer_hash", "kmer_pos", "seq_kmer_pos", "kmer_pairs", "count_kmers",
           "count_kmers_fq_sh_rp", "seq_kmer_depth_sh", "kmer_spec_sh_n", "counts_table",
           "set_row_order", "ExtPtr",
           "KmerHashError", "KMER_HASH_TAG", "SUFFIX_HASH_N_TAG", "FIELDS"]
