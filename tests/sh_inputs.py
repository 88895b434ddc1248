"""Inputs of the read-counting parity cases (count.kmers.fq.sh.rp / seq.kmer.depth.sh /
kmer.spec.sh.n): FASTX files and depth query strings.  Deterministic; shared by
tests/golden/make_sh_golden.py and the tests.

The reference's own FASTQ files (repeat_40.fq, test_10.fastq, test.fastq.gz) are kept as data
fixtures under tests/golden/."""
import os

import numpy as np

from kmer_hasher_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_FILES = ["repeat_40.fq", "test_10.fastq", "test.fastq.gz"]


def tricky_fastx() -> bytes:
    """Every kseq / iterator corner the reader must reproduce: multi-line FASTA and FASTQ, CRLF,
    N and lower-case bases, '@' and '+' inside qualities, records no longer than k, empty
    records, a quality run below the threshold, '!' qualities, and a truncated final record
    (kseq error -2 ends the file).  FASTA records come first: after a FASTQ record the
    reference's iterator keeps the previous record's quality pointer for a FASTA record
    (kmer_iterator_begin never clears it->qual, src/kmer_util.c:100-102) and reads stale kseq
    buffer bytes -- undefined, so mixed files are only compared in this order."""
    parts = [
        b"junk before the first record\n",
        b">fa1 a comment\nACGTACGTNNACGTACGTAACCGGTTAC\nACGTTTGCATTGACCAGT\n\n",
        b">fa2\nacgtnacgtacgtacgtggaccaGGTTNNNNNNNNNNacgtacgtacgtacgtacgt\n",
        b"@q1\r\nACGTACGTACGTAAGGCCTTACGTGGATCCA\r\n+\r\nIIIIIIIIII#IIIIIIIIIIIIIII!IIII\r\n",
        b"@q2 desc here\nACGTNACGTACGTTTGACCA\nGGTACATTGACAT\n+q2\nIIIII5IIII\n"
        b"IIIIIIIIIIIIIIIIIIIIIII\n",
        b"@short\nACGTA\n+\nIIIII\n",
        b"@lowq\nACGTACGTTTGGCCAAACGTACGTTTGGCCAAGGTT\n+\nIIIII$$$$$$$$$IIIIIIIIIIIIIIIIIIIIII\n",
        b"@atq\nTTGACCATGGACCATTGGACACAGTTAGG\n+\n@IIIIIII+IIIIIIIII>IIIIIIIIII\n",
        b"@empty\n\n+\n\n",
        b"@nq\nNNNNACGTACGTACGTACGTNACGTACGTACGTACGTACGTAC\n+\n"
        b"############IIIIIIIIIIIIIIIIIIIIIIIIIIIIIII\n",
        b"@bang\nACGTACGTACGTACGTACGTACGTACGT\n+\n!!!!!!!!!!!!!!!!!!!!!!!!!!!!\n",
        b"@trunc\nACGTACGTACGTACGTACGTACGTACGTACGT\n+\nIIII\n",
        b"@after\nACGTACGTACGTACGTACGTACGTACGTACGT\n+\nIIIIIIIIIIIIIIIIIIIIIIIIIIIIIIII\n",
    ]
    return b"".join(parts)


def random_fastx(n_records: int, seed: int) -> bytes:
    """Random records (FASTA and FASTQ, multi-line, CRLF, N runs, random phred) for a fuzz;
    FASTA records first (see tricky_fastx)."""
    rng = np.random.default_rng(seed)
    out, fa = [], []
    for i in range(n_records):
        ln = int(rng.integers(0, 90))
        s = rng.choice(list(b"ACGTacgtNNRY"), ln,
                       p=[.205, .205, .205, .205, .03, .03, .03, .03, .02, .02, .01, .01]).astype(np.uint8)
        nl = b"\r\n" if rng.random() < 0.2 else b"\n"
        if rng.random() < 0.25:
            body = s.tobytes()
            cut = int(rng.integers(0, ln + 1))
            fa.append(b">s%d x%s%s%s%s%s" % (i, nl, body[:cut], nl, body[cut:], nl))
        else:
            q = rng.integers(33, 75, ln).astype(np.uint8)
            if rng.random() < 0.3:
                q[rng.random(ln) < 0.3] = 35
            qb = q.tobytes()
            cut = int(rng.integers(0, ln + 1)) if rng.random() < 0.3 else ln
            qual = qb[:cut] + nl + qb[cut:] + nl if cut < ln else qb + nl
            out.append(b"@r%d%s%s%s+%s%s" % (i, nl, s.tobytes(), nl, nl, qual))
    return b"".join(fa + out)


def sim_reads_fastq(n_reads: int, read_len: int, seed: int, genome_len: int = 20000):
    """(genome bytes, FASTQ bytes) of reads sampled from an iid genome with N-runs."""
    g = synth.add_n_runs(synth.iid(genome_len, seed), 0.002, seed + 1, max_run=20)
    s, q = synth.reads(g, n_reads, read_len, seed + 2)
    return g.tobytes(), synth.fastq_bytes(s, q)


def depth_strings(genome: bytes, k: int) -> list:
    """Depth query strings: the genome, pieces of it with N-runs placed to create segments of
    length < k, == k (the reference's gap-spanning 'stale' windows) and > k, a trailing N-run,
    all-N, shorter than k, empty."""
    g = genome
    N = b"N"
    seg_k = g[100:100 + k]
    pieces = [
        g[:3000],
        g[:200] + N * 3 + seg_k + N * 2 + g[400:700] + N + g[800:800 + k - 3] + N * 4 + g[900:1300],
        seg_k + N + g[2000:2000 + k] + N + g[2100:2100 + k] + N * 2 + g[2200:2300],
        g[500:900] + N * 5,
        g[500:900] + N + g[1000:1000 + k // 2],
        g[500:900] + N + g[1000:1000 + k],
        N * 40,
        g[:k - 1],
        g[:k],
        g[:k + 1],
        b"",
        N * 3 + g[3000:3000 + k] + N * 3,
        g[4000:4300].lower(),
    ]
    return pieces


def materialise(tmpdir: str):
    """(files {name: path}, sim genome) of the golden cases (tests/golden/make_sh_golden.py)."""
    files = {f: os.path.join(GOLDEN, f) for f in REF_FILES}
    for name, data in [("tricky.fq", tricky_fastx()), ("random.fq", random_fastx(400, 1))]:
        p = os.path.join(tmpdir, name)
        open(p, "wb").write(data)
        files[name] = p
    g, fq = sim_reads_fastq(3000, 100, 11)
    p = os.path.join(tmpdir, "sim.fq")
    open(p, "wb").write(fq)
    files["sim.fq"] = p
    return files, g


def load_golden():
    import json
    with open(os.path.join(GOLDEN, "sh_golden.json")) as f:
        return json.load(f)
