"""Reference (numpy) of the multi-GPU wire formats, for the tests.

Rows: a run is a maximal stretch of consecutive rows (i, j), (i + 1, j + 1), ...; it travels as
{its first row's index, i, j} (kmhg_rows_runs / kmhg_runs_expand, kmhg_kernels.hip R_count /
R_emit / R_expand).  Sequences: 16 chars per u32 word of 2-bit codes (c >> 1) & 3 and u16 word
of N flags ((c | 0x20) == 'n'), MSB first; unpacked as "ACTG"[code] or 'N' (kmhg_seq_pack /
kmhg_seq_unpack)."""
import numpy as np
import torch


def encode(rows: np.ndarray) -> np.ndarray:
    """(H, 2) int32 rows -> (n_runs, 3) int32 runs."""
    r = np.asarray(rows, np.int32).reshape(-1, 2)
    if r.shape[0] == 0:
        return np.zeros((0, 3), np.int32)
    u = r.astype(np.int64)
    start = np.ones(r.shape[0], bool)
    start[1:] = ((u[1:, 0] - u[:-1, 0]) % (1 << 32) != 1) | ((u[1:, 1] - u[:-1, 1]) % (1 << 32) != 1)
    idx = np.flatnonzero(start)
    return np.stack([idx.astype(np.int32), r[idx, 0], r[idx, 1]], 1)


def decode(runs: np.ndarray, n_rows: int) -> np.ndarray:
    """(n_runs, 3) runs -> the (n_rows, 2) int32 rows."""
    runs = np.asarray(runs, np.int64).reshape(-1, 3)
    if n_rows == 0:
        return np.zeros((0, 2), np.int32)
    lens = np.diff(np.append(runs[:, 0], n_rows))
    d = np.arange(n_rows) - np.repeat(runs[:, 0], lens)
    out = np.stack([np.repeat(runs[:, 1], lens) + d, np.repeat(runs[:, 2], lens) + d], 1)
    return out.astype(np.int64).astype(np.uint32).view(np.int32).reshape(-1, 2)


class NumpyRunCodec:
    """dist.gather_rows' codec interface over CPU tensors (the gloo tests' stand-in for
    dist.HipRunCodec): runs only where they are smaller than the rows."""

    @staticmethod
    def encode(rows: torch.Tensor):
        runs = encode(rows.numpy())
        return torch.from_numpy(runs) if 3 * runs.shape[0] < 2 * rows.shape[0] else None

    @staticmethod
    def decode(runs: torch.Tensor, n_rows: int, out: torch.Tensor):
        out.copy_(torch.from_numpy(decode(runs.numpy(), n_rows)))


def seq_pack(seq: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """uint8 chars -> (int32 code words, int16 N-flag words), 16 chars each, MSB first; the
    tail padded with 'A'."""
    c = np.asarray(seq, np.uint8)
    L = c.size
    words = (L + 15) // 16
    pad = np.full(words * 16, ord("A"), np.uint8)
    pad[:L] = c
    codes = ((pad >> 1) & 3).astype(np.uint64).reshape(-1, 16)
    isn = ((pad | 0x20) == ord("n")).astype(np.uint64).reshape(-1, 16)
    sh2 = np.uint64(30) - np.arange(16, dtype=np.uint64) * np.uint64(2)
    sh1 = np.uint64(15) - np.arange(16, dtype=np.uint64)
    code = (codes << sh2).sum(1).astype(np.uint32).view(np.int32)
    nbit = (isn << sh1).sum(1).astype(np.uint16).view(np.int16)
    return code, nbit


def seq_unpack(code: np.ndarray, nbit: np.ndarray, word0: int, a: int, b: int,
               out: np.ndarray) -> np.ndarray:
    """chars [a, b) of `out` from the words held from word0 on."""
    if b <= a:
        return out
    lut = np.frombuffer(b"ACTG", np.uint8)
    pos = np.arange(a, b)
    w = pos // 16 - word0
    q = (pos % 16).astype(np.uint32)
    cw = np.asarray(code).view(np.uint32)[w]
    nw = np.asarray(nbit).view(np.uint16)[w].astype(np.uint32)
    ch = lut[(cw >> (np.uint32(30) - 2 * q)) & 3]
    out[a:b] = np.where((nw >> (np.uint32(15) - q)) & 1, np.uint8(ord("N")), ch)
    return out


class NumpySeqCodec:
    """dist's sequence codec over CPU tensors (the gloo tests' stand-in for dist.HipSeqCodec)."""

    @staticmethod
    def pack(seq: torch.Tensor):
        code, nbit = seq_pack(seq.numpy())
        return torch.from_numpy(code), torch.from_numpy(nbit)

    @staticmethod
    def unpack(code: torch.Tensor, nbit: torch.Tensor, word0: int, a: int, b: int,
               out: torch.Tensor):
        seq_unpack(code.numpy(), nbit.numpy(), word0, a, b, out.numpy())
