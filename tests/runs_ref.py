"""Reference (numpy) of the row gather's diagonal-run format, for the tests: a run is a maximal
stretch of consecutive rows (i, j), (i + 1, j + 1), ...; it travels as {its first row's index,
i, j} (kmhg_rows_runs / kmhg_runs_expand, kmhg_kernels.hip R_count / R_emit / R_expand)."""
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
