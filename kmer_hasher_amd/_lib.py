"""ctypes binding of libkmhgpu.so (the C-ABI declared in include/kmhgpu.h).

The product path has exactly one implementation: the HIP kernels in this shared library.  If the
library is missing or cannot be loaded, every entry point raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkmhgpu.so")
if os.environ.get("KMHG_LIB_VARIANT"):      # A/B experiments only (tools/ab.sh): a variant build
    LIB_PATH = os.path.join(_HERE, f"libkmhgpu_{os.environ['KMHG_LIB_VARIANT']}.so")
HEADER = os.path.join(os.path.dirname(_HERE), "include", "kmhgpu.h")

KMHG_OK, KMHG_EINVAL, KMHG_ENOMEM, KMHG_EDEVICE, KMHG_EOVERFLOW = 0, 1, 2, 3, 4
KMHG_ORDER_FIRST, KMHG_ORDER_KHASH = 0, 1
KMHG_BUILD_GLOBAL, KMHG_BUILD_PARTITIONED, KMHG_BUILD_PARTITIONED_BALLOT = 1, 2, 3


class KmhgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


class Info(C.Structure):
    _fields_ = [("k", C.c_int32), ("device", C.c_int32), ("seq_len", C.c_int64),
                ("n_kmers", C.c_int64), ("n_positions", C.c_int64), ("n_pairs", C.c_int64),
                ("max_count", C.c_int64), ("table_slots", C.c_int64), ("device_bytes", C.c_int64),
                ("sources", C.c_int32), ("kind", C.c_int32), ("kmer_count", C.c_int64),
                ("build", C.c_int32), ("fallback", C.c_int32)]


class ImageSizes(C.Structure):
    _fields_ = [("table_bytes", C.c_int64), ("positions_bytes", C.c_int64),
                ("codes_bytes", C.c_int64)]


_LIB = None
vp = C.c_void_p
i64p = C.POINTER(C.c_int64)

_PROTOS = {
    "kmhg_last_error": (C.c_char_p, []),
    "kmhg_version": (C.c_int, []),
    "kmhg_build": (C.c_int, [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(vp)]),
    "kmhg_build_device": (C.c_int, [vp, C.c_size_t, C.c_int, C.c_int, vp, C.POINTER(vp)]),
    "kmhg_free": (C.c_int, [vp]),
    "kmhg_index_wait": (C.c_int, [vp]),
    "kmhg_index_info": (C.c_int, [vp, C.POINTER(Info)]),
    "kmhg_set_row_order": (C.c_int, [vp, C.c_int]),
    "kmhg_get_row_order": (C.c_int, [vp, C.POINTER(C.c_int)]),
    "kmhg_khash_order": (C.c_int, [vp, C.c_int64, vp]),
    "kmhg_positions_size": (C.c_int, [vp, C.c_uint32, i64p, i64p, i64p, i64p]),
    "kmhg_positions_fill": (C.c_int, [vp, C.c_uint32, vp, vp, vp, vp]),
    "kmhg_positions_fill_device": (C.c_int, [vp, C.c_uint32, vp, vp, vp, vp, vp]),
    "kmhg_query_run": (C.c_int, [vp, C.c_char_p, C.c_size_t, C.c_int, C.POINTER(vp), i64p]),
    "kmhg_query_run_device": (C.c_int, [vp, vp, C.c_size_t, C.c_int, vp, C.POINTER(vp), i64p]),
    "kmhg_query_run_device_range": (C.c_int, [vp, vp, C.c_size_t, C.c_int, C.c_int64, C.c_int64,
                                              vp, C.POINTER(vp), i64p]),
    "kmhg_query_run_device_part": (C.c_int, [vp, vp, C.c_size_t, C.c_int, vp, C.POINTER(vp),
                                             i64p]),
    "kmhg_query_run_device_range_runs": (C.c_int, [vp, vp, C.c_size_t, C.c_int, C.c_int64,
                                                   C.c_int64, vp, vp, i64p, i64p]),
    "kmhg_query_runs_device": (C.c_int, [vp, vp]),
    "kmhg_query_tile_offsets": (C.c_int, [vp, vp, i64p, vp]),
    "kmhg_seq_pack": (C.c_int, [vp, C.c_int64, vp, vp, vp]),
    "kmhg_seq_unpack": (C.c_int, [vp, vp, C.c_int64, C.c_int64, C.c_int64, vp, vp]),
    "kmhg_rows_runs": (C.c_int, [vp, C.c_int64, vp, C.c_int64, i64p, vp]),
    "kmhg_rows_to_host": (C.c_int, [vp, C.c_int64, vp, vp]),
    "kmhg_runs_expand": (C.c_int, [vp, C.c_int64, C.c_int64, vp, vp]),
    "kmhg_merge_part_rows": (C.c_int, [vp, vp, vp, C.c_int, C.c_int64, C.c_int, C.c_int64, vp,
                                       vp]),
    "kmhg_pairs_run": (C.c_int, [vp, vp, C.POINTER(vp), i64p]),
    "kmhg_pairs_run_device": (C.c_int, [vp, vp, vp, C.POINTER(vp), i64p]),
    "kmhg_query_fill": (C.c_int, [vp, vp]),
    "kmhg_query_rows_device": (C.c_int, [vp, C.POINTER(vp)]),
    "kmhg_query_copy_device": (C.c_int, [vp, vp, vp]),
    "kmhg_query_free": (C.c_int, [vp]),
    "kmhg_count": (C.c_int, [C.POINTER(vp), C.POINTER(C.c_char_p), C.POINTER(C.c_size_t),
                             C.c_int64, C.c_int, C.c_int, C.c_int]),
    "kmhg_count_device": (C.c_int, [C.POINTER(vp), vp, C.c_size_t, C.c_int, C.c_int, C.c_int,
                                    vp]),
    "kmhg_sh_count_fastq": (C.c_int, [C.POINTER(vp), C.c_char_p, vp]),
    "kmhg_fastx_read": (C.c_int, [C.c_char_p, C.c_int64, C.c_int, C.POINTER(vp)]),
    "kmhg_reads_info": (C.c_int, [vp, i64p, i64p, i64p]),
    "kmhg_reads_copy": (C.c_int, [vp, vp, vp, vp, vp]),
    "kmhg_reads_free": (C.c_int, [vp]),
    "kmhg_sh_count_reads": (C.c_int, [C.POINTER(vp), vp, vp]),
    "kmhg_sh_count_reads_device": (C.c_int, [C.POINTER(vp), vp, vp, vp, vp, C.c_int64, vp, vp]),
    "kmhg_sh_depth": (C.c_int, [vp, C.c_char_p, C.c_size_t, C.c_int, vp]),
    "kmhg_sh_depth_device": (C.c_int, [vp, vp, C.c_size_t, C.c_int, vp, vp]),
    "kmhg_sh_spectrum": (C.c_int, [vp, C.c_int, vp, vp, C.c_int, vp, C.c_int, vp,
                                   C.POINTER(C.c_int)]),
    "kmhg_counts_export": (C.c_int, [vp, vp, vp]),
    "kmhg_sh_last_batch": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int)]),
    "kmhg_image_sizes_get": (C.c_int, [vp, C.POINTER(ImageSizes), i64p]),
    "kmhg_image_export": (C.c_int, [vp, vp, vp, vp, vp]),
    "kmhg_image_import": (C.c_int, [i64p, vp, vp, vp, vp, C.POINTER(vp)]),
    "kmhg_build_device_part": (C.c_int, [vp, C.c_size_t, C.c_int, C.c_int, C.c_int, vp,
                                         C.POINTER(vp)]),
    "kmhg_part_info": (C.c_int, [vp, i64p]),
    "kmhg_part_export": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp]),
    "kmhg_check_lds_lane_order": (C.c_int, [C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "kmhg_timing_enable": (C.c_int, [C.c_int]),
    "kmhg_timing_select": (C.c_int, [C.c_char_p]),
    "kmhg_timing_reset": (C.c_int, []),
    "kmhg_timing_report": (C.c_int, [C.c_char_p, C.c_size_t]),
    "kmhg_pool_trim": (C.c_int, []),
    "kmhg_pool_cached_bytes": (C.c_int64, []),
}


def header_symbols() -> list[str]:
    """Every function declared in include/kmhgpu.h."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(kmhg_[a-z_]+)\s*\(", txt)))


def _load(path: str):
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    # Load after torch (if present) so both share one HIP runtime (soname libamdhip64.so.7).
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    L = C.CDLL(path)
    for name, (res, args) in _PROTOS.items():
        if os.environ.get("KMHG_LIB_VARIANT") and not hasattr(L, name):
            continue              # an older A/B build may predate an entry point
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


def lib():
    """Load libkmhgpu.so (raises if absent: the HIP path is the only path)."""
    global _LIB
    if _LIB is None:
        _LIB = _load(LIB_PATH)
    return _LIB


TEST_LIB_PATH = os.path.join(_HERE, "libkmhgpu_test.so")
_TEST_LIB = None


class using_test_build:
    """Context in which every entry point goes to libkmhgpu_test.so: the same kernels, with the
    host orchestrator compiled -DKMHG_TEST_BUILD, the only build that reads the path selectors
    and fault injection (kmhg_engine.cpp "Environment knobs").  For the GPU tests that force a
    path; every handle made inside must be freed inside (the two libraries keep separate
    pools)."""

    def __enter__(self):
        global _LIB, _TEST_LIB
        lib()
        if _TEST_LIB is None:
            _TEST_LIB = _load(TEST_LIB_PATH)
        self.prev, _LIB = _LIB, _TEST_LIB
        return _TEST_LIB

    def __exit__(self, *exc):
        global _LIB
        import gc
        gc.collect()                   # handles of the test build die with it
        try:
            _TEST_LIB.kmhg_pool_trim()
        finally:
            _LIB = self.prev
        return False


def check(rc: int) -> None:
    if rc != KMHG_OK:
        msg = lib().kmhg_last_error().decode(errors="replace")
        raise KmhgError(rc, msg)
