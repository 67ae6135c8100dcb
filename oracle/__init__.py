"""oracle — TEST INFRASTRUCTURE ONLY.

ctypes binding of the CPU restatement (oracle/liboracle.so, from
xxh_oracle.c) and of the reference's own xxHash compiled in place
(oracle/_ref/libxxhash_ref.so, see oracle/Makefile).  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg — always as the
checker or the CPU baseline, never as the measured or shipped path.

Parity pinning: the restatement is checked against the committed golden
vectors (tests/golden/xxh_golden.json, generated from the compiled reference
by tests/golden/gen_golden.py) and, where oracle/_ref exists, against the
reference library directly (tests/test_oracle.py).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libxxhash_ref.so")

_u64, _sz, _vp = ctypes.c_uint64, ctypes.c_size_t, ctypes.c_void_p
_oracle = None
_ref = None


def build(ref: bool = True) -> None:
    """Compile liboracle.so (and _ref when /root/reference is present)."""
    subprocess.run(["make", "-C", HERE, "-s", "ref" if ref else "all"], check=True)


def lib() -> ctypes.CDLL:
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            build(ref=False)
        so = ctypes.CDLL(ORACLE_SO)
        sig = {
            "oracle_xxh3_64": ([_vp, _sz], _u64),
            "oracle_xxh64": ([_vp, _sz, _u64], _u64),
            "oracle_page_xxh3": ([_vp, _sz], _u64),
            "oracle_page_xxh64": ([_vp, _sz], _u64),
            "oracle_set_checksum": ([_vp, _sz], None),
            "oracle_validate_checksum": ([_vp, _sz], ctypes.c_int),
            "oracle_manifest_checksum": ([_vp, _sz], _u64),
            "oracle_pages_digest": ([_vp, _sz, _sz, ctypes.c_int, _vp], None),
            "oracle_desc_digest": ([_vp, _vp, _vp, _sz, ctypes.c_int, _vp], None),
            "oracle_desc_raw_xxh3": ([_vp, _vp, _vp, _sz, _vp], None),
            "oracle_fill_pages": ([_vp, _sz, _sz, _u64, _u64], None),
            "oracle_splitmix_word": ([_u64, _u64, _u64], _u64),
        }
        for name, (args, res) in sig.items():
            f = getattr(so, name)
            f.argtypes, f.restype = args, res
        _oracle = so
    return _oracle


def ref_lib():
    """The reference's external/xxhash.c compiled in place, or None."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        so = ctypes.CDLL(REF_SO)
        so.XXH3_64bits.argtypes, so.XXH3_64bits.restype = [_vp, _sz], _u64
        so.XXH64.argtypes, so.XXH64.restype = [_vp, _sz, _u64], _u64
        so.XXH_versionNumber.restype = ctypes.c_uint
        so.ref_pages_digest.argtypes = [_vp, _sz, _sz, ctypes.c_int, _vp]
        so.ref_pages_digest.restype = None
        if hasattr(so, "ref_scan_file"):
            so.ref_scan_file.argtypes = [ctypes.c_char_p, _sz, _u64, _u64, _vp]
            so.ref_scan_file.restype = ctypes.c_longlong
        if hasattr(so, "ref_desc_digest"):
            so.ref_desc_digest.argtypes = [_vp, _vp, _vp, _sz, ctypes.c_int, _vp]
            so.ref_desc_digest.restype = None
        _ref = so
    return _ref


def _buf(b):
    a = np.frombuffer(b, dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.ascontiguousarray(b)
    return a, a.ctypes.data


def xxh3_64(data) -> int:
    a, p = _buf(data)
    return lib().oracle_xxh3_64(p, a.nbytes)


def xxh64(data, seed: int = 0) -> int:
    a, p = _buf(data)
    return lib().oracle_xxh64(p, a.nbytes, seed)


def manifest_checksum(data) -> int:
    a, p = _buf(data)
    return lib().oracle_manifest_checksum(p, a.nbytes)


def pages_digest(pages: np.ndarray, page_size: int, algo: int = 0) -> np.ndarray:
    """pages: contiguous uint8 array of n * page_size bytes."""
    pages = np.ascontiguousarray(pages)
    n = pages.nbytes // page_size
    out = np.empty(n, dtype=np.uint64)
    lib().oracle_pages_digest(pages.ctypes.data, page_size, n, algo, out.ctypes.data)
    return out


def desc_digest(base: np.ndarray, off: np.ndarray, length: np.ndarray, algo: int = 0) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty(len(off), dtype=np.uint64)
    lib().oracle_desc_digest(base.ctypes.data, off.ctypes.data, length.ctypes.data, len(off), algo, out.ctypes.data)
    return out


def desc_raw_xxh3(base: np.ndarray, off: np.ndarray, length: np.ndarray) -> np.ndarray:
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty(len(off), dtype=np.uint64)
    lib().oracle_desc_raw_xxh3(base.ctypes.data, off.ctypes.data, length.ctypes.data, len(off), out.ctypes.data)
    return out


def ref_pages_digest(pages: np.ndarray, page_size: int, algo: int = 0) -> np.ndarray:
    """Reference xxHash, one call per page (page.cpp:18-31), or None without _ref."""
    ref = ref_lib()
    if ref is None:
        return None
    pages = np.ascontiguousarray(pages)
    n = pages.nbytes // page_size
    out = np.empty(n, dtype=np.uint64)
    ref.ref_pages_digest(pages.ctypes.data, page_size, n, algo, out.ctypes.data)
    return out


def ref_desc_digest(base: np.ndarray, off: np.ndarray, length: np.ndarray, algo: int = 0):
    """Reference xxHash over mixed-size pages, one call per page, or None without _ref."""
    ref = ref_lib()
    if ref is None or not hasattr(ref, "ref_desc_digest"):
        return None
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    out = np.empty(len(off), dtype=np.uint64)
    ref.ref_desc_digest(base.ctypes.data, off.ctypes.data, length.ctypes.data, len(off), algo, out.ctypes.data)
    return out


def fill_pages(page_size: int, n: int, seed: int, first_page: int = 0) -> np.ndarray:
    out = np.empty(n * page_size, dtype=np.uint8)
    lib().oracle_fill_pages(out.ctypes.data, page_size, n, seed, first_page)
    return out


def page_digest_sample(seed: int, page_size: int, page_index: int, algo: int = 0) -> int:
    """Digest of synthetic page `page_index` (generator rule shared with pcs_gen_pages_dev)."""
    page = fill_pages(page_size, 1, seed, page_index)
    return int(pages_digest(page, page_size, algo)[0])


def ref_scan_file(path: str, page_size: int, first_page: int, n_pages: int):
    """Config 1: the reference's per-page read + ValidateChecksum loop over a
    file range on the calling thread (oracle/ref_pages.c).  Returns (bytes read,
    failing pages), or None without _ref.  ctypes drops the GIL for the call,
    so Python threads scanning disjoint ranges run in parallel."""
    ref = ref_lib()
    if ref is None or not hasattr(ref, "ref_scan_file"):
        return None
    bad = ctypes.c_uint64(0)
    got = ref.ref_scan_file(path.encode(), page_size, first_page, n_pages, ctypes.byref(bad))
    if got < 0:
        raise OSError(f"ref_scan_file failed on {path}")
    return int(got), int(bad.value)
