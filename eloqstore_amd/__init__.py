"""eloqstore_amd — Python binding of the MI355X page-checksum engine.

The product is the native library ``libeloqstore_pcs.so`` (HIP kernels for
gfx950 + C ABI declared in ``include/eloqstore_pcs.h`` + the C++ drop-in
``include/eloqstore/page_checksum.h``).  This module is the thin ctypes layer
the tests and ``bench.py`` drive it through; device memory and streams come
from PyTorch (plumbing only).  There is no CPU fallback: every compute call
raises ``PcsError`` when the library or the GPU is unavailable.

Mirrors the reference call surface (src/storage/page.cpp:18-31):
``set_checksum`` / ``validate_checksum`` on one host page, plus batched
device and host forms.
"""
from __future__ import annotations

import ctypes
import os
import re

import numpy as np

import torch  # noqa: F401  (loads the process's HIP runtime before the library)

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libeloqstore_pcs.so")
DROPIN_LIB_PATH = os.path.join(HERE, "libeloqstore_pcs_dropin.so")  # opt-in single-page C++ symbols
TOOL_PATH = os.path.join(HERE, "page_checksum_tool")
HEADER_PATH = os.path.join(ROOT, "include", "eloqstore_pcs.h")

XXH3_64 = 0
XXH64 = 1
PCS_OK = 0
PCS_ERR_INVALID = -1
PCS_ERR_NO_DEVICE = -2
PCS_ERR_HIP = -3
PCS_ERR_NOMEM = -4

_u64, _u32, _i32, _vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
_P = ctypes.POINTER

# name -> argtypes (restype int unless listed in _STR)
_SIGS = {
    "pcs_device_count": [_P(_i32)],
    "pcs_set_device": [_i32],
    "pcs_synchronize": [_vp],
    "pcs_pages_digest_dev": [_vp, _u64, _u64, _i32, _vp, _vp],
    "pcs_pages_validate_dev": [_vp, _u64, _u64, _i32, _vp, _vp, _vp],
    "pcs_pages_stamp_dev": [_vp, _u64, _u64, _i32, _vp],
    "pcs_desc_digest_dev": [_vp, _vp, _vp, _u64, _i32, _vp, _vp],
    "pcs_desc_validate_dev": [_vp, _vp, _vp, _u64, _i32, _vp, _vp, _vp],
    "pcs_desc_stamp_dev": [_vp, _vp, _vp, _u64, _i32, _vp],
    "pcs_xxh3_64_ranges_dev": [_vp, _vp, _vp, _u64, _vp, _vp],
    "pcs_xxh64_ranges_dev": [_vp, _vp, _vp, _u64, _u64, _vp, _vp],
    "pcs_pages_validate_host": [_vp, _u64, _u64, _i32, _vp, _vp],
    "pcs_pages_validate_host_ex": [_vp, _u64, _u64, _i32, _vp, _vp, _u32],
    "pcs_pages_stamp_host": [_vp, _u64, _u64, _i32],
    "pcs_pages_digest_host": [_vp, _u64, _u64, _i32, _vp],
    "pcs_shard_range": [_u64, _i32, _i32, _P(_u64), _P(_u64)],
    "pcs_gen_pages_dev": [_vp, _u64, _u64, _u64, _u64, _vp],
    "pcs_gen_desc_dev": [_vp, _vp, _vp, _u64, _u64, _u64, _vp],
    "pcs_flip_byte_dev": [_vp, _u64, _u64, _u64, _u64, _vp],
    "pcs_stream_read_dev": [_vp, _u64, _vp, _vp],
    "pcs_host_alloc_pinned": [_u64, _P(_vp)],
    "pcs_host_free_pinned": [_vp],
    "pcs_host_register": [_vp, _u64],
    "pcs_host_unregister": [_vp],
    "pcs_batch_create": [_P(_vp)],
    "pcs_batch_submit": [_vp, _i32, _vp, _u64, _u64, _i32],
    "pcs_batch_submit_ex": [_vp, _i32, _vp, _u64, _u64, _i32, _u32],
    "pcs_batch_poll": [_vp],
    "pcs_batch_wait": [_vp],
    "pcs_batch_result": [_vp, _vp, _vp, _vp],
    "pcs_batch_destroy": [_vp],
    "pcs_manifest_checksum_dev": [_vp, _u64, _vp, _vp],
    "pcs_manifest_checksum_host": [_vp, _u64, _P(_u64)],
    "pcs_manifest_validate_host": [_vp, _u64, _P(_i32)],
    "pcs_set_tuning": [_i32, ctypes.c_int64],
    "pcs_get_tuning": [_i32],
    "pcs_counter": [_i32],
    "pcs_service_start": [_i32, _u32],
    "pcs_service_start_ex": [_i32, _i32, _u32],
    "pcs_service_stop": [],
    "pcs_service_running": [],
    "pcs_last_path": [],
    "pcs_thread_prepare": [],
    "pcs_batch_path": [_vp],
    "pcs_version": [],
    "pcs_abi_version": [],
    "pcs_last_error": [],
}
_STR = {"pcs_version", "pcs_last_error"}
_I64 = {"pcs_get_tuning", "pcs_counter"}


class PcsError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_lib = None


def lib() -> ctypes.CDLL:
    """Load libeloqstore_pcs.so (built by __graft_entry__.build())."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PcsError("load", PCS_ERR_NO_DEVICE,
                           f"{LIB_PATH} missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        so = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            f = getattr(so, name)
            f.argtypes = args
            f.restype = ctypes.c_char_p if name in _STR else ctypes.c_int64 if name in _I64 else ctypes.c_int
        _lib = so
    return _lib


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Every pcs_* function declared in the public C header."""
    with open(path) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(pcs_[a-z0-9_]+)\s*\(", text)))


def _check(fn: str, rc: int) -> None:
    if rc != PCS_OK:
        raise PcsError(fn, rc, lib().pcs_last_error().decode(errors="replace"))


def _call(fn: str, *args) -> None:
    _check(fn, getattr(lib(), fn)(*args))


def _ptr(t) -> int:
    if t is None:
        return 0
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _stream(stream) -> int:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


TUNE_XXH3_BLOCKS_PER_CU = 1
TUNE_XXH64_BLOCKS_PER_CU = 2
TUNE_NT_LOADS = 3
TUNE_XXH64_LAYOUT = 6
TUNE_ZERO_COPY = 7
TUNE_XXH3_RT_BATCH = 8
TUNE_XXH3_SPLIT_PAGES = 9
TUNE_INLINE_LIST = 11
TUNE_MANIFEST_WIDE = 13
TUNE_XXH64_WAVES = 15
TUNE_ZC_POLL = 23
TUNE_SERVICE_STREAM = 24
TUNE_SERVICE_TEAR_TEST = 26  # test only
TUNE_FAIL_INJECT = 27  # test only
TUNE_SERVICE_MAX_CALLERS = 28
TUNE_SERVICE_REPOST_TEST = 30  # test only
TUNE_ZC_STAMP_POLL_PAGES = 31
TUNE_SERVICE_SLOW_EXIT_TEST = 33  # test only
TUNE_ZC_BATCH_EVENT = 34
TUNE_SYNC_SPIN_US = 35
TUNE_SERVICE_DEPARTURE = 36

# PCS_PATH_* bits (pcs_last_path / pcs_batch_path)
PATH_SERVED = 1
PATH_LAUNCHED = 2
PATH_FALLBACK = 4
PATH_REPOSTED = 8
PATH_NEW_GENERATION = 16
PATH_LOCK_SKIPPED = 32

COUNTER_ZERO_COPY_LAUNCHES = 0
COUNTER_DIRECT_DMA_CHUNKS = 1
COUNTER_GATHER_CHUNKS = 2
COUNTER_SERVICE_BATCHES = 3
COUNTER_SERVICE_TORN_REQUESTS = 4
COUNTER_SERVICE_REPOSTS = 5


def counter(which: int) -> int:
    """pcs_counter: how host batches were served (process-wide, monotonic)."""
    return int(lib().pcs_counter(which))


def set_tuning(key: int, value: int) -> None:
    _call("pcs_set_tuning", key, value)


def get_tuning(key: int) -> int:
    return int(lib().pcs_get_tuning(key))


def version() -> str:
    return lib().pcs_version().decode()


ABI_VERSION = 6  # PCS_ABI_VERSION of include/eloqstore_pcs.h this binding was written for


def abi_version() -> int:
    return int(lib().pcs_abi_version())


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().pcs_device_count(ctypes.byref(n))
    return n.value if rc == PCS_OK else 0


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    b, e = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _call("pcs_shard_range", n, world, rank, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


# ---- device-resident batches (torch tensors on cuda) ------------------------

def pages_digest(pages, page_size: int, n: int, algo: int = XXH3_64, out=None, stream=None):
    """digests[i] = hash of page i over [8, page_size); pages: uint8 device tensor."""
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=pages.device)
    _call("pcs_pages_digest_dev", _ptr(pages), page_size, n, algo, _ptr(out), _stream(stream))
    return out


def pages_validate(pages, page_size: int, n: int, algo: int = XXH3_64, ok=None, first_bad=None, stream=None):
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=pages.device)
    if first_bad is None:
        first_bad = torch.empty(1, dtype=torch.int64, device=pages.device)
    _call("pcs_pages_validate_dev", _ptr(pages), page_size, n, algo, _ptr(ok), _ptr(first_bad), _stream(stream))
    return ok, first_bad


def pages_stamp(pages, page_size: int, n: int, algo: int = XXH3_64, stream=None) -> None:
    _call("pcs_pages_stamp_dev", _ptr(pages), page_size, n, algo, _stream(stream))


def desc_digest(base, off, length, n: int, algo: int = XXH3_64, out=None, stream=None):
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=base.device)
    _call("pcs_desc_digest_dev", _ptr(base), _ptr(off), _ptr(length), n, algo, _ptr(out), _stream(stream))
    return out


def desc_validate(base, off, length, n: int, algo: int = XXH3_64, ok=None, first_bad=None, stream=None):
    if ok is None:
        ok = torch.empty(n, dtype=torch.uint8, device=base.device)
    if first_bad is None:
        first_bad = torch.empty(1, dtype=torch.int64, device=base.device)
    _call("pcs_desc_validate_dev", _ptr(base), _ptr(off), _ptr(length), n, algo, _ptr(ok), _ptr(first_bad),
          _stream(stream))
    return ok, first_bad


def desc_stamp(base, off, length, n: int, algo: int = XXH3_64, stream=None) -> None:
    _call("pcs_desc_stamp_dev", _ptr(base), _ptr(off), _ptr(length), n, algo, _stream(stream))


def xxh3_64_ranges(base, off, length, n: int, out=None, stream=None):
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=base.device)
    _call("pcs_xxh3_64_ranges_dev", _ptr(base), _ptr(off), _ptr(length), n, _ptr(out), _stream(stream))
    return out


def xxh64_ranges(base, off, length, n: int, seed: int = 0, out=None, stream=None):
    if out is None:
        out = torch.empty(n, dtype=torch.int64, device=base.device)
    _call("pcs_xxh64_ranges_dev", _ptr(base), _ptr(off), _ptr(length), n, seed, _ptr(out), _stream(stream))
    return out


def gen_pages(pages, page_size: int, n: int, seed: int, first_page: int = 0, stream=None) -> None:
    _call("pcs_gen_pages_dev", _ptr(pages), page_size, n, seed, first_page, _stream(stream))


def gen_desc(base, off, length, n: int, seed: int, first_page: int = 0, stream=None) -> None:
    _call("pcs_gen_desc_dev", _ptr(base), _ptr(off), _ptr(length), n, seed, first_page, _stream(stream))


def flip_byte(pages, page_size: int, n: int, every: int, byte_offset: int = 10, stream=None) -> None:
    _call("pcs_flip_byte_dev", _ptr(pages), page_size, n, every, byte_offset, _stream(stream))


def stream_read(buf, nbytes: int, out, stream=None) -> None:
    """pcs_stream_read_dev: plain streaming read of nbytes (the read ceiling);
    out receives one folded u64 per 4 KiB page (ceil(nbytes / 4096) words)."""
    _call("pcs_stream_read_dev", _ptr(buf), nbytes, _ptr(out), _stream(stream))


def manifest_checksum_host(content: bytes) -> int:
    """ManifestBuilder::CalcChecksum (root_meta.cpp:150-174) on the GPU."""
    buf = (ctypes.c_char * max(1, len(content))).from_buffer_copy(content or b"\0")
    out = ctypes.c_uint64(0)
    _call("pcs_manifest_checksum_host", buf, len(content), ctypes.byref(out))
    return out.value


def manifest_validate_host(record: bytes) -> bool:
    buf = (ctypes.c_char * max(1, len(record))).from_buffer_copy(record or b"\0")
    v = ctypes.c_int(0)
    _call("pcs_manifest_validate_host", buf, len(record), ctypes.byref(v))
    return bool(v.value)


class Batch:
    """Asynchronous host batch (pcs_batch_*): submit, poll without blocking, read results."""

    DIGEST, VALIDATE, STAMP = 0, 1, 2

    def __init__(self):
        self._b = ctypes.c_void_p()
        _call("pcs_batch_create", ctypes.byref(self._b))
        self._keep = None
        self.n = 0

    def submit(self, mode: int, pages: list, page_size: int, algo: int = XXH3_64, skip_verify: bool = False) -> None:
        arr, keep = _page_ptrs(pages)
        self._keep = (arr, keep)
        self.n = len(pages)
        self.mode = mode
        _call("pcs_batch_submit_ex", self._b, mode, arr, page_size, len(pages), algo, _flags(skip_verify))

    def submit_ptrs(self, mode: int, ptrs, page_size: int, algo: int = XXH3_64, skip_verify: bool = False) -> None:
        """Submit raw page addresses (a uint64 array of host pointers)."""
        ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
        self._keep = ptrs
        self.n = len(ptrs)
        self.mode = mode
        _call("pcs_batch_submit_ex", self._b, mode, ptrs.ctypes.data, page_size, len(ptrs), algo,
              _flags(skip_verify))

    def poll(self) -> bool:
        rc = lib().pcs_batch_poll(self._b)
        if rc < 0:
            _check("pcs_batch_poll", rc)
        return rc == 1

    def wait(self) -> None:
        _call("pcs_batch_wait", self._b)

    def path(self) -> int:
        """PCS_PATH_* bits of the last submission (which path served it)."""
        return int(lib().pcs_batch_path(self._b))

    def result(self):
        fb = ctypes.c_uint64(0)
        if self.mode == self.VALIDATE:
            ok = (ctypes.c_uint8 * max(1, self.n))()
            _call("pcs_batch_result", self._b, ok, None, ctypes.byref(fb))
            return list(ok)[: self.n], (None if fb.value == (1 << 64) - 1 else fb.value)
        dig = (ctypes.c_uint64 * max(1, self.n))()
        _call("pcs_batch_result", self._b, None, dig, ctypes.byref(fb))
        return list(dig)[: self.n]

    def close(self) -> None:
        if self._b:
            lib().pcs_batch_destroy(self._b)
            self._b = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- host-memory forms (reference call surface) ------------------------------

FLAG_NONE, FLAG_SKIP_VERIFY = 0, 1  # pcs_flags


def _flags(skip_verify: bool) -> int:
    """KvOptions::skip_verify_checksum (kv_options.h:41) -> PCS_FLAG_SKIP_VERIFY."""
    return FLAG_SKIP_VERIFY if skip_verify else FLAG_NONE


def _page_ptrs(pages: list) -> tuple:
    bufs = [p if isinstance(p, ctypes.Array) else (ctypes.c_char * len(p)).from_buffer(p) for p in pages]
    arr = (ctypes.c_void_p * len(bufs))(*[ctypes.addressof(b) for b in bufs])
    return arr, bufs


def set_checksum(page: bytearray) -> None:
    """eloqstore::SetChecksum (page.cpp:18-23) on one writable host page."""
    arr, _keep = _page_ptrs([page])
    _call("pcs_pages_stamp_host", arr, len(page), 1, XXH3_64)


def validate_checksum(page) -> bool:
    """eloqstore::ValidateChecksum (page.cpp:25-31) on one host page."""
    buf = page if isinstance(page, bytearray) else bytearray(page)
    arr, _keep = _page_ptrs([buf])
    ok = (ctypes.c_uint8 * 1)()
    _call("pcs_pages_validate_host", arr, len(buf), 1, XXH3_64, ok, None)
    return bool(ok[0])


def validate_checksums(pages: list, page_size: int, algo: int = XXH3_64, skip_verify: bool = False):
    """Batched ValidateChecksum over scattered host pages -> (ok list, first_bad or None)."""
    arr, _keep = _page_ptrs(pages)
    ok = (ctypes.c_uint8 * max(1, len(pages)))()
    fb = ctypes.c_uint64(0)
    _call("pcs_pages_validate_host_ex", arr, page_size, len(pages), algo, ok, ctypes.byref(fb),
          _flags(skip_verify))
    return list(ok), (None if fb.value == (1 << 64) - 1 else fb.value)


def set_checksums(pages: list, page_size: int, algo: int = XXH3_64) -> None:
    arr, _keep = _page_ptrs(pages)
    _call("pcs_pages_stamp_host", arr, page_size, len(pages), algo)


def page_digests_host(pages: list, page_size: int, algo: int = XXH3_64) -> list:
    arr, _keep = _page_ptrs(pages)
    out = (ctypes.c_uint64 * len(pages))()
    _call("pcs_pages_digest_host", arr, page_size, len(pages), algo, out)
    return list(out)


# ---- raw pointer arrays and registered page pools -----------------------------

def host_register(addr: int, nbytes: int) -> None:
    """pcs_host_register: page-lock + map a host region for zero-copy batches."""
    _call("pcs_host_register", addr, nbytes)


def host_unregister(addr: int) -> None:
    _call("pcs_host_unregister", addr)


def validate_ptrs(ptrs, page_size: int, algo: int = XXH3_64, skip_verify: bool = False):
    """pcs_pages_validate_host_ex over raw host page addresses -> (ok array, first_bad or None)."""
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    ok = np.zeros(max(1, len(ptrs)), dtype=np.uint8)
    fb = ctypes.c_uint64(0)
    _call("pcs_pages_validate_host_ex", ptrs.ctypes.data, page_size, len(ptrs), algo, ok.ctypes.data,
          ctypes.byref(fb), _flags(skip_verify))
    return ok[: len(ptrs)], (None if fb.value == (1 << 64) - 1 else fb.value)


def stamp_ptrs(ptrs, page_size: int, algo: int = XXH3_64) -> None:
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    _call("pcs_pages_stamp_host", ptrs.ctypes.data, page_size, len(ptrs), algo)


def digest_ptrs(ptrs, page_size: int, algo: int = XXH3_64) -> np.ndarray:
    ptrs = np.ascontiguousarray(ptrs, dtype=np.uint64)
    out = np.zeros(max(1, len(ptrs)), dtype=np.uint64)
    _call("pcs_pages_digest_host", ptrs.ctypes.data, page_size, len(ptrs), algo, out.ctypes.data)
    return out[: len(ptrs)]


class ValidateService:
    """pcs_service_start / pcs_service_stop as a context manager: while it is
    open, validate_ptrs / validate_checksums batches of up to 256 registered
    XXH3 pages go to a resident kernel instead of a launch each."""

    def __init__(self, workgroups: int = 4, idle_us: int = 1000, lines: int = 1):
        self.workgroups, self.idle_us, self.lines = workgroups, idle_us, lines

    def __enter__(self):
        _call("pcs_service_start_ex", self.lines, self.workgroups, self.idle_us)
        return self

    def __exit__(self, *exc):
        _call("pcs_service_stop")


class PagePool:
    """A page-aligned host region of n_pages x page_size, like one chunk of
    EloqStore's PagesPool (page.cpp:95-120), registered for zero-copy batches.
    `.pages` is a (n_pages, page_size) uint8 view; `.ptr(i)` a page address."""

    def __init__(self, n_pages: int, page_size: int, register: bool = True):
        import mmap
        self.n, self.P = n_pages, page_size
        self._map = mmap.mmap(-1, max(1, n_pages * page_size))
        self.pages = np.frombuffer(self._map, dtype=np.uint8)[: n_pages * page_size].reshape(n_pages, page_size)
        self.base = self.pages.ctypes.data
        self.registered = False
        if register:
            host_register(self.base, n_pages * page_size)
            self.registered = True

    def ptr(self, i) -> np.ndarray:
        return np.uint64(self.base) + np.asarray(i, dtype=np.uint64) * np.uint64(self.P)

    def close(self) -> None:
        if self.registered:
            host_unregister(self.base)
            self.registered = False
        self.pages = None
        if self._map is not None:
            try:
                self._map.close()
            except BufferError:  # a view is still alive; let GC unmap it
                pass
            self._map = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
