#!/usr/bin/env python3
"""Generate tests/golden/xxh_golden.json from the REFERENCE's own xxHash.

The digests come from oracle/_ref/libxxhash_ref.so, i.e. the reference's
vendored external/xxhash.c (v0.8.3) compiled unmodified by `make -C oracle ref`
(its page convention: src/storage/page.cpp:18-31).  At generation time every
digest is cross-checked against the system libxxhash (0.8.1) and python-xxhash
(3.8.1 / libxxhash 0.8.2) when those are importable in the build container.

Inputs are synthetic and fully defined by (seed, page index, word index) via
splitmix64 (oracle_splitmix_word / pcs_gen_pages_dev), so the fixture only
stores seeds, sizes and digests.

Run from the repo root:  python tests/golden/gen_golden.py
"""
import ctypes
import ctypes.util
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from workload import splitmix_words, mixed_sizes  # noqa: E402

U64 = ctypes.c_uint64


def load_ref():
    path = os.path.join(ROOT, "oracle", "_ref", "libxxhash_ref.so")
    lib = ctypes.CDLL(path)
    lib.XXH3_64bits.restype = U64
    lib.XXH3_64bits.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    lib.XXH64.restype = U64
    lib.XXH64.argtypes = [ctypes.c_void_p, ctypes.c_size_t, U64]
    lib.XXH_versionNumber.restype = ctypes.c_uint
    return lib


def cross_checkers():
    out = []
    try:
        import xxhash  # third-party, build container only

        out.append(("python-xxhash " + xxhash.VERSION,
                    lambda b: xxhash.xxh3_64_intdigest(b), lambda b: xxhash.xxh64_intdigest(b)))
    except ImportError:
        pass
    name = ctypes.util.find_library("xxhash")
    if name:
        sysl = ctypes.CDLL(name)
        sysl.XXH3_64bits.restype = U64
        sysl.XXH3_64bits.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        sysl.XXH64.restype = U64
        sysl.XXH64.argtypes = [ctypes.c_char_p, ctypes.c_size_t, U64]
        out.append((f"system {name}",
                    lambda b, s=sysl: s.XXH3_64bits(b, len(b)), lambda b, s=sysl: s.XXH64(b, len(b), 0)))
    return out


def main():
    ref = load_ref()
    checks = cross_checkers()

    def h3(b: bytes) -> int:
        v = ref.XXH3_64bits(b, len(b))
        for name, f3, _ in checks:
            assert f3(b) == v, (name, len(b))
        return v

    def h64(b: bytes) -> int:
        v = ref.XXH64(b, len(b), 0)
        for name, _, f64 in checks:
            assert f64(b) == v, (name, len(b))
        return v

    fx = {
        "generator": "tests/golden/gen_golden.py",
        "source": "reference external/xxhash.c compiled by oracle/Makefile (oracle/_ref)",
        "xxh_version_number": int(ref.XXH_versionNumber()),
        "cross_checked_with": [c[0] for c in checks],
        "word_rule": "word w of page p = splitmix64((seed ^ p) + (w+1)*0x9E3779B97F4A7C15)",
    }

    # 1) raw length sweep over one buffer at several start offsets
    seed = 0x5EED0000
    buf = splitmix_words(seed, 0, 8256).tobytes()  # 66048 bytes
    lengths = list(range(0, 1100)) + list(range(1100, 2200, 7)) + [
        2047, 2048, 2049, 3000, 4088, 4095, 4096, 4097, 5000, 8184, 8192, 12345,
        16376, 16384, 32760, 32768, 65528, 65536]
    sweep = []
    for start in (0, 8, 13):
        for L in lengths:
            if start + L > len(buf):
                continue
            b = buf[start:start + L]
            sweep.append([start, L, f"{h3(b):016x}", f"{h64(b):016x}"])
    fx["sweep"] = {"seed": seed, "page_index": 0, "words": 8256, "rows": sweep,
                   "columns": ["start", "len", "xxh3_64", "xxh64_seed0"]}

    # 2) fixed-size pages, page convention over [8, P)
    pages = []
    for P in (256, 512, 768, 1024, 1280, 2048, 3072, 4096, 8192, 16384, 32768, 65536):
        seed = 0x5EED0001
        idx = [0, 1, 2, 3, 4, 5, 6, 7, 1000, 262143]
        rows = []
        for p in idx:
            page = splitmix_words(seed, p, P // 8).tobytes()
            rows.append([p, f"{h3(page[8:]):016x}", f"{h64(page[8:]):016x}"])
        pages.append({"page_size": P, "seed": seed, "rows": rows})
    fx["pages"] = pages

    # 3) config samples (BASELINE.json configs 2, 4, 5)
    samples = []
    for name, seed, P, idx in (
        ("config2_4k", 0x5EED0002, 4096, [0, 1, 2, 3, 4, 511, 4096, 1048575]),
        ("config4_64k", 0x5EED0004, 65536, [0, 1, 262143]),
        ("config5_4k", 0x5EED0005, 4096, [0, 8388607, 8388608, 67108863]),
    ):
        rows = []
        for p in idx:
            page = splitmix_words(seed, p, P // 8).tobytes()
            rows.append([p, f"{h3(page[8:]):016x}", f"{h64(page[8:]):016x}"])
        samples.append({"name": name, "seed": seed, "page_size": P, "rows": rows})
    fx["config_samples"] = samples

    # 4) mixed 4/8/16 KiB pages (config 3): sizes by splitmix, packed contiguously
    seed = 0x5EED0003
    n = 96
    sizes = mixed_sizes(seed, 0, n)
    rows = []
    for i in range(n):
        page = splitmix_words(seed, i, int(sizes[i]) // 8).tobytes()
        rows.append([i, int(sizes[i]), f"{h3(page[8:]):016x}", f"{h64(page[8:]):016x}"])
    fx["mixed"] = {"seed": seed, "rows": rows}

    # 5) manifest CalcChecksum (src/storage/root_meta.cpp:150-174)
    def manifest(content: bytes) -> int:
        agg = 0
        mask = (1 << 64) - 1
        for off in range(0, len(content), 1 << 20):
            h = h3(content[off:off + (1 << 20)])
            agg = (((agg << 1) | (agg >> 63)) & mask) ^ h
            agg = (agg * 0x9E3779B97F4A7C15) & mask
        return agg

    mbuf = splitmix_words(0x5EED0006, 0, (3 << 20) // 8 + 8).tobytes()
    rows = []
    for L in (0, 1, 12, 20, 200, 4096, (1 << 20) - 1, 1 << 20, (1 << 20) + 5, (3 << 20) + 17):
        rows.append([L, f"{manifest(mbuf[:L]):016x}"])
    fx["manifest"] = {"seed": 0x5EED0006, "rows": rows}

    out = os.path.join(ROOT, "tests", "golden", "xxh_golden.json")
    with open(out, "w") as f:
        json.dump(fx, f, indent=0, separators=(",", ":"))
    print("wrote", out, os.path.getsize(out), "bytes;", len(sweep), "sweep rows")


if __name__ == "__main__":
    main()
