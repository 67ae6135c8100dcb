"""Pin the CPU oracle (oracle/xxh_oracle.c) to the reference.

(1) every committed golden vector (generated from the reference's own
    external/xxhash.c by tests/golden/gen_golden.py);
(2) the compiled reference itself (oracle/_ref) on fresh random data, when
    present;
(3) the numpy workload generator against the C generator.
"""
import json
import os

import numpy as np
import pytest

import oracle
from workload import fill_pages, mixed_layout, mixed_sizes, splitmix_words

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "xxh_golden.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


def test_golden_version(golden):
    assert golden["xxh_version_number"] == 803  # external/xxhash.h:548-550 (v0.8.3)


def test_sweep_all_lengths(golden):
    sw = golden["sweep"]
    buf = splitmix_words(sw["seed"], sw["page_index"], sw["words"]).view(np.uint8)
    bad = []
    for start, L, h3, h64 in sw["rows"]:
        b = buf[start:start + L]
        if oracle.xxh3_64(b) != int(h3, 16) or oracle.xxh64(b) != int(h64, 16):
            bad.append((start, L))
    assert not bad, bad[:10]
    assert len(sw["rows"]) > 3000


def test_pages(golden):
    for blk in golden["pages"]:
        P = blk["page_size"]
        for p, h3, h64 in blk["rows"]:
            page = fill_pages(blk["seed"], p, 1, P).reshape(-1)
            assert oracle.pages_digest(page, P, 0)[0] == int(h3, 16), (P, p)
            assert oracle.pages_digest(page, P, 1)[0] == int(h64, 16), (P, p)


def test_config_samples(golden):
    for blk in golden["config_samples"]:
        for p, h3, h64 in blk["rows"]:
            assert oracle.page_digest_sample(blk["seed"], blk["page_size"], p, 0) == int(h3, 16)
            assert oracle.page_digest_sample(blk["seed"], blk["page_size"], p, 1) == int(h64, 16)


def test_mixed(golden):
    mx = golden["mixed"]
    n = len(mx["rows"])
    sizes = mixed_sizes(mx["seed"], 0, n)
    offs, lens, total = mixed_layout(mx["seed"], 0, n)
    buf = np.zeros(total, dtype=np.uint8)
    for i in range(n):
        buf[int(offs[i]):int(offs[i]) + int(lens[i])] = splitmix_words(mx["seed"], i, int(lens[i]) // 8).view(np.uint8)
    d3 = oracle.desc_digest(buf, offs, lens, 0)
    d64 = oracle.desc_digest(buf, offs, lens, 1)
    for i, size, h3, h64 in mx["rows"]:
        assert sizes[i] == size
        assert d3[i] == int(h3, 16) and d64[i] == int(h64, 16)


def test_manifest(golden):
    mf = golden["manifest"]
    longest = max(r[0] for r in mf["rows"])
    buf = splitmix_words(mf["seed"], 0, longest // 8 + 8).view(np.uint8)
    for L, h in mf["rows"]:
        assert oracle.manifest_checksum(buf[:L]) == int(h, 16), L


def test_page_convention_roundtrip():
    # SetChecksum then ValidateChecksum; flip byte 10 (tests/persist.cpp:241-246) -> invalid
    P = 4096
    page = fill_pages(0x1234, 0, 1, P).reshape(-1).copy()
    lib = oracle.lib()
    lib.oracle_set_checksum(page.ctypes.data, P)
    assert lib.oracle_validate_checksum(page.ctypes.data, P) == 1
    assert int(page[:8].view(np.uint64)[0]) == oracle.xxh3_64(page[8:])
    page[10] ^= 0xFF
    assert lib.oracle_validate_checksum(page.ctypes.data, P) == 0


def test_c_generator_matches_numpy():
    for P in (256, 4096):
        a = oracle.fill_pages(P, 5, 0x5EED0002, 77)
        b = fill_pages(0x5EED0002, 77, 5, P).reshape(-1)
        assert np.array_equal(a, b)


@pytest.mark.skipif(oracle.ref_lib() is None, reason="oracle/_ref not built (reference tree absent)")
def test_oracle_vs_compiled_reference_random():
    ref = oracle.ref_lib()
    rng = np.random.default_rng(20261015)
    buf = rng.integers(0, 256, size=70000, dtype=np.uint8)
    lengths = list(range(0, 600)) + list(rng.integers(600, 69000, size=300))
    for L in lengths:
        L = int(L)
        for start in (0, 3):
            b = buf[start:start + L]
            p = b.ctypes.data
            assert oracle.xxh3_64(b) == ref.XXH3_64bits(p, L), L
            assert oracle.xxh64(b, 0) == ref.XXH64(p, L, 0), L
            assert oracle.xxh64(b, 0xDEADBEEF) == ref.XXH64(p, L, 0xDEADBEEF), L


def test_reference_loops_match_oracle_pages_and_mixed():
    """The reference-side per-page loops (oracle/ref_pages.c over the compiled
    external/xxhash.c; bench.py's cpu_baseline) agree with the oracle."""
    if oracle.ref_lib() is None:
        pytest.skip("oracle/_ref not built")
    from workload import fill_desc
    offs, lens, total = mixed_layout(0x5EED0003, 0, 2000)
    host = fill_desc(0x5EED0003, 0, offs, lens, total)
    pages = fill_pages(0x5EED0002, 0, 300, 4096).reshape(-1)
    for algo in (0, 1):
        assert np.array_equal(oracle.ref_desc_digest(host, offs, lens, algo), oracle.desc_digest(host, offs, lens, algo))
        assert np.array_equal(oracle.ref_pages_digest(pages, 4096, algo), oracle.pages_digest(pages, 4096, algo))
