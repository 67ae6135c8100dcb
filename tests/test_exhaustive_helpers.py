"""CPU check of test_gpu_exhaustive.py's host-side checker: chunked copies and
16-thread hashing return exactly the oracle's digest of every page, whatever
the chunk size (smaller than a page, page-aligned or not)."""
import concurrent.futures as cf

import numpy as np
import pytest
import torch

import oracle
import test_gpu_exhaustive as ex
from workload import fill_desc, mixed_layout


@pytest.fixture(scope="module")
def pool():
    with cf.ThreadPoolExecutor(ex.THREADS) as p:
        yield p


@pytest.mark.parametrize("chunk", [1000, 4096 * 7 + 5, 1 << 20])
@pytest.mark.parametrize("algo", [0, 1])
def test_desc_reference_chunked(pool, monkeypatch, chunk, algo):
    monkeypatch.setattr(ex, "CHUNK", chunk)
    n = 700
    offs, lens, total = mixed_layout(0x5EED0003, 123, n)
    host = fill_desc(0x5EED0003, 123, offs, lens, total)
    got = ex.desc_reference(pool, torch.from_numpy(host), offs, lens, algo)
    assert np.array_equal(got, oracle.desc_digest(host, offs, lens, algo))


@pytest.mark.parametrize("P,n", [(4096, 300), (65536, 21), (8192, 1)])
@pytest.mark.parametrize("chunk", [100, 4096 * 5 + 3, 1 << 20])
def test_fixed_reference_chunked(pool, monkeypatch, P, n, chunk):
    monkeypatch.setattr(ex, "CHUNK", chunk)
    pages = oracle.fill_pages(P, n, 0x5EED0002, 99)
    for algo in (0, 1):
        got = ex.fixed_reference(pool, torch.from_numpy(pages), P, n, algo)
        assert np.array_equal(got, oracle.pages_digest(pages, P, algo))
