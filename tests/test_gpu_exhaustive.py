"""Exhaustive parity at BASELINE's full sizes: EVERY digest of configs 2, 3
(XXH3 and XXH64), 4 and 5 (rank 7's shard of the 8-GPU run), computed by the
HIP kernels through the C ABI, equals the reference's own xxHash
(`external/xxhash.c` v0.8.3 compiled in place as oracle/_ref, one call per
page as page.cpp:18-31 makes it) -- or the repo's C restatement where _ref was
not built.  The pages are copied to the host in 1 GiB chunks and hashed there
by 16 threads (ctypes drops the GIL), so config 5's 32 GiB takes seconds.

Then, on the same full batch, the write and read paths: every header the
stamp kernel wrote equals the checker's digest, every page validates, and
after byte 10 of every 1000th page is flipped (persist.cpp:241-246) exactly
those pages fail, with first_bad = 0.  (test_gpu_parity.py's full-size tests
sample digests; this file checks all of them.)
"""
import concurrent.futures as cf

import numpy as np
import pytest
import torch

import eloqstore_amd as pcs
import oracle
from workload import mixed_layout

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
CHUNK = 1 << 30  # host bytes per copy
THREADS = 16     # the GPU box's CPU share


@pytest.fixture(scope="module", autouse=True)
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    yield
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def pool():
    with cf.ThreadPoolExecutor(THREADS) as ex:
        yield ex


def checker():
    """'reference' when oracle/_ref is present (it travels with the tree),
    else 'oracle' (the restatement, pinned against the reference's goldens)."""
    return "reference" if oracle.ref_lib() is not None else "oracle"


def host_pages_digest(pool, pages: np.ndarray, P: int, algo: int) -> np.ndarray:
    n = pages.nbytes // P
    parts = np.array_split(np.arange(n), THREADS)
    fn = oracle.ref_pages_digest if checker() == "reference" else oracle.pages_digest

    def run(idx):
        if len(idx) == 0:
            return np.empty(0, dtype=np.uint64)
        return fn(pages[int(idx[0]) * P:(int(idx[-1]) + 1) * P], P, algo)

    return np.concatenate(list(pool.map(run, parts)))


def host_desc_digest(pool, base: np.ndarray, offs: np.ndarray, lens: np.ndarray, algo: int) -> np.ndarray:
    parts = np.array_split(np.arange(len(offs)), THREADS)
    fn = oracle.ref_desc_digest if checker() == "reference" else oracle.desc_digest

    def run(idx):
        if len(idx) == 0:
            return np.empty(0, dtype=np.uint64)
        return fn(base, offs[idx], lens[idx], algo)

    return np.concatenate(list(pool.map(run, parts)))


def fixed_reference(pool, buf: torch.Tensor, P: int, n: int, algo: int) -> np.ndarray:
    """The checker's digest of every page of a device-resident fixed-size batch."""
    per = max(1, CHUNK // P)
    out = []
    for i0 in range(0, n, per):
        i1 = min(n, i0 + per)
        host = buf[i0 * P:i1 * P].cpu().numpy()
        out.append(host_pages_digest(pool, host, P, algo))
    return np.concatenate(out)


def desc_reference(pool, base: torch.Tensor, offs: np.ndarray, lens: np.ndarray, algo: int) -> np.ndarray:
    """The checker's digest of every page of a packed descriptor batch."""
    n = len(offs)
    out = []
    i0 = 0
    while i0 < n:
        lo = int(offs[i0])
        i1 = int(np.searchsorted(offs, lo + CHUNK, side="left"))
        i1 = max(i0 + 1, min(n, i1))
        while i1 > i0 + 1 and int(offs[i1 - 1]) + int(lens[i1 - 1]) - lo > CHUNK:
            i1 -= 1
        hi = int(offs[i1 - 1]) + int(lens[i1 - 1])
        host = base[lo:hi].cpu().numpy()
        out.append(host_desc_digest(pool, host, offs[i0:i1] - np.uint64(lo), lens[i0:i1], algo))
        i0 = i1
    return np.concatenate(out)


def u64(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def headers(buf: torch.Tensor, P: int, n: int) -> np.ndarray:
    return u64(buf.view(-1, P)[:n, :8].contiguous().view(torch.int64).reshape(-1))


@pytest.mark.parametrize("cfg,P,n,seed,first,algo", [
    (2, 4096, 1 << 20, 0x5EED0002, 0, pcs.XXH3_64),              # the metric's batch
    (4, 65536, 1 << 18, 0x5EED0004, 0, pcs.XXH3_64),             # 16 GiB of 64 KiB chunks
    (5, 4096, 1 << 23, 0x5EED0005, 7 << 23, pcs.XXH3_64),        # 32 GiB: rank 7's shard of 64 M pages
    (2, 4096, 1 << 20, 0x5EED0002, 0, pcs.XXH64),                # the XXH64 LDS kernel at config 2's shape
])
def test_every_digest_fixed(pool, cfg, P, n, seed, first, algo):
    buf = torch.empty(n * P, dtype=torch.uint8, device=DEV)
    pcs.gen_pages(buf, P, n, seed, first)
    # content is the BASELINE generator's (first, middle and last pages)
    for i in (0, n // 2, n - 1):
        want = oracle.fill_pages(P, 1, seed, first + i)
        assert np.array_equal(buf[i * P:(i + 1) * P].cpu().numpy(), want), (cfg, i)
    want = fixed_reference(pool, buf, P, n, algo)
    got = u64(pcs.pages_digest(buf, P, n, algo))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"config {cfg}: {bad.size} digests differ from the {checker()}, first {bad[:8]}"
    # write path: every header the stamp kernel wrote is the checker's digest
    pcs.pages_stamp(buf, P, n, algo)
    hb = np.nonzero(headers(buf, P, n) != want)[0]
    assert hb.size == 0, f"config {cfg}: {hb.size} stamped headers differ, first {hb[:8]}"
    # read path: all valid, then exactly the flipped pages fail
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert int(ok.sum()) == n and int(u64(fb)[0]) == (1 << 64) - 1
    pcs.flip_byte(buf, P, n, every=1000, byte_offset=10)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert np.array_equal(np.nonzero(ok.cpu().numpy() == 0)[0], np.arange(0, n, 1000))
    assert int(u64(fb)[0]) == 0
    del buf, ok, fb


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_every_digest_config3(pool, algo):
    n, seed = 1 << 20, 0x5EED0003
    offs, lens, total = mixed_layout(seed, 0, n)
    base = torch.empty(total, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    pcs.gen_desc(base, d_off, d_len, n, seed, 0)
    want = desc_reference(pool, base, offs, lens, algo)
    assert len(want) == n
    got = u64(pcs.desc_digest(base, d_off, d_len, n, algo))
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"config 3: {bad.size} digests differ from the {checker()}, first {bad[:8]}"
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    hdr = u64(base[torch.from_numpy(offs.view(np.int64)).to(DEV)[:, None]
                   + torch.arange(8, device=DEV)[None, :]].contiguous().view(torch.int64).reshape(-1))
    hb = np.nonzero(hdr != want)[0]
    assert hb.size == 0, f"config 3: {hb.size} stamped headers differ, first {hb[:8]}"
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert int(ok.sum()) == n
    flips = np.arange(0, n, 1000)
    base[torch.from_numpy((offs[flips] + 10).astype(np.int64)).to(DEV)] ^= 0x5A
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert np.array_equal(np.nonzero(ok.cpu().numpy() == 0)[0], flips)
    assert int(u64(fb)[0]) == 0
    del base, d_off, d_len
