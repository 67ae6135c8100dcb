"""Every launch variant selectable through pcs_set_tuning computes the same
bits.  The knobs pick between kernels and layouts (non-temporal loads, grid
caps, XXH64 LDS depth and waves per workgroup, split pages, 4-block run-time
batches); each must stay bit-exact with the oracle in digest, validate and
stamp modes.  (Variants measured slower were retired in round 2: in-place
stamp, XXH64 quad layout, descriptor slices / sorts; their keys now fail.)
"""
import numpy as np
import pytest
import torch

import eloqstore_amd as pcs
import oracle
from workload import mixed_layout

pytestmark = pytest.mark.gpu

DEV = "cuda:0"

VARIANTS = {
    "default": {},
    "no_nt": {pcs.TUNE_NT_LOADS: 0},
    "grid_stride": {pcs.TUNE_XXH3_BLOCKS_PER_CU: 1, pcs.TUNE_XXH64_BLOCKS_PER_CU: 1},
    "x64_depth1": {pcs.TUNE_XXH64_LAYOUT: 2},
    "x64_depth4": {pcs.TUNE_XXH64_LAYOUT: 4},
    # depth 3 (layout 5): the only depth that is not a power of two, so segment
    # counts that are not a multiple of 3 leave through the in-loop break
    "x64_depth3": {pcs.TUNE_XXH64_LAYOUT: 5},
    "x64_two_waves_depth3": {pcs.TUNE_XXH64_WAVES: 2, pcs.TUNE_XXH64_LAYOUT: 5},
    "rt_one_block": {pcs.TUNE_XXH3_RT_BATCH: 0},
    "no_split": {pcs.TUNE_XXH3_SPLIT_PAGES: 0},
    "split_16k": {pcs.TUNE_XXH3_SPLIT_PAGES: 16384},
    "split_64k": {pcs.TUNE_XXH3_SPLIT_PAGES: 65536},
    "x64_one_wave": {pcs.TUNE_XXH64_WAVES: 1},
    "x64_two_waves_depth4": {pcs.TUNE_XXH64_WAVES: 2, pcs.TUNE_XXH64_LAYOUT: 4},
}


@pytest.fixture
def tuned(request):
    keys = [k for k in range(1, 30) if pcs.get_tuning(k) >= 0 and k not in (26, 27)]  # retired keys read -1
    saved = {k: pcs.get_tuning(k) for k in keys}
    for k, v in VARIANTS[request.param].items():
        pcs.set_tuning(k, v)
    yield request.param
    for k, v in saved.items():
        pcs.set_tuning(k, v)


@pytest.mark.parametrize("tuned", list(VARIANTS), indirect=True)
@pytest.mark.parametrize("P,n", [(4096, 1000), (8192, 77), (16384, 45), (32768, 19), (65536, 21), (1280, 300),
                                 (5120, 33), (4160, 50), (192, 300)])
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_variant_pages(tuned, P, n, algo):
    buf = torch.empty(n * P, dtype=torch.uint8, device=DEV)
    pcs.gen_pages(buf, P, n, 0xA11 + P, 5)
    want = oracle.pages_digest(buf.cpu().numpy(), P, algo)
    got = pcs.pages_digest(buf, P, n, algo).cpu().numpy().view(np.uint64)
    assert np.array_equal(got, want), (tuned, np.flatnonzero(got != want)[:8])
    pcs.pages_stamp(buf, P, n, algo)
    host = buf.cpu().numpy().reshape(n, P)
    assert np.array_equal(host[:, :8].copy().view(np.uint64).ravel(), want)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert ok.cpu().numpy().all() and int(fb.cpu().numpy().view(np.uint64)[0]) == 2**64 - 1
    # corrupt every 9th page (byte 10, persist.cpp:241-246) and validate again
    pcs.flip_byte(buf, P, n, 9, 10)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert np.array_equal(np.flatnonzero(ok.cpu().numpy() == 0), np.arange(0, n, 9)), tuned
    assert int(fb.cpu().numpy().view(np.uint64)[0]) == 0


@pytest.mark.parametrize("tuned", ["default", "no_nt", "rt_one_block", "x64_depth1", "x64_depth4", "x64_one_wave",
                                   "x64_two_waves_depth4", "x64_depth3", "x64_two_waves_depth3"],
                         indirect=True)
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_variant_mixed_desc(tuned, algo):
    n = 2000
    offs, lens, total = mixed_layout(0x5EED0003, 0, n)
    base = torch.empty(total, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    pcs.gen_desc(base, d_off, d_len, n, 0x5EED0003, 0)
    host = base.cpu().numpy()
    want = np.array([oracle.pages_digest(host[o:o + l], int(l), algo)[0] for o, l in zip(offs, lens)], dtype=np.uint64)
    got = pcs.desc_digest(base, d_off, d_len, n, algo).cpu().numpy().view(np.uint64)
    assert np.array_equal(got, want), (tuned, np.flatnonzero(got != want)[:8])
    # stamp, validate, corrupt every 7th page from page 3: verdicts and the
    # first bad index must not depend on the order pages are hashed in
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    hdr = base.cpu().numpy()
    assert np.array_equal(np.array([hdr[o:o + 8].view(np.uint64)[0] for o in offs], dtype=np.uint64), want)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert ok.cpu().numpy().all()
    bad = np.arange(3, n, 7)
    flip = torch.from_numpy((offs[bad] + 10).astype(np.int64)).to(DEV)
    base[flip] ^= 0x5A
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert np.array_equal(np.flatnonzero(ok.cpu().numpy() == 0), bad), tuned
    assert int(fb.cpu().numpy().view(np.uint64)[0]) == 3


@pytest.mark.parametrize("tuned,algo", [("default", 0), ("no_nt", 0), ("rt_one_block", 0), ("default", 1)], indirect=["tuned"])
@pytest.mark.parametrize("mode", ["digest", "validate", "stamp"])
def test_desc_mixed_with_leftovers(tuned, algo, mode):
    """XXH3 and XXH64 descriptor batches of every shape class: 4-16 KiB pages and
    32 KiB pages and 256-byte multiples (one group per page), odd sizes and
    8-byte-aligned offsets (generic lanes), runs of one size, a zero-length
    and a 7-byte page, and pages out of offset order.  Every page must match
    the oracle."""
    rng = np.random.default_rng(5)
    n = 3001
    sizes = rng.choice([4096, 8192, 12288, 16384, 4096, 8192, 16384, 32768, 5120, 1280, 1000, 7, 0], size=n)
    sizes[100:160] = 4096  # a run of 1-slice pages
    sizes[200:230] = 16384  # a run of 4-slice pages
    sizes[300:400] = 1280  # a run of 256-byte-multiple pages
    pad = rng.choice([0, 0, 0, 8], size=n)  # some 8-byte-aligned starts
    offs = np.zeros(n, dtype=np.uint64)
    o = 0
    for i in range(n):
        o += int(pad[i])
        offs[i] = o
        o += int(sizes[i])
    perm = np.arange(n)
    perm[1000:1100] = perm[1000:1100][::-1]  # descriptors out of offset order
    offs, sizes = offs[perm], sizes[perm].astype(np.uint32)
    base = torch.from_numpy(rng.integers(0, 256, size=o + 64, dtype=np.uint8)).to(DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(sizes.view(np.int32)).to(DEV)
    host = base.cpu().numpy()

    def want_of(h):
        return np.array([oracle.pages_digest(h[int(a):int(a) + int(L)], int(L), algo)[0] if L >= 8 else 0
                         for a, L in zip(offs, sizes)], dtype=np.uint64)

    want = want_of(host)
    if mode == "digest":
        got = pcs.desc_digest(base, d_off, d_len, n, algo).cpu().numpy().view(np.uint64)
        assert np.array_equal(got, want), (tuned, np.flatnonzero(got != want)[:8])
    elif mode == "stamp":
        pcs.desc_stamp(base, d_off, d_len, n, algo)
        h2 = base.cpu().numpy()
        for a, L, wv in zip(offs, sizes, want):
            if L >= 8:
                assert h2[int(a):int(a) + 8].view(np.uint64)[0] == wv
    else:
        pcs.desc_stamp(base, d_off, d_len, n, algo)
        ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
        okh = ok.cpu().numpy()
        assert np.array_equal(okh, (sizes >= 8).astype(np.uint8)), tuned
        bad = [i for i in range(5, n, 11) if sizes[i] >= 16]
        flip = torch.from_numpy((offs[bad] + 10).astype(np.int64)).to(DEV)
        base[flip] ^= 0x5A
        ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
        expect_bad = sorted(set(bad) | set(np.flatnonzero(sizes < 8).tolist()))
        assert np.array_equal(np.flatnonzero(ok.cpu().numpy() == 0), expect_bad), tuned
        assert int(fb.cpu().numpy().view(np.uint64)[0]) == expect_bad[0]


def test_retired_tuning_keys_fail():
    """Keys of the variants retired in round 2 are refused, and read -1."""
    for k in (4, 5, 10, 12, 14, 16, 17, 18, 19, 20, 21, 22, 25, 99):
        assert pcs.get_tuning(k) == -1
        with pytest.raises(pcs.PcsError):
            pcs.set_tuning(k, 1)
