"""Every launch variant selectable through pcs_set_tuning computes the same
bits.  The knobs pick between kernels and layouts (non-temporal loads, grid
caps, XXH64 LDS depth / quad layout, in-place vs two-pass stamp, split 64 KiB
pages, 4-block run-time batches); each must stay bit-exact with the oracle in
digest, validate and stamp modes.
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
    "stamp_inplace_8": {pcs.TUNE_STAMP_BYTES: 8},
    "stamp_inplace_64": {pcs.TUNE_STAMP_BYTES: 64},
    "x64_quad": {pcs.TUNE_XXH64_LAYOUT: 1},
    "x64_quad_nt": {pcs.TUNE_XXH64_LAYOUT: 1, pcs.TUNE_XXH64_NT_LOADS: 1},
    "x64_depth1": {pcs.TUNE_XXH64_LAYOUT: 2},
    "x64_depth4": {pcs.TUNE_XXH64_LAYOUT: 4},
    "rt_one_block": {pcs.TUNE_XXH3_RT_BATCH: 0},
    "no_split": {pcs.TUNE_XXH3_SPLIT_PAGES: 0},
    "split_16k": {pcs.TUNE_XXH3_SPLIT_PAGES: 16384},
    "split_64k": {pcs.TUNE_XXH3_SPLIT_PAGES: 65536},
    "desc_sort": {pcs.TUNE_DESC_SORT: 1},
    "desc_split": {pcs.TUNE_DESC_SPLIT: 1},
    "x64_desc_sort": {pcs.TUNE_XXH64_DESC_SORT: 1},
    "x64_desc_sort_depth1": {pcs.TUNE_XXH64_DESC_SORT: 1, pcs.TUNE_XXH64_LAYOUT: 2},
    "x64_one_wave": {pcs.TUNE_XXH64_WAVES: 1},
    "x64_two_waves_depth4": {pcs.TUNE_XXH64_WAVES: 2, pcs.TUNE_XXH64_LAYOUT: 4},
}


@pytest.fixture
def tuned(request):
    keys = list(range(1, 16))
    saved = {k: pcs.get_tuning(k) for k in keys}
    for k, v in VARIANTS[request.param].items():
        pcs.set_tuning(k, v)
    yield request.param
    for k, v in saved.items():
        pcs.set_tuning(k, v)


@pytest.mark.parametrize("tuned", list(VARIANTS), indirect=True)
@pytest.mark.parametrize("P,n", [(4096, 1000), (8192, 77), (16384, 45), (32768, 19), (65536, 21), (1280, 300),
                                 (5120, 33)])
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


@pytest.mark.parametrize("tuned", ["default", "no_nt", "rt_one_block", "x64_depth1", "x64_depth4", "x64_quad",
                                   "desc_sort", "desc_split", "x64_desc_sort", "x64_desc_sort_depth1", "x64_one_wave",
                                   "x64_two_waves_depth4"],
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
