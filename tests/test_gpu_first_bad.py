"""The validate calls' first_bad word on every validate kernel family (fixed,
split, any-size stride, XXH64 LDS and stride, descriptor XXH3, descriptor
XXH64 with its generic second pass), against the oracle's verdicts, repeated
calls and two streams interleaved.  The word is pre-filled with garbage every
time, so a path that never writes it fails.  (A fill-free form, a
self-resetting slot written by the kernels' last block, measured 37 % slower
and was not kept: DESIGN.md §4.6.)"""
import numpy as np
import pytest
import torch

import eloqstore_amd as pcs
import oracle
from workload import mixed_layout

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
NONE = (1 << 64) - 1


def garbage_word():
    return torch.full((1,), 0x1234, dtype=torch.int64, device=DEV)


def fb_value(fb):
    return int(fb.cpu().numpy().view(np.uint64)[0])


def stamped(P, n, algo, seed):
    buf = torch.empty(n * P, dtype=torch.uint8, device=DEV)
    pcs.gen_pages(buf, P, n, seed, 0)
    pcs.pages_stamp(buf, P, n, algo)
    return buf


def corrupt(buf, P, idx):
    if idx:
        pos = torch.tensor(idx, dtype=torch.int64, device=DEV) * P + 10
        buf[pos] ^= 0x40


# (P, n, algo): k_xxh3_fixed, k_xxh3_split (16 and 64 KiB), k_xxh3_stride any-size,
# k_xxh64_lds, k_xxh64_stride (P % 64 != 0)
SHAPES = [(4096, 5000, 0), (16384, 700, 0), (65536, 90, 0), (1000, 3000, 0), (4096, 5000, 1), (1000, 3000, 1)]


@pytest.mark.parametrize("P,n,algo", SHAPES)
def test_pages_first_bad(P, n, algo):
    buf = stamped(P, n, algo, 0xFB00 + P)
    patterns = [[], [n - 1], [17, 4000 % n, n // 2], list(range(0, n, 3)), list(range(n))]
    for bad in patterns:
        corrupt(buf, P, bad)
        for _rep in range(3):  # the slot must come back reset every call
            fb = garbage_word()
            ok, _ = pcs.pages_validate(buf, P, n, algo, first_bad=fb)
            want_ok = oracle.pages_digest(buf.cpu().numpy(), P, algo) == buf.cpu().numpy().reshape(n, P)[:, :8].copy().view(np.uint64).ravel()
            assert np.array_equal(ok.cpu().numpy().astype(bool), want_ok)
            assert fb_value(fb) == (min(bad) if bad else NONE), (bad[:3], fb_value(fb))
        corrupt(buf, P, bad)  # restore


@pytest.mark.parametrize("algo", [0, 1])
def test_desc_first_bad(algo):
    """Config-3-style mixed pages plus off-shape pages (unaligned, short,
    header-less): for XXH64 those take the generic second launch, whose blocks
    complete the call's count."""
    n = 3000
    offs, lens, total = mixed_layout(0xFB3, 0, n)
    offs = offs.copy()
    lens = lens.copy()
    lens[[5, 900, 2999]] = [1000, 7, 4100]  # off the line shape / shorter than the header
    base = torch.empty(total + 64, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    pcs.gen_desc(base, d_off, d_len, n, 0xFB3, 0)
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    for bad in ([], [2999], [1234, 2000], [5]):
        for i in bad:
            base[int(offs[i]) + 10] ^= 0x40
        for _rep in range(3):
            fb = garbage_word()
            ok, _ = pcs.desc_validate(base, d_off, d_len, n, algo, first_bad=fb)
            expect = sorted(set(bad) | {900})  # page 900 is 7 bytes: never valid
            assert np.array_equal(np.flatnonzero(ok.cpu().numpy() == 0), expect)
            assert fb_value(fb) == expect[0]
        for i in bad:
            base[int(offs[i]) + 10] ^= 0x40


def test_zero_pages_writes_none():
    buf = torch.empty(4096, dtype=torch.uint8, device=DEV)
    ok = torch.empty(1, dtype=torch.uint8, device=DEV)
    fb = garbage_word()
    pcs.pages_validate(buf, 4096, 0, 0, ok=ok, first_bad=fb)
    assert fb_value(fb) == NONE


def test_word_follows_each_call():
    P, n = 4096, 1000
    buf = stamped(P, n, 0, 0xFB7)
    corrupt(buf, P, [3])
    ok, _ = pcs.pages_validate(buf, P, n, 0, first_bad=None)
    assert int((ok == 0).sum()) == 1
    fb = garbage_word()
    ok, _ = pcs.pages_validate(buf, P, n, 0, first_bad=fb)
    assert fb_value(fb) == 3


def test_streams_interleaved():
    """Two streams validating different batches back to back: leases keep
    their slots apart; each call's word is its own batch's first bad page."""
    P = 4096
    a = stamped(P, 4096, 0, 0xFB10)
    b = stamped(P, 2048, 1, 0xFB11)
    corrupt(a, P, [100, 3000])
    corrupt(b, P, [2047])
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    fa = [garbage_word() for _ in range(20)]
    fbs = [garbage_word() for _ in range(20)]
    oka = torch.empty(4096, dtype=torch.uint8, device=DEV)
    okb = torch.empty(2048, dtype=torch.uint8, device=DEV)
    torch.cuda.synchronize()
    for i in range(20):
        pcs.pages_validate(a, P, 4096, 0, ok=oka, first_bad=fa[i], stream=sa)
        pcs.pages_validate(b, P, 2048, 1, ok=okb, first_bad=fbs[i], stream=sb)
    torch.cuda.synchronize()
    assert [fb_value(x) for x in fa] == [100] * 20
    assert [fb_value(x) for x in fbs] == [2047] * 20


def test_large_grid():
    """A 1 GiB batch of 4 KiB pages: 16,384 blocks count into one slot."""
    P, n = 4096, 1 << 18
    buf = stamped(P, n, 0, 0xFB20)
    corrupt(buf, P, [n - 5, 200000])
    fb = garbage_word()
    ok, _ = pcs.pages_validate(buf, P, n, 0, first_bad=fb)
    assert int((ok == 0).sum()) == 2 and fb_value(fb) == 200000
    corrupt(buf, P, [n - 5, 200000])
    pcs.pages_validate(buf, P, n, 0, ok=ok, first_bad=fb)
    assert fb_value(fb) == NONE
