"""GPU parity: HIP kernels (through the C ABI) vs the CPU oracle and the
reference-generated golden vectors.  Bit-exact on every digest.

Runs only on an MI355X (`pytest -m gpu`).  Every call goes through
libeloqstore_pcs.so; the oracle is only the checker.
"""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest
import torch

import eloqstore_amd as pcs
import oracle
from workload import mixed_layout, splitmix_words

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "xxh_golden.json")
DEV = "cuda:0"


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    assert pcs.device_count() >= 1
    yield
    torch.cuda.synchronize()


def u64(t: torch.Tensor) -> np.ndarray:
    return t.cpu().numpy().view(np.uint64)


def dev_pages(P: int, n: int, seed: int, first: int = 0, extra: int = 0) -> torch.Tensor:
    buf = torch.empty(n * P + extra, dtype=torch.uint8, device=DEV)
    if n:
        pcs.gen_pages(buf, P, n, seed, first)
    return buf


PAGE_SIZES = [256, 512, 768, 1024, 1280, 2048, 3072, 4096, 8192, 16384, 32768, 65536]
ODD_SIZES = [8, 16, 40, 48, 136, 248, 264, 1000, 1032, 4104, 5000]


@pytest.mark.parametrize("P", PAGE_SIZES + ODD_SIZES)
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_pages_digest_vs_oracle(P, algo):
    for n in (1, 3, 17, 64 + 5):
        buf = dev_pages(P, n, 0x5EED0001 + P, 11)
        got = u64(pcs.pages_digest(buf, P, n, algo))
        want = oracle.pages_digest(buf.cpu().numpy(), P, algo)
        assert np.array_equal(got, want), (P, n, np.nonzero(got != want)[0][:8])


def test_pages_golden(golden):
    for blk in golden["pages"]:
        P = blk["page_size"]
        for p, h3, h64 in blk["rows"]:
            buf = dev_pages(P, 1, blk["seed"], p)
            assert int(u64(pcs.pages_digest(buf, P, 1, pcs.XXH3_64))[0]) == int(h3, 16), (P, p)
            assert int(u64(pcs.pages_digest(buf, P, 1, pcs.XXH64))[0]) == int(h64, 16), (P, p)


def test_config_samples_golden(golden):
    for blk in golden["config_samples"]:
        P = blk["page_size"]
        for p, h3, h64 in blk["rows"]:
            buf = dev_pages(P, 1, blk["seed"], p)
            assert int(u64(pcs.pages_digest(buf, P, 1, pcs.XXH3_64))[0]) == int(h3, 16)
            assert int(u64(pcs.pages_digest(buf, P, 1, pcs.XXH64))[0]) == int(h64, 16)


def test_zero_pages_is_noop():
    buf = torch.empty(4096, dtype=torch.uint8, device=DEV)
    out = torch.full((1,), 7, dtype=torch.int64, device=DEV)
    pcs.pages_digest(buf, 4096, 0, out=out)
    ok, fb = pcs.pages_validate(buf, 4096, 0)
    torch.cuda.synchronize()
    assert int(out[0]) == 7
    assert int(u64(fb)[0]) == (1 << 64) - 1


def test_adversarial_page_contents():
    # all-zero, all-0xFF and words that make lo32*hi32 overflow paths hit
    P = 4096
    n = 4
    host = np.zeros((n, P), dtype=np.uint8)
    host[1, :] = 0xFF
    host[2, :] = np.arange(P, dtype=np.uint32).astype(np.uint8)
    host[3].view(np.uint64)[:] = np.uint64(0xFFFFFFFF00000001)
    buf = torch.from_numpy(host.reshape(-1)).to(DEV)
    for algo in (pcs.XXH3_64, pcs.XXH64):
        got = u64(pcs.pages_digest(buf, P, n, algo))
        assert np.array_equal(got, oracle.pages_digest(host.reshape(-1), P, algo))


@pytest.mark.parametrize("P", [256, 4096, 16384, 65536, 1000])
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_stamp_validate_corrupt(P, algo):
    n = 203
    buf = dev_pages(P, n, 0x5EED00A0, 0)
    pcs.pages_stamp(buf, P, n, algo)
    host = buf.cpu().numpy()
    stored = host.reshape(n, P)[:, :8].copy().view(np.uint64).reshape(-1)
    assert np.array_equal(stored, oracle.pages_digest(host, P, algo))
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert ok.cpu().numpy().all() and int(u64(fb)[0]) == (1 << 64) - 1
    # persist.cpp:241-246 flips one byte; here byte 10 of every 7th page
    pcs.flip_byte(buf, P, n, every=7, byte_offset=10)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    okh = ok.cpu().numpy()
    bad = np.nonzero(okh == 0)[0]
    assert np.array_equal(bad, np.arange(0, n, 7))
    assert int(u64(fb)[0]) == 0
    # a flip in the stored digest itself is detected too
    buf2 = dev_pages(P, 3, 1, 0)
    pcs.pages_stamp(buf2, P, 3, algo)
    pcs.flip_byte(buf2, P, 3, every=2, byte_offset=3)
    ok, fb = pcs.pages_validate(buf2, P, 3, algo)
    assert list(ok.cpu().numpy()) == [0, 1, 0] and int(u64(fb)[0]) == 0


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_mixed_desc(golden, algo):
    mx = golden["mixed"]
    n = len(mx["rows"])
    offs, lens, total = mixed_layout(mx["seed"], 0, n)
    base = torch.empty(total, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    pcs.gen_desc(base, d_off, d_len, n, mx["seed"], 0)
    got = u64(pcs.desc_digest(base, d_off, d_len, n, algo))
    col = 2 if algo == pcs.XXH3_64 else 3
    want = np.array([int(r[col], 16) for r in mx["rows"]], dtype=np.uint64)
    assert np.array_equal(got, want)
    # validate / stamp / corrupt on the descriptor path
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert ok.cpu().numpy().all()
    host = base.cpu().numpy()
    host[int(offs[5]) + 10] ^= 0xFF
    host[int(offs[40]) + int(lens[40]) - 1] ^= 0x01
    base.copy_(torch.from_numpy(host))
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert list(np.nonzero(ok.cpu().numpy() == 0)[0]) == [5, 40]
    assert int(u64(fb)[0]) == 5


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_desc_odd_shapes(algo):
    # unaligned offsets, odd lengths, pages shorter than the header, mixed with fast-path pages
    rng = np.random.default_rng(7)
    lens = np.array([4096, 4100, 7, 8, 9, 100, 255, 256, 257, 1023, 1024, 8192, 3, 0, 65536, 4096, 300, 16384],
                    dtype=np.uint32)
    gaps = rng.integers(0, 40, size=len(lens))
    gaps[[0, 7, 11, 15]] = 16  # keep some 16-byte aligned
    offs = np.zeros(len(lens), dtype=np.uint64)
    pos = 0
    for i, L in enumerate(lens):
        pos += int(gaps[i])
        if i in (0, 7, 11, 15):
            pos = (pos + 15) // 16 * 16
        offs[i] = pos
        pos += int(L)
    host = rng.integers(0, 256, size=pos + 64, dtype=np.uint8)
    base = torch.from_numpy(host).to(DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    got = u64(pcs.desc_digest(base, d_off, d_len, len(lens), algo))
    want = np.array([oracle.pages_digest(host[int(o):int(o) + int(L)], int(L), algo)[0] if L >= 8 else 0
                     for o, L in zip(offs, lens)], dtype=np.uint64)
    assert np.array_equal(got, want), np.nonzero(got != want)
    ok, fb = pcs.desc_validate(base, d_off, d_len, len(lens), algo)
    okh = ok.cpu().numpy()
    assert okh[lens < 8].sum() == 0  # header-less pages never validate
    # stamp at unaligned offsets (two-pass: digests, then k_scatter_stamp_desc):
    # headers of pages >= 8 bytes get the digest, shorter pages stay untouched
    pcs.desc_stamp(base, d_off, d_len, len(lens), algo)
    h2 = base.cpu().numpy()
    for o, L, w in zip(offs, lens, want):
        o, L = int(o), int(L)
        if L >= 8:
            assert h2[o:o + 8].tobytes() == int(w).to_bytes(8, "little")
        hdr = 8 if L >= 8 else 0
        assert np.array_equal(h2[o + hdr:o + L], host[o + hdr:o + L])
    ok, fb = pcs.desc_validate(base, d_off, d_len, len(lens), algo)
    assert np.array_equal(ok.cpu().numpy().astype(bool), lens >= 8)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_desc_random_shapes(algo, seed):
    """Descriptor batches of random page sizes (0-20000 bytes, plus every
    length-class and block edge) at random offsets of any alignment, in random
    order: every branch of k_xxh3_desc (chunked body, any-size body, short
    pages on one lane) and of the XXH64 path (LDS kernel, generic lanes) next
    to each other in the same tiles.  Digest, stamp and validate vs the oracle."""
    rng = np.random.default_rng(seed)
    edges = np.array([0, 1, 7, 8, 9, 16, 24, 25, 136, 137, 248, 249, 250, 256, 257, 263, 264, 1032, 1033, 1040,
                      1096, 2056, 4096, 4104, 8192, 8200, 16384, 65535], dtype=np.uint32)
    n = 2500
    lens = np.where(rng.random(n) < 0.25, edges[rng.integers(0, len(edges), n)],
                    rng.integers(0, 20001, n)).astype(np.uint32)
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(rng.integers(0, 40))
        if rng.random() < 0.5:
            pos = (pos + 15) // 16 * 16
        offs[i] = pos
        pos += int(lens[i])
    perm = rng.permutation(n)  # descriptors not in memory order
    offs, lens = offs[perm], lens[perm]
    host = rng.integers(0, 256, size=pos + 64, dtype=np.uint8)
    want = np.zeros(n, dtype=np.uint64)  # header-less pages (< 8 bytes) digest to 0 (the reference assumes >= 8)
    hdr = lens >= 8
    want[hdr] = oracle.desc_digest(host, offs[hdr], lens[hdr], algo)
    base = torch.from_numpy(host).to(DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    got = u64(pcs.desc_digest(base, d_off, d_len, n, algo))
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, [(int(i), int(lens[i]), int(offs[i]) % 16) for i in bad[:8]]
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert np.array_equal(ok.cpu().numpy().astype(bool), lens >= 8)
    h2 = base.cpu().numpy()
    for i in np.flatnonzero(lens >= 8)[:400]:
        o = int(offs[i])
        assert h2[o:o + 8].tobytes() == int(want[i]).to_bytes(8, "little")


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_desc_mixed_wide(algo):
    """Many pages of many sizes in random order: every kernel split of the
    descriptor path (run-time-size groups, XXH64 LDS and quad kernels, generic
    lanes) sees neighbours of other shapes."""
    rng = np.random.default_rng(0xD35C)
    sizes = np.array([4096, 8192, 12288, 16384, 20480, 32768, 5120, 1280, 256, 4104, 65536, 100], dtype=np.uint32)
    n = 3000
    lens = sizes[rng.integers(0, len(sizes), size=n)]
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i, L in enumerate(lens):
        pos += 8 if rng.random() < 0.05 else 0  # a few 8-byte-misaligned pages
        offs[i] = pos
        pos += int(L)
        pos = (pos + 15) // 16 * 16 if rng.random() < 0.95 else pos
    host = rng.integers(0, 256, size=pos + 64, dtype=np.uint8)
    base = torch.from_numpy(host).to(DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    want = np.array([oracle.pages_digest(host[int(o):int(o) + int(L)], int(L), algo)[0] for o, L in zip(offs, lens)],
                    dtype=np.uint64)
    _desc_mixed_wide_checks(base, d_off, d_len, n, algo, offs, lens, want)


def _desc_mixed_wide_checks(base, d_off, d_len, n, algo, offs, lens, want):
    got = u64(pcs.desc_digest(base, d_off, d_len, n, algo))
    assert np.array_equal(got, want), np.flatnonzero(got != want)[:10]
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    h2 = base.cpu().numpy()
    stamped = np.array([h2[int(o):int(o) + 8].view(np.uint64)[0] for o in offs], dtype=np.uint64)
    assert np.array_equal(stamped, want)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert ok.cpu().numpy().all() and int(u64(fb)[0]) == 2**64 - 1
    bad = [7, 1500, 2999]
    for i in bad:
        h2[int(offs[i]) + int(lens[i]) // 2] ^= 0x10
    base.copy_(torch.from_numpy(h2))
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert list(np.flatnonzero(ok.cpu().numpy() == 0)) == bad and int(u64(fb)[0]) == 7


def test_raw_ranges_sweep(golden):
    sw = golden["sweep"]
    buf = splitmix_words(sw["seed"], sw["page_index"], sw["words"]).view(np.uint8)
    base = torch.from_numpy(buf.copy()).to(DEV)
    rows = sw["rows"]
    offs = np.array([r[0] for r in rows], dtype=np.uint64)
    lens = np.array([r[1] for r in rows], dtype=np.uint32)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    g3 = u64(pcs.xxh3_64_ranges(base, d_off, d_len, len(rows)))
    g64 = u64(pcs.xxh64_ranges(base, d_off, d_len, len(rows), 0))
    w3 = np.array([int(r[2], 16) for r in rows], dtype=np.uint64)
    w64 = np.array([int(r[3], 16) for r in rows], dtype=np.uint64)
    assert np.array_equal(g3, w3), [rows[i][:2] for i in np.nonzero(g3 != w3)[0][:10]]
    assert np.array_equal(g64, w64), [rows[i][:2] for i in np.nonzero(g64 != w64)[0][:10]]
    gs = u64(pcs.xxh64_ranges(base, d_off, d_len, len(rows), 0xDEADBEEF12345678))
    ws = np.array([oracle.xxh64(buf[int(o):int(o) + int(L)], 0xDEADBEEF12345678) for o, L in zip(offs, lens)],
                  dtype=np.uint64)
    assert np.array_equal(gs, ws)


def test_manifest_chunks(golden):
    # ManifestBuilder::CalcChecksum (root_meta.cpp:150-174): XXH3 per <=1 MiB chunk on the GPU,
    # serial rotl/mul fold on the host
    mf = golden["manifest"]
    longest = max(r[0] for r in mf["rows"])
    buf = splitmix_words(mf["seed"], 0, longest // 8 + 8).view(np.uint8)
    base = torch.from_numpy(buf.copy()).to(DEV)
    mask = (1 << 64) - 1
    for L, h in mf["rows"]:
        offs = np.arange(0, L, 1 << 20, dtype=np.uint64)
        lens = np.minimum(np.uint64(1 << 20), np.uint64(L) - offs).astype(np.uint32)
        agg = 0
        if len(offs):
            d = u64(pcs.xxh3_64_ranges(base, torch.from_numpy(offs.view(np.int64)).to(DEV),
                                       torch.from_numpy(lens.view(np.int32)).to(DEV), len(offs)))
            for x in d:
                agg = ((((agg << 1) | (agg >> 63)) & mask) ^ int(x))
                agg = (agg * 0x9E3779B97F4A7C15) & mask
        assert agg == int(h, 16), L


def test_host_single_page_api():
    P = 4096
    page = bytearray(splitmix_words(99, 0, P // 8).tobytes())
    pcs.set_checksum(page)
    assert int.from_bytes(page[:8], "little") == oracle.xxh3_64(bytes(page[8:]))
    assert pcs.validate_checksum(page)
    page[10] ^= 0xFF
    assert not pcs.validate_checksum(page)
    short = bytearray(100)
    pcs.set_checksum(short)
    assert int.from_bytes(short[:8], "little") == oracle.xxh3_64(bytes(short[8:]))


@pytest.mark.parametrize("P", [4096, 8192, 1000, 5000])
def test_host_batch_api(P):
    n = 300
    pages = [bytearray(splitmix_words(5, i, P // 8).tobytes()) for i in range(n)]
    digests = pcs.page_digests_host(pages, P)
    assert digests == [oracle.xxh3_64(bytes(p[8:])) for p in pages]
    pcs.set_checksums(pages, P)
    ok, fb = pcs.validate_checksums(pages, P)
    assert all(ok) and fb is None
    for i in (17, 250):
        pages[i][P - 1] ^= 0x40
    ok, fb = pcs.validate_checksums(pages, P)
    assert [i for i, v in enumerate(ok) if not v] == [17, 250] and fb == 17
    d64 = pcs.page_digests_host(pages, P, pcs.XXH64)
    assert d64 == [oracle.xxh64(bytes(p[8:])) for p in pages]


def test_host_batch_multi_chunk():
    # more than one 32 MiB staging slot: exercises the double-buffered pipeline
    P = 65536
    n = 1200
    pages = [bytearray(P) for _ in range(n)]
    for i in range(0, n, 37):
        pages[i][100:108] = i.to_bytes(8, "little")
    pcs.set_checksums(pages, P)
    ok, fb = pcs.validate_checksums(pages, P)
    assert all(ok)
    pages[1199][9] = 1
    ok, fb = pcs.validate_checksums(pages, P)
    assert fb == 1199 and sum(ok) == n - 1


def test_cli(tmp_path):
    f = tmp_path / "data.bin"
    tool = pcs.TOOL_PATH
    r = subprocess.run([tool, "--gen", str(f), "64", "4096", "0x5EED0001"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    raw = np.fromfile(f, dtype=np.uint8)
    ref = oracle.fill_pages(4096, 64, 0x5EED0001, 0).reshape(64, 4096)
    assert np.array_equal(raw.reshape(64, 4096)[:, 8:], ref[:, 8:])
    assert np.array_equal(raw.reshape(64, 4096)[:, :8].copy().view(np.uint64).reshape(-1),
                          oracle.pages_digest(raw, 4096))
    r = subprocess.run([tool, str(f), "0x1000"], capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.startswith("Checksum OK for page at offset 4096\n")
    lines = r.stdout.splitlines()
    assert lines[1] == "Page bytes (offset:value)" and len(lines) == 2 + 256
    assert lines[2] == "000000: " + "".join(f"{b:02x} " for b in raw[4096:4112])
    raw[5 * 4096 + 10] ^= 0xFF
    raw.tofile(f)
    r = subprocess.run([tool, str(f), str(5 * 4096)], capture_output=True, text=True)
    assert r.returncode == 2 and r.stdout.startswith("Checksum FAILED for page at offset 20480")
    r = subprocess.run([tool, "--scan", str(f)], capture_output=True, text=True)
    assert r.returncode == 2 and "64 pages of 4096 bytes: 1 corrupted, first at offset 20480" in r.stdout
    r = subprocess.run([tool, "--stamp", str(f)], capture_output=True, text=True)
    assert r.returncode == 0 and "Stamped 64 pages" in r.stdout
    r = subprocess.run([tool, "--scan", str(f)], capture_output=True, text=True)
    assert r.returncode == 0 and "64 pages of 4096 bytes: 0 corrupted" in r.stdout
    raw = np.fromfile(f, dtype=np.uint8)
    assert np.array_equal(raw.reshape(64, 4096)[:, :8].copy().view(np.uint64).reshape(-1),
                          oracle.pages_digest(raw, 4096))
    r = subprocess.run([tool, str(f), "0", "0"], capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid page size" in r.stderr
    r = subprocess.run([tool, str(f), "262141"], capture_output=True, text=True)
    assert r.returncode == 1 and "exceeds file size" in r.stderr


@pytest.mark.parametrize("P", [4096, 5000])
def test_cli_scan_windows(tmp_path, P):
    """Whole-file scrub over several 64 MiB chunks (two batches in flight,
    reads split over threads): every corrupted page is counted, the first
    offset reported, a trailing partial page ignored; the same with small
    chunks and one reader thread."""
    f = tmp_path / "big.bin"
    tool = pcs.TOOL_PATH
    n = (300 << 20) // P + 3
    r = subprocess.run([tool, "--gen", str(f), str(n), str(P), "0x5EED0009"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    with open(f, "r+b") as fh:
        for pg in (n - 2, (260 << 20) // P, 7):  # second window, across the boundary region, first window
            fh.seek(pg * P + P // 2)
            b = fh.read(1)
            fh.seek(pg * P + P // 2)
            fh.write(bytes([b[0] ^ 0x20]))
        fh.seek(0, 2)
        fh.write(b"\x01" * (P // 3))  # partial trailing page
    for env in (dict(os.environ), dict(os.environ, PCS_SCAN_THREADS="1", PCS_SCAN_CHUNK_MIB="5")):
        r = subprocess.run([tool, "--scan", str(f), str(P)], capture_output=True, text=True, env=env)
        assert r.returncode == 2, r.stdout + r.stderr
        assert f"{n} pages of {P} bytes: 3 corrupted, first at offset {7 * P}" in r.stdout, r.stdout


@pytest.mark.parametrize("P,n,algo", [
    (4096, 1 << 20, pcs.XXH3_64),    # BASELINE config 2 (fixed-size kernel)
    (16384, 1 << 18, pcs.XXH3_64),   # 16 KiB sweep (split-page kernel)
    (65536, 1 << 16, pcs.XXH3_64),   # config 4 shape, 4 GiB (split-page kernel)
    (4096, 1 << 20, pcs.XXH64),      # XXH64 LDS kernel
    (65536, 1 << 16, pcs.XXH64),     # XXH64 LDS kernel, one workgroup per 64 large pages
])
def test_full_size_properties(P, n, algo):
    """4 GiB device-resident batches at the bench's shapes.  Size-independent
    properties: stamp -> all valid; flip byte 10 of every 4096th page ->
    exactly those fail; sampled digests equal the oracle."""
    buf = dev_pages(P, n, 0x5EED0002, 0)
    dig = pcs.pages_digest(buf, P, n, algo)
    step = max(1, n // 256)
    sample = np.r_[0:64, n - 64:n, step:n:step]
    got = u64(dig)[sample]
    host = buf.view(-1, P)[torch.from_numpy(sample).to(DEV)].cpu().numpy()
    assert np.array_equal(got, oracle.pages_digest(host.reshape(-1), P, algo))
    pcs.pages_stamp(buf, P, n, algo)
    stored = buf.view(-1, P)[:, :8].contiguous().view(torch.int64).reshape(-1)
    assert torch.equal(stored, dig)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert int(ok.sum()) == n and int(u64(fb)[0]) == (1 << 64) - 1
    every = 4096 if n >= 1 << 20 else 1000
    pcs.flip_byte(buf, P, n, every=every, byte_offset=10)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    okh = ok.cpu().numpy()
    assert np.array_equal(np.nonzero(okh == 0)[0], np.arange(0, n, every))
    assert int(u64(fb)[0]) == 0
    del buf, dig
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_full_size_mixed_config3(algo):
    """BASELINE config 3 at full size: 1 M mixed 4/8/16 KiB pages (9.33 GiB)
    through the descriptor kernels.  Sampled digests equal the oracle; stamp
    -> all valid; a byte flipped in every 1000th page -> exactly those fail."""
    n = 1 << 20
    offs, lens, total = mixed_layout(0x5EED0003, 0, n)
    base = torch.empty(total, dtype=torch.uint8, device=DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    pcs.gen_desc(base, d_off, d_len, n, 0x5EED0003, 0)
    dig = u64(pcs.desc_digest(base, d_off, d_len, n, algo))
    sample = np.r_[0:32, n - 32:n, 4099:n:4099]
    for k in sample:
        o, L = int(offs[k]), int(lens[k])
        page = base[o:o + L].cpu().numpy()
        assert int(dig[k]) == int(oracle.pages_digest(page, L, algo)[0]), k
    pcs.desc_stamp(base, d_off, d_len, n, algo)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert int(ok.sum()) == n
    bad = np.arange(0, n, 1000)
    flip = torch.from_numpy((offs[bad] + 10).astype(np.int64)).to(DEV)
    base[flip] ^= 0x5A
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, algo)
    assert np.array_equal(np.nonzero(ok.cpu().numpy() == 0)[0], bad)
    assert int(u64(fb)[0]) == 0
    del base
    torch.cuda.empty_cache()


def test_full_size_64k_chunks_sampled():
    """BASELINE config 4 shape (64 KiB chunks), 16 K chunks; digests sampled vs oracle."""
    P, n = 65536, 16384
    buf = dev_pages(P, n, 0x5EED0004, 0)
    got = u64(pcs.pages_digest(buf, P, n))
    sample = np.r_[0:8, n - 8:n, 1000:n:1000]
    host = buf.view(-1, P)[torch.from_numpy(sample).to(DEV)].cpu().numpy()
    assert np.array_equal(got[sample], oracle.pages_digest(host.reshape(-1), P))
    del buf
    torch.cuda.empty_cache()


def _stream_fold(buf: np.ndarray) -> np.ndarray:
    """What pcs_stream_read_dev computes per 4 KiB page: lane g of the page's
    group folds its 16 pieces (bytes 256c + 16g) with xor/add, the 16 lanes
    xor-reduced; a partial page reads only its whole 16 B pieces."""
    nbytes = buf.nbytes - buf.nbytes % 16
    npg = (nbytes + 4095) // 4096
    pad = np.zeros(npg * 4096, dtype=np.uint8)
    pad[:nbytes] = buf[:nbytes]
    w = pad.view(np.uint32).reshape(npg, 16, 16, 4)  # page, chunk c, lane g, word
    x = np.bitwise_xor.reduce(w[..., 0], axis=1).astype(np.uint64)
    y = w[..., 1].astype(np.uint64).sum(axis=1) & 0xFFFFFFFF
    z = np.bitwise_xor.reduce(w[..., 2], axis=1).astype(np.uint64)
    ww = w[..., 3].astype(np.uint64).sum(axis=1) & 0xFFFFFFFF
    r = ((x ^ z) << np.uint64(32)) | ((y + ww) & np.uint64(0xFFFFFFFF))
    return np.bitwise_xor.reduce(r, axis=1)


@pytest.mark.parametrize("nbytes", [16, 4096, 65536, 65536 * 7, 65536 * 300 + 4096 + 48, 65536 * 5 + 23,
                                    4096 * 17 + 4000])
def test_stream_read_fold(nbytes):
    """The read-ceiling kernel reads every (whole 16-byte piece of every) byte
    of the range exactly once, whole and partial pages and tiles alike."""
    host = np.random.default_rng(nbytes).integers(0, 256, size=nbytes, dtype=np.uint8)
    buf = torch.from_numpy(host).to(DEV)
    npg = (nbytes - nbytes % 16 + 4095) // 4096
    out = torch.zeros(npg + 1, dtype=torch.int64, device=DEV)
    pcs.stream_read(buf, nbytes, out)
    got = u64(out)
    assert np.array_equal(got[:npg], _stream_fold(host)) and got[npg] == 0


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_host_direct_pinned_path(algo):
    """Contiguous pinned pages take the direct-DMA branch of the host pipeline
    (no gather); pageable pages of the same content take the gather branch."""
    P, n = 4096, 20000  # > 2 staging chunks of 32 MiB
    dev = dev_pages(P, n, 0x5EED00B0, 0)
    pinned = torch.empty(n * P, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(dev)
    want = oracle.pages_digest(pinned.numpy(), P, algo)
    out = np.empty(n, dtype=np.uint64)
    pageable = pinned.numpy().copy()  # keep a reference: the pointer must outlive the call
    for base in (pinned.data_ptr(), pageable.ctypes.data):
        ptrs = np.arange(n, dtype=np.uint64) * np.uint64(P) + np.uint64(base)
        rc = pcs.lib().pcs_pages_digest_host(ptrs.ctypes.data, P, n, algo, out.ctypes.data)
        assert rc == 0, pcs.lib().pcs_last_error()
        assert np.array_equal(out, want)
    # validate through the direct path, with corruption
    pcs.pages_stamp(dev, P, n, algo)
    pinned.copy_(dev)
    host = pinned.numpy()
    host[777 * P + 10] ^= 0xFF
    ptrs = np.arange(n, dtype=np.uint64) * np.uint64(P) + np.uint64(pinned.data_ptr())
    ok = np.empty(n, dtype=np.uint8)
    fb = ctypes.c_uint64(0)
    rc = pcs.lib().pcs_pages_validate_host(ptrs.ctypes.data, P, n, algo, ok.ctypes.data, ctypes.byref(fb))
    assert rc == 0 and fb.value == 777 and int((ok == 0).sum()) == 1


def test_long_ranges_vs_oracle():
    """Raw XXH3 ranges long enough for the workgroup-per-range kernel (>= 2 KiB,
    8-byte aligned), every tail shape: full/partial last block, odd lengths
    (unaligned last stripe), exact multiples of 1 KiB, 1 MiB manifest chunks."""
    rng = np.random.default_rng(11)
    lens = [2048, 2049, 2055, 2056, 3071, 3072, 3073, 4088, 4096, 5000, 65536, 65535 + 1024 * 3, 131072 + 17,
            (1 << 20), (1 << 20) - 1, 1000000, 777777] + [int(x) for x in rng.integers(2048, 300000, size=40)]
    offs, pos = [], 0
    for i, L in enumerate(lens):
        offs.append(pos + (8 if i % 3 == 1 else 0))  # mix 16-aligned and 8-mod-16 starts
        pos = offs[-1] + L + 8
        pos = (pos + 7) // 8 * 8
    host = rng.integers(0, 256, size=pos + 16, dtype=np.uint8)
    base = torch.from_numpy(host).to(DEV)
    o = np.array(offs, dtype=np.uint64)
    ln = np.array(lens, dtype=np.uint32)
    got = u64(pcs.xxh3_64_ranges(base, torch.from_numpy(o.view(np.int64)).to(DEV),
                                 torch.from_numpy(ln.view(np.int32)).to(DEV), len(lens)))
    want = oracle.desc_raw_xxh3(host, o, ln)
    assert np.array_equal(got, want), [lens[i] for i in np.nonzero(got != want)[0]]


def test_manifest_api_vs_golden(golden):
    mf = golden["manifest"]
    longest = max(r[0] for r in mf["rows"])
    buf = splitmix_words(mf["seed"], 0, longest // 8 + 8).view(np.uint8)
    dbuf = torch.from_numpy(buf.copy()).to(DEV)
    d_out = torch.empty(1, dtype=torch.int64, device=DEV)
    for L, h in mf["rows"]:
        assert pcs.manifest_checksum_host(buf[:L].tobytes()) == int(h, 16), L
        pcs._call("pcs_manifest_checksum_dev", dbuf.data_ptr(), L, d_out.data_ptr(), pcs._stream(None))
        assert int(u64(d_out)[0]) == int(h, 16), L


def test_manifest_record_validate():
    content = splitmix_words(5, 1, 40000).view(np.uint8).tobytes()[:300000]
    for L in (0, 12, 4000, 300000 - 20):
        rec = bytearray(8) + bytearray(content[: 12 + L])  # root|ttl|len + payload
        h = pcs.manifest_checksum_host(bytes(rec[8:]))
        assert h == oracle.manifest_checksum(bytes(rec[8:]))
        rec[:8] = h.to_bytes(8, "little")
        assert pcs.manifest_validate_host(bytes(rec))
        rec[-1] ^= 0x80
        assert not pcs.manifest_validate_host(bytes(rec))
    assert not pcs.manifest_validate_host(b"\0" * 19)  # shorter than the 20-byte header


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_async_batches(algo):
    P = 4096
    pages = [bytearray(splitmix_words(21, i, P // 8).tobytes()) for i in range(256)]
    stamp = pcs.Batch()
    stamp.submit(pcs.Batch.STAMP, pages, P, algo)
    while not stamp.poll():
        pass
    for p in pages:
        h = oracle.xxh3_64(bytes(p[8:])) if algo == 0 else oracle.xxh64(bytes(p[8:]))
        assert int.from_bytes(p[:8], "little") == h
    pages[99][2000] ^= 4
    v1, v2 = pcs.Batch(), pcs.Batch()
    v1.submit(pcs.Batch.VALIDATE, pages[:128], P, algo)
    v2.submit(pcs.Batch.VALIDATE, pages[128:], P, algo)
    v2.wait()
    while not v1.poll():
        pass
    ok1, fb1 = v1.result()
    ok2, fb2 = v2.result()
    assert fb1 == 99 and sum(ok1) == 127 and fb2 is None and all(ok2)
    d = pcs.Batch()
    d.submit(pcs.Batch.DIGEST, pages[:10], P, algo)
    d.wait()
    want = [(oracle.xxh3_64 if algo == 0 else oracle.xxh64)(bytes(p[8:])) for p in pages[:10]]
    assert d.result() == want
    empty = pcs.Batch()
    empty.submit(pcs.Batch.VALIDATE, [], P, algo)
    assert empty.poll() and empty.result() == ([], None)


def test_cpp_dropin_program():
    exe = os.path.join(os.path.dirname(__file__), "cpp", "dropin_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "dropin ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("order", ["ref_first", "pcs_first"])
def test_batch_api_beside_page_cpp_in_any_link_order(order):
    """page.cpp's single-page functions in a shared object beside the batch
    library, both link orders: single-page calls reach page.cpp (call
    counter), the batched validate / stamp run on the GPU and match the
    oracle, and never call page.cpp's functions (tests/cpp/linkorder_test.cpp)."""
    exe = os.path.join(os.path.dirname(__file__), "cpp", f"linkorder_{order}")
    r = subprocess.run([exe, "--gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "linkorder ok (gpu)" in r.stdout, r.stdout + r.stderr


ANY_SIZES =[249, 250, 255, 257, 1000, 1032, 1033, 1039, 1040, 1096, 2047, 2049, 4000, 4095, 4097, 4104, 4160, 5000,
             8000, 12345, 16000, 65535]


@pytest.mark.parametrize("P", ANY_SIZES)
@pytest.mark.parametrize("shift", [0, 8, 3])
def test_xxh3_any_page_size(P, shift):
    """XXH3 pages off the 256-byte grid and at any alignment (the any-size
    group body, xxh3_page_any: full blocks by 16-byte lane loads, the final
    block by 8-byte stripe loads), through the fixed-stride and the
    descriptor entry points, digest / validate / stamp.  Sizes cover every
    final-block shape: 0..15 ordinary stripes, NB = 0 (P < 1033), the last
    stripe across a chunk edge, EloqStore's largest data_page_size (65535).
    The batch ends at the end of its buffer."""
    rng = np.random.default_rng(P * 8 + shift)
    n = 19 if P < 20000 else 5
    host = rng.integers(0, 256, size=n * P, dtype=np.uint8)
    want = oracle.pages_digest(host, P, pcs.XXH3_64)
    buf = torch.empty(n * P + shift, dtype=torch.uint8, device=DEV)
    buf[shift:] = torch.from_numpy(host).to(DEV)
    pages = buf[shift:]
    assert np.array_equal(u64(pcs.pages_digest(pages, P, n, pcs.XXH3_64)), want)
    offs = (np.arange(n, dtype=np.uint64) * np.uint64(P) + np.uint64(shift)).view(np.int64)
    d_off = torch.from_numpy(offs).to(DEV)
    d_len = torch.full((n,), P, dtype=torch.int32, device=DEV)
    assert np.array_equal(u64(pcs.desc_digest(buf, d_off, d_len, n, pcs.XXH3_64)), want)
    pcs.pages_stamp(pages, P, n, pcs.XXH3_64)
    h2 = pages.cpu().numpy()
    for i in range(n):
        assert h2[i * P:i * P + 8].tobytes() == int(want[i]).to_bytes(8, "little")
    ok, fb = pcs.desc_validate(buf, d_off, d_len, n, pcs.XXH3_64)
    assert ok.cpu().numpy().all()
    pcs.flip_byte(pages, P, n, every=4, byte_offset=P - 1)  # the page's last byte: the last stripe
    ok, fb = pcs.pages_validate(pages, P, n, pcs.XXH3_64)
    assert list(np.flatnonzero(ok.cpu().numpy() == 0)) == list(range(0, n, 4)) and int(u64(fb)[0]) == 0


@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
@pytest.mark.parametrize("shift", [1, 8, 24])
def test_unaligned_page_base(algo, shift):
    """Pages whose base is not 16-byte aligned take the descriptor fallback;
    results must not change."""
    P, n = 4096, 37
    buf = dev_pages(P, n, 0x5EED00C0, 0, extra=64)
    host = buf.cpu().numpy()
    shifted = torch.empty(n * P + 64, dtype=torch.uint8, device=DEV)
    shifted[shift:shift + n * P] = buf[: n * P]
    got = u64(pcs.pages_digest(shifted[shift:], P, n, algo))
    assert np.array_equal(got, oracle.pages_digest(host[: n * P], P, algo))
    pcs.pages_stamp(shifted[shift:], P, n, algo)
    ok, fb = pcs.pages_validate(shifted[shift:], P, n, algo)
    assert int(ok.sum()) == n


def test_host_api_concurrent_threads():
    """Host batches from several threads at once (each thread owns its staging
    and streams; ctypes drops the GIL during the call)."""
    import threading

    P = 4096
    errors = []

    def worker(tid):
        try:
            pages = [bytearray(splitmix_words(700 + tid, i, P // 8).tobytes()) for i in range(300)]
            for _ in range(3):
                pcs.set_checksums(pages, P)
                ok, fb = pcs.validate_checksums(pages, P)
                assert all(ok) and fb is None
                pages[tid * 7][100] ^= 1
                ok, fb = pcs.validate_checksums(pages, P)
                assert fb == tid * 7
                pages[tid * 7][100] ^= 1
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


@pytest.mark.parametrize("use_side_stream", [False, True])
def test_stamp_while_gpu_busy(use_side_stream):
    """Two-pass stamp and the manifest path enqueued while the GPU is still
    busy with earlier work: their device scratch must not be reused or
    released before the queued kernels ran (regression: stream-ordered
    scratch lost 7 % of the headers, profiles/r01/stamp_lab.txt)."""
    P, n = 4096, 1 << 18
    buf = dev_pages(P, n, 0x5EED0002, 0)
    want = pcs.pages_digest(buf, P, n).clone()
    stream = torch.cuda.Stream() if use_side_stream else torch.cuda.current_stream()
    content = bytes(np.random.default_rng(3).integers(0, 256, size=(3 << 20) + 77, dtype=np.uint8))
    with torch.cuda.stream(stream):
        for _ in range(6):
            torch.cuda._sleep(3_000_000)  # keep the GPU busy while we enqueue
            buf.view(-1, P)[:, :8].zero_()
            pcs.pages_stamp(buf, P, n, stream=stream)
        stream.synchronize()
    stored = buf.view(-1, P)[:, :8].contiguous().view(torch.int64).reshape(-1)
    assert torch.equal(stored, want)
    ok, fb = pcs.pages_validate(buf, P, n)
    assert int(ok.sum()) == n
    for _ in range(3):
        torch.cuda._sleep(3_000_000)
        assert pcs.manifest_checksum_host(content) == oracle.manifest_checksum(content)


@pytest.mark.parametrize("wide", [1, 0])
def test_manifest_forms_vs_oracle(wide):
    """ManifestBuilder::CalcChecksum (root_meta.cpp:150-174) through both the
    wide (block sums over the GPU + chain per chunk) and the per-chunk-
    workgroup forms: last chunks in every XXH3 length class, aligned and
    unaligned content."""
    MiB = 1 << 20
    lens = [1, 16, 17, 128, 129, 240, 241, 2047, 2048, 2049, 100000, MiB - 1, MiB, MiB + 1, MiB + 16, MiB + 200,
            MiB + 2047, MiB + 2048, 3 * MiB + 777, 7 * MiB]
    host = np.random.default_rng(17).integers(0, 256, size=7 * MiB + 64, dtype=np.uint8)
    dbuf = torch.from_numpy(host).to(DEV)
    d_out = torch.empty(1, dtype=torch.int64, device=DEV)
    saved = pcs.get_tuning(pcs.TUNE_MANIFEST_WIDE)
    pcs.set_tuning(pcs.TUNE_MANIFEST_WIDE, wide)
    try:
        for shift in (0, 8, 3):  # 16-aligned, 8-aligned, unaligned content
            for L in lens:
                want = oracle.manifest_checksum(host[shift:shift + L])
                pcs._call("pcs_manifest_checksum_dev", dbuf.data_ptr() + shift, L, d_out.data_ptr(),
                          pcs._stream(None))
                assert int(u64(d_out)[0]) == want, (wide, shift, L)
        assert pcs.manifest_checksum_host(host[:3 * MiB + 5].tobytes()) == oracle.manifest_checksum(host[:3 * MiB + 5])
    finally:
        pcs.set_tuning(pcs.TUNE_MANIFEST_WIDE, saved)


@pytest.mark.parametrize("P,n", [(131072, 3), (1 << 20, 2), ((16 << 20) + 256, 1), ((4 << 20) + 4104, 2)])
@pytest.mark.parametrize("algo", [pcs.XXH3_64, pcs.XXH64])
def test_huge_pages(P, n, algo):
    """Pages far above EloqStore's 64 KiB (whole objects hashed with the page
    convention): one group per page walks 128 KiB - 16 MiB (the run-time-size
    and any-size bodies, the XXH64 LDS kernel at P % 64 == 0, the stride
    kernel at P % 64 != 0).  Digest, stamp, validate, and a flip of the last
    byte (the XXH3 last stripe / XXH64 tail), against the oracle."""
    buf = dev_pages(P, n, 0xB16 + P, 3)
    want = oracle.pages_digest(buf.cpu().numpy(), P, algo)
    assert np.array_equal(u64(pcs.pages_digest(buf, P, n, algo)), want)
    pcs.pages_stamp(buf, P, n, algo)
    host = buf.cpu().numpy().reshape(n, P)
    assert np.array_equal(host[:, :8].copy().view(np.uint64).ravel(), want)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert ok.cpu().numpy().all() and int(u64(fb)[0]) == (1 << 64) - 1
    pcs.flip_byte(buf, P, n, every=n, byte_offset=P - 1)
    ok, fb = pcs.pages_validate(buf, P, n, algo)
    assert list(ok.cpu().numpy()) == [0] + [1] * (n - 1) and int(u64(fb)[0]) == 0


def test_xxh64_desc_sparse_offshape_pages():
    """XXH64 descriptor batch of 100,000 line-shaped 4 KiB pages with three
    off-shape pages (8-byte-aligned, lengths not a multiple of 64) at the
    first, a middle and the last index: the LDS kernel flags the call, the
    gated generic pass (one block per CU, grid-stride) picks exactly those
    pages up; the same batch without them leaves the generic pass idle.
    (Round 5 measured hashing them inside the LDS kernel instead, one launch
    per call, and kept the two launches: DESIGN.md §4.2.)
    Digests against the oracle at the odd pages and a sample of the rest;
    then validate after a stamp, with one off-shape and one line-shaped page
    corrupted and a 4-byte page (shorter than its header, never valid)
    added: verdicts and first_bad exact."""
    n, P = 100_000, 4096
    lens = np.full(n, P, dtype=np.uint32)
    odd = [0, 51_234, n - 1]
    lens[odd] = [4100, 1000, 4168]
    offs = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        if i in odd:
            pos += 8  # 8-byte aligned only: off the line shape
        offs[i] = pos
        pos += int(lens[i])
        pos = (pos + 15) // 16 * 16
    # room for both layouts: the packed one (shorter, one page is 1000 bytes)
    # and the n x 4 KiB one below
    host = np.random.default_rng(64).integers(0, 256, size=max(pos, n * P) + 64, dtype=np.uint8)
    base = torch.from_numpy(host).to(DEV)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int32)).to(DEV)
    got = u64(pcs.desc_digest(base, d_off, d_len, n, pcs.XXH64))
    check = np.unique(np.concatenate([odd, np.arange(1, n, 997)]))
    want = oracle.desc_digest(host, offs[check], lens[check], pcs.XXH64)
    assert np.array_equal(got[check], want)
    # all line-shaped: the generic pass must not touch anything
    lens2 = np.full(n, P, dtype=np.uint32)
    offs2 = (np.arange(n, dtype=np.uint64) * P)
    d_off2 = torch.from_numpy(offs2.view(np.int64)).to(DEV)
    d_len2 = torch.from_numpy(lens2.view(np.int32)).to(DEV)
    base2 = base[: n * P]
    got2 = u64(pcs.desc_digest(base2, d_off2, d_len2, n, pcs.XXH64))
    want2 = oracle.desc_digest(host[: n * P], offs2[check], lens2[check], pcs.XXH64)
    assert np.array_equal(got2[check], want2)
    # validate: stamp the packed batch, corrupt an off-shape page (the middle
    # one) and a line-shaped one after it, then shrink page 70,000 to 4 bytes
    pcs.desc_stamp(base, d_off, d_len, n, pcs.XXH64)
    ok, fb = pcs.desc_validate(base, d_off, d_len, n, pcs.XXH64)
    assert int(ok.sum().item()) == n and int(fb.item()) == -1  # UINT64_MAX read as int64
    b = base.cpu().numpy()
    for i, byte in ((odd[1], 20), (60_000, 3000)):
        b[int(offs[i]) + byte] ^= 0x40
    lens3 = lens.copy()
    lens3[70_000] = 4
    base3 = torch.from_numpy(b).to(DEV)
    d_len3 = torch.from_numpy(lens3.view(np.int32)).to(DEV)
    ok, fb = pcs.desc_validate(base3, d_off, d_len3, n, pcs.XXH64)
    bad = np.flatnonzero(ok.cpu().numpy() == 0).tolist()
    assert bad == [odd[1], 60_000, 70_000], bad
    assert int(fb.item()) == odd[1]
