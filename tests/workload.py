"""Synthetic page workloads shared by tests, the golden generator and bench.py.

Numpy mirror of the device generator (pcs_gen_pages_dev / pcs_gen_desc_dev in
eloqstore_amd/csrc/pcs_kernels.hip) and of oracle_fill_pages:

    word w of page p = splitmix64((seed ^ p) + (w + 1) * 0x9E3779B97F4A7C15)

Mixed-size batches (BASELINE.json config 3) draw each page's size from
{4, 8, 16} KiB with splitmix64(seed ^ p, word index 0x5A5A5A5A) % 3 and pack
pages contiguously (offset = exclusive prefix sum of sizes).
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
SIZE_CLASSES = np.array([4096, 8192, 16384], dtype=np.uint32)
SIZE_WORD = 0x5A5A5A5A


def _mix(z):
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def splitmix_words(seed: int, page_index: int, n_words: int) -> np.ndarray:
    """The n_words little-endian u64 words of one synthetic page."""
    with np.errstate(over="ignore"):
        base = np.uint64((seed ^ page_index) & 0xFFFFFFFFFFFFFFFF)
        w = np.arange(1, n_words + 1, dtype=np.uint64)
        return _mix(base + w * GOLDEN)


def fill_pages(seed: int, first_page: int, n_pages: int, page_size: int) -> np.ndarray:
    """(n_pages, page_size) uint8 array of synthetic pages."""
    words = page_size // 8
    with np.errstate(over="ignore"):
        p = (np.arange(first_page, first_page + n_pages, dtype=np.uint64) ^ np.uint64(seed))[:, None]
        w = np.arange(1, words + 1, dtype=np.uint64)[None, :]
        out = _mix(p + w * GOLDEN)
    return out.view(np.uint8).reshape(n_pages, page_size)


def fill_pages_at(seed: int, page_indices, page_size: int) -> np.ndarray:
    """(len(page_indices), page_size) uint8 array: the synthetic pages at
    those global indices (any order, gaps allowed)."""
    words = page_size // 8
    with np.errstate(over="ignore"):
        p = (np.asarray(page_indices, dtype=np.uint64) ^ np.uint64(seed))[:, None]
        w = np.arange(1, words + 1, dtype=np.uint64)[None, :]
        out = _mix(p + w * GOLDEN)
    return out.view(np.uint8).reshape(len(page_indices), page_size)


def mixed_sizes(seed: int, first_page: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        p = np.arange(first_page, first_page + n, dtype=np.uint64) ^ np.uint64(seed)
        sel = _mix(p + np.uint64(SIZE_WORD + 1) * GOLDEN) % np.uint64(3)
    return SIZE_CLASSES[sel.astype(np.int64)]


def mixed_layout(seed: int, first_page: int, n: int):
    """(offsets u64, lengths u32, total_bytes) for a packed mixed-size batch."""
    lens = mixed_sizes(seed, first_page, n)
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        np.cumsum(lens[:-1], dtype=np.uint64, out=offs[1:])
    total = int(offs[-1]) + int(lens[-1]) if n else 0
    return offs, lens.astype(np.uint32), total


def fill_desc(seed: int, first_page: int, offs, lens, total: int) -> np.ndarray:
    buf = np.zeros(total, dtype=np.uint8)
    for i in range(len(lens)):
        o, L = int(offs[i]), int(lens[i])
        buf[o:o + L] = splitmix_words(seed, first_page + i, L // 8).view(np.uint8)
    return buf
