"""Zero-copy host batches over registered page pools (pcs_host_register).

EloqStore's pages live in pool chunks of 1024 pages (PagesPool::Extend,
src/storage/page.cpp:95-120) and are handed to the checksum call sites as
scattered pointers (ReadPages, async_io_manager.cpp:353-366; FlushBatchPages,
write_task.cpp:155-167).  With the chunk registered, a batch is one kernel
launch that reads the pages in place over PCIe.  Every result is checked
against the CPU oracle; the path counters prove which path ran.
"""
import numpy as np
import pytest

import eloqstore_amd as pcs
import oracle

pytestmark = pytest.mark.gpu

ZC = pcs.COUNTER_ZERO_COPY_LAUNCHES
GATHER = pcs.COUNTER_GATHER_CHUNKS


def _zc_delta(fn):
    before = (pcs.counter(ZC), pcs.counter(GATHER))
    out = fn()
    return out, pcs.counter(ZC) - before[0], pcs.counter(GATHER) - before[1]


def _scattered(pool, n, seed):
    """A ReadPages-like pointer list: distinct pool pages in random order."""
    idx = np.random.default_rng(seed).permutation(pool.n)[:n]
    return idx, pool.ptr(idx)


@pytest.mark.parametrize("algo,P", [(0, 4096), (0, 16384), (0, 65536), (0, 1280), (1, 4096), (1, 8192), (1, 192)])
def test_zero_copy_digest_validate_stamp(algo, P):
    n_pool = 1024 if P <= 16384 else 64  # one PagesPool chunk (page.cpp:95-120)
    with pcs.PagePool(n_pool, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, n_pool, 0x2C0 + P).reshape(n_pool, P)
        want = oracle.pages_digest(pool.pages, P, algo)
        idx, ptrs = _scattered(pool, min(300, n_pool), seed=P)

        dig, zc, g = _zc_delta(lambda: pcs.digest_ptrs(ptrs, P, algo))
        assert zc == 1 and g == 0
        assert np.array_equal(dig, want[idx])

        _, zc, _ = _zc_delta(lambda: pcs.stamp_ptrs(ptrs, P, algo))
        assert zc == 1
        stamped = pool.pages[idx, :8].copy().view(np.uint64).ravel()
        assert np.array_equal(stamped, want[idx])

        (ok, fb), zc, _ = _zc_delta(lambda: pcs.validate_ptrs(ptrs, P, algo))
        assert zc == 1 and ok.all() and fb is None

        # persist.cpp:241-246 style corruption: byte 10 of every 7th listed page
        bad = idx[::7]
        pool.pages[bad, 10] ^= 0xFF
        ok, fb = pcs.validate_ptrs(ptrs, P, algo)
        assert np.array_equal(np.flatnonzero(ok == 0), np.arange(0, len(idx), 7))
        assert fb == 0


def test_zero_copy_sees_host_rewrites():
    """The pool is reused batch after batch: the GPU must never serve a page
    from a stale cached copy after the host rewrote it."""
    P = 4096
    with pcs.PagePool(256, P) as pool:
        ptrs = pool.ptr(np.arange(256))
        for round_ in range(4):
            pool.pages[:] = oracle.fill_pages(P, 256, 0x900 + round_).reshape(256, P)
            want = oracle.pages_digest(pool.pages, P, 0)
            assert np.array_equal(pcs.digest_ptrs(ptrs, P), want)
            pcs.stamp_ptrs(ptrs, P)
            assert np.array_equal(pool.pages[:, :8].copy().view(np.uint64).ravel(), want)
            ok, fb = pcs.validate_ptrs(ptrs, P)
            assert ok.all() and fb is None


def test_zero_copy_async_batch():
    P = 4096
    with pcs.PagePool(512, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, 512, 0x77).reshape(512, P)
        want = oracle.pages_digest(pool.pages, P, 0)
        idx, ptrs = _scattered(pool, 128, seed=5)  # max_read_pages_batch (kv_options.h:18-19)
        b = pcs.Batch()
        try:
            before = pcs.counter(ZC)
            b.submit_ptrs(pcs.Batch.STAMP, ptrs, P)
            b.wait()
            assert pcs.counter(ZC) == before + 1
            assert b.result() == [int(x) for x in want[idx]]
            assert np.array_equal(pool.pages[idx, :8].copy().view(np.uint64).ravel(), want[idx])
            pool.pages[idx[3], 100] ^= 1
            b.submit_ptrs(pcs.Batch.VALIDATE, ptrs, P)
            while not b.poll():
                pass
            ok, fb = b.result()
            assert fb == 3 and ok.count(0) == 1
        finally:
            b.close()


def test_partially_registered_batch_falls_back():
    """One page outside every registered region: the staging path runs, same results."""
    P = 4096
    with pcs.PagePool(64, P) as pool, pcs.PagePool(8, P, register=False) as loose:
        pool.pages[:] = oracle.fill_pages(P, 64, 1).reshape(64, P)
        loose.pages[:] = oracle.fill_pages(P, 8, 2).reshape(8, P)
        ptrs = np.concatenate([pool.ptr(np.arange(10)), loose.ptr([3])])
        want = np.concatenate([oracle.pages_digest(pool.pages[:10], P), oracle.pages_digest(loose.pages[3:4], P)])
        dig, zc, g = _zc_delta(lambda: pcs.digest_ptrs(ptrs, P))
        assert zc == 0 and g == 1
        assert np.array_equal(dig, want)


def test_zero_copy_policy_knob():
    P = 4096
    with pcs.PagePool(64, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, 64, 3).reshape(64, P)
        want = oracle.pages_digest(pool.pages, P)
        contiguous = pool.ptr(np.arange(64))
        old = pcs.get_tuning(pcs.TUNE_ZERO_COPY)
        try:
            pcs.set_tuning(pcs.TUNE_ZERO_COPY, 0)  # stage: gather, or direct DMA of a contiguous run
            dig, zc, g = _zc_delta(lambda: pcs.digest_ptrs(contiguous[::-1], P))
            assert zc == 0 and g == 1 and np.array_equal(dig, want[::-1])
            before = pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS)
            dig, zc, _ = _zc_delta(lambda: pcs.digest_ptrs(contiguous, P))
            assert zc == 0 and pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS) == before + 1
            assert np.array_equal(dig, want)
            pcs.set_tuning(pcs.TUNE_ZERO_COPY, 1)  # registered -> zero-copy, contiguous or not
            dig, zc, _ = _zc_delta(lambda: pcs.digest_ptrs(contiguous, P))
            assert zc == 1 and np.array_equal(dig, want)
        finally:
            pcs.set_tuning(pcs.TUNE_ZERO_COPY, old)


def test_register_rejects_overlap_and_bad_unregister():
    with pcs.PagePool(16, 4096) as pool:
        with pytest.raises(pcs.PcsError):
            pcs.host_register(pool.base + 4096, 4096)
        with pytest.raises(pcs.PcsError):
            pcs.host_unregister(pool.base + 4096)


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_pinned_run_that_overruns_its_allocation_is_gathered(zero_copy):
    """a contiguous run that starts in pinned (registered) memory
    and runs past the end of that allocation must not be DMA'd as one pinned
    range: both ends are checked and must belong to one allocation."""
    P = 4096
    with pcs.PagePool(64, P, register=False) as pool:
        pool.pages[:] = oracle.fill_pages(P, 64, 9).reshape(64, P)
        want = oracle.pages_digest(pool.pages, P)
        pcs.host_register(pool.base, 32 * P)  # only the first half is pinned
        old = pcs.get_tuning(pcs.TUNE_ZERO_COPY)
        try:
            pcs.set_tuning(pcs.TUNE_ZERO_COPY, zero_copy)
            direct0 = pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS)
            dig, zc, g = _zc_delta(lambda: pcs.digest_ptrs(pool.ptr(np.arange(64)), P))
            assert zc == 0 and g == 1 and pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS) == direct0
            assert np.array_equal(dig, want)
            # the pinned half alone is one allocation: direct (or zero-copy)
            direct0 = pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS)
            dig, zc, g = _zc_delta(lambda: pcs.digest_ptrs(pool.ptr(np.arange(32)), P))
            assert g == 0 and (zc == 1 if zero_copy else pcs.counter(pcs.COUNTER_DIRECT_DMA_CHUNKS) == direct0 + 1)
            assert np.array_equal(dig, want[:32])
        finally:
            pcs.set_tuning(pcs.TUNE_ZERO_COPY, old)
            pcs.host_unregister(pool.base)


def test_batch_skip_verify_and_failed_submit():
    """skip_verify_checksum (kv_options.h:41) on the async batch, and ADVICE
    r01: a submit that fails after a completed batch leaves the batch idle, so
    poll/result refuse instead of returning the previous batch's verdicts."""
    P = 4096
    with pcs.PagePool(16, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, 16, 4).reshape(16, P)  # never stamped: all invalid
        b = pcs.Batch()
        b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(np.arange(16)), P)
        b.wait()
        ok, fb = b.result()
        assert ok == [0] * 16 and fb == 0
        b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(np.arange(16)), P, skip_verify=True)
        assert b.poll()  # complete at submit
        ok, fb = b.result()
        assert ok == [1] * 16 and fb is None
        with pytest.raises(pcs.PcsError):  # skip applies to validate only
            b.submit_ptrs(pcs.Batch.STAMP, pool.ptr(np.arange(16)), P, skip_verify=True)
        with pytest.raises(pcs.PcsError):  # batch is idle now
            b.poll()
        with pytest.raises(pcs.PcsError):
            b.result()
        b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(np.arange(16)), P)
        with pytest.raises(pcs.PcsError):
            b.submit_ptrs(pcs.Batch.VALIDATE, np.array([pool.base, 0], dtype=np.uint64), P)  # in flight
        b.wait()
        with pytest.raises(pcs.PcsError):  # null page pointer
            b.submit_ptrs(pcs.Batch.VALIDATE, np.array([pool.base, 0], dtype=np.uint64), P)
        with pytest.raises(pcs.PcsError):
            b.result()
        b.close()


@pytest.mark.parametrize("poll,event,spin", [(1, 0, 0), (0, 0, 0), (1, 1, 0), (1, 0, 1)])
def test_zero_copy_validate_completion_forms(poll, event, spin):
    """PCS_TUNE_ZC_POLL: a zero-copy validate completes when every verdict
    has landed in host memory (1, default) or on the launch's completion
    signal (0).  PCS_TUNE_ZC_BATCH_EVENT: an async batch completing from its
    verdicts has no event behind its kernel (0, default) or one (1).
    PCS_TUNE_SYNC_SPIN_US: sync callers spin throughout (0, default) or sleep
    between checks after 1 us (every wait of this test then sleeps).
    Back-to-back sync calls and async batches, inline (<= 256 pages) and
    host-memory page lists, each call with a different corrupted page, the
    pool rewritten between calls: every verdict and first-bad index must
    match the oracle."""
    P = 4096
    saved = pcs.get_tuning(pcs.TUNE_ZC_POLL)
    saved_ev = pcs.get_tuning(pcs.TUNE_ZC_BATCH_EVENT)
    saved_spin = pcs.get_tuning(pcs.TUNE_SYNC_SPIN_US)
    pcs.set_tuning(pcs.TUNE_ZC_POLL, poll)
    pcs.set_tuning(pcs.TUNE_ZC_BATCH_EVENT, event)
    pcs.set_tuning(pcs.TUNE_SYNC_SPIN_US, spin)
    try:
        with pcs.PagePool(1024, P) as pool:
            pool.pages[:] = oracle.fill_pages(P, 1024, 0x2CC).reshape(1024, P)
            for i in range(1024):
                pool.pages[i, :8] = np.frombuffer(oracle.pages_digest(pool.pages[i], P, 0).tobytes(), np.uint8)
            rng = np.random.default_rng(poll)
            b1, b2 = pcs.Batch(), pcs.Batch()
            try:
                for it in range(40):
                    n = (6, 48, 128, 256, 700, 1024)[it % 6]
                    idx = rng.permutation(1024)[:n]
                    ptrs = pool.ptr(idx)
                    j = int(rng.integers(n))
                    pool.pages[idx[j], 10] ^= 0x20
                    ok, fb = pcs.validate_ptrs(ptrs, P)
                    assert fb == j and np.flatnonzero(ok == 0).tolist() == [j], (it, n)
                    b = b1 if it % 2 else b2
                    b.submit_ptrs(pcs.Batch.VALIDATE, ptrs, P)
                    while not b.poll():
                        pass
                    okb, fbb = b.result()
                    assert fbb == j and okb.count(0) == 1, (it, n)
                    pool.pages[idx[j], 10] ^= 0x20  # restore before the next round
                    ok, fb = pcs.validate_ptrs(ptrs, P)
                    assert ok.all() and fb is None
            finally:
                b1.close()
                b2.close()
    finally:
        pcs.set_tuning(pcs.TUNE_ZC_POLL, saved)
        pcs.set_tuning(pcs.TUNE_ZC_BATCH_EVENT, saved_ev)
        pcs.set_tuning(pcs.TUNE_SYNC_SPIN_US, saved_spin)


@pytest.mark.parametrize("poll", [0, 1])
@pytest.mark.parametrize("P", [4096, 8192, 1280])
def test_zero_copy_stamp_completion_forms(poll, P):
    """PCS_TUNE_ZC_POLL on stamps: a zero-copy XXH3 stamp of up to
    PCS_TUNE_ZC_STAMP_POLL_PAGES (256) pages completes from per-page done
    bytes, each a system-scope store released after its header (1), or on the
    completion signal (0).  Back-to-back sync
    stamps and async batches (poll and wait) with the pool's bytes rewritten
    between calls: every header (and an async batch's digests) must be the
    oracle's digest of the new bytes once the call returns, and pages outside
    the batch untouched."""
    saved = pcs.get_tuning(pcs.TUNE_ZC_POLL)
    pcs.set_tuning(pcs.TUNE_ZC_POLL, poll)
    try:
        with pcs.PagePool(512, P) as pool:
            rng = np.random.default_rng(100 + poll)
            b = pcs.Batch()
            try:
                for it in range(36):
                    n = (1, 6, 48, 129, 256, 300)[it % 6]
                    form = it // 6 % 3  # sync call, async poll(), async wait()
                    pool.pages[:] = oracle.fill_pages(P, 512, 0x57A0 + it).reshape(512, P)
                    pool.pages[:, :8] = 0
                    idx = rng.permutation(512)[:n]
                    if form == 0:
                        pcs.stamp_ptrs(pool.ptr(idx), P)
                    else:
                        b.submit_ptrs(pcs.Batch.STAMP, pool.ptr(idx), P)
                        if form == 1:
                            while not b.poll():
                                pass
                        else:
                            b.wait()
                    hdr = pool.pages[:, :8].copy().view(np.uint64).ravel()
                    want = oracle.pages_digest(pool.pages[idx].reshape(-1), P, 0)
                    assert np.array_equal(hdr[idx], want), (it, n, form)
                    if form:
                        assert np.array_equal(np.array(b.result(), dtype=np.uint64), want), (it, n, form)
                    rest = np.setdiff1d(np.arange(512), idx)
                    assert not hdr[rest].any()
            finally:
                b.close()
    finally:
        pcs.set_tuning(pcs.TUNE_ZC_POLL, saved)


@pytest.mark.parametrize("poll", [1, 0])
@pytest.mark.parametrize("source", ["gather", "direct"])
def test_staged_validate_completion_forms(poll, source):
    """PCS_TUNE_ZC_POLL also covers staged validate batches (pages
    gathered into pinned staging, or a contiguous pinned run DMA'd as is):
    with polling on, the call completes once the D2H-copied verdict bytes have
    all landed, off on the stream's signal.  Sync calls (one chunk and a
    9,000-page batch over two 32 MiB slots) and async batches, a different
    corrupted page each round: verdicts and first_bad against the oracle, and
    the path counters prove the staged path ran."""
    P, N = 4096, 9000
    saved_poll, saved_zc = pcs.get_tuning(pcs.TUNE_ZC_POLL), pcs.get_tuning(pcs.TUNE_ZERO_COPY)
    pcs.set_tuning(pcs.TUNE_ZC_POLL, poll)
    pcs.set_tuning(pcs.TUNE_ZERO_COPY, 0)  # a registered run is DMA'd directly, not read in place
    try:
        with pcs.PagePool(N, P, register=source == "direct") as pool:
            pool.pages[:] = oracle.fill_pages(P, N, 0x57A6).reshape(N, P)
            want = oracle.pages_digest(pool.pages.reshape(-1), P, 0)
            pool.pages[:, :8] = want.view(np.uint8).reshape(N, 8)
            rng = np.random.default_rng(poll * 2 + (source == "direct"))
            counter = pcs.COUNTER_GATHER_CHUNKS if source == "gather" else pcs.COUNTER_DIRECT_DMA_CHUNKS
            b = pcs.Batch()
            try:
                for it in range(12):
                    n = (5, 128, 256, 2000, N)[it % 5]
                    first = int(rng.integers(0, N - n + 1))
                    idx = np.arange(first, first + n) if source == "direct" else rng.permutation(N)[:n]
                    j = int(rng.integers(n))
                    pool.pages[idx[j], 4000] ^= 0x08
                    c0 = pcs.counter(counter)
                    ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                    assert pcs.counter(counter) > c0 and pcs.counter(ZC) >= 0
                    assert fb == j and np.flatnonzero(ok == 0).tolist() == [j], (it, n)
                    if n <= 2000:
                        b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
                        if it % 2:
                            b.wait()
                        else:
                            while not b.poll():
                                pass
                        okb, fbb = b.result()
                        assert fbb == j and okb.count(0) == 1 and okb[j] == 0, (it, n)
                    pool.pages[idx[j], 4000] ^= 0x08
            finally:
                b.close()
    finally:
        pcs.set_tuning(pcs.TUNE_ZC_POLL, saved_poll)
        pcs.set_tuning(pcs.TUNE_ZERO_COPY, saved_zc)
