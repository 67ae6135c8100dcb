"""Pre-armed validate service (pcs_service_*): while it is on, host validate
batches of up to 256 registered pages are served by a resident kernel polling
a request line in pinned memory (small ReadPages batches);
it leaves after idle_us without a request or 2 * idle_us of life and the next
request starts a new generation.  Every verdict and first-bad index is checked
against the CPU oracle; the path counters prove which path served each batch.
Batches the service does not take (more than 256 pages, pages outside
registered memory, XXH64, page sizes off the 256-byte grid) come back right
through the launch path, and the resident kernel holds up a
device-synchronising call for no longer than its limits."""
import threading
import time

import numpy as np
import pytest

import eloqstore_amd as pcs
import oracle

pytestmark = pytest.mark.gpu

SVC = pcs.COUNTER_SERVICE_BATCHES
ZC = pcs.COUNTER_ZERO_COPY_LAUNCHES


@pytest.fixture
def service():
    assert pcs.lib().pcs_service_running() == 0
    with pcs.ValidateService(4, 1000):
        assert pcs.lib().pcs_service_running() == 1
        yield
    assert pcs.lib().pcs_service_running() == 0


def stamped_pool(n, P, seed):
    pool = pcs.PagePool(n, P)
    pool.pages[:] = oracle.fill_pages(P, n, seed).reshape(n, P)
    pcs.stamp_ptrs(pool.ptr(np.arange(n)), P)
    return pool


def counters():
    return pcs.counter(SVC), pcs.counter(ZC)


@pytest.mark.parametrize("P", [4096, 16384, 1280])
def test_service_serves_small_batches(service, P):
    n_pool = 1024 if P <= 4096 else 256
    with stamped_pool(n_pool, P, 0x5E1 + P) as pool:
        rng = np.random.default_rng(P)
        for n in (1, 5, 6, 7, 16, 100, 256):
            idx = rng.permutation(n_pool)[:n]
            ptrs = pool.ptr(idx)
            s0, z0 = counters()
            ok, fb = pcs.validate_ptrs(ptrs, P)
            assert ok.all() and fb is None
            assert counters() == (s0 + 1, z0), n
            assert pcs.lib().pcs_last_path() & pcs.PATH_SERVED and not pcs.lib().pcs_last_path() & pcs.PATH_LAUNCHED
            for j in sorted({0, n // 2, n - 1}):
                pool.pages[idx[j], P - 1] ^= 0x01  # the last stripe
                ok, fb = pcs.validate_ptrs(ptrs, P)
                hdr = pool.pages[idx, :8].copy().view(np.uint64).ravel()
                want = oracle.pages_digest(pool.pages[idx].reshape(-1), P, 0) == hdr
                assert np.array_equal(ok.astype(bool), want) and fb == j, (n, j)
                pool.pages[idx[j], P - 1] ^= 0x01


@pytest.mark.parametrize("P", [4096, 16384])
def test_service_stamps_small_batches(service, P):
    """Stamp requests: the kernel writes each digest into its page header
    (system-scope store, then the done word released after it); headers are
    checked against the oracle, pages outside the batch are untouched."""
    n_pool = 512 if P == 4096 else 128
    with pcs.PagePool(n_pool, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, n_pool, 0x5E7 + P).reshape(n_pool, P)
        pool.pages[:, :8] = 0
        want = oracle.pages_digest(pool.pages.reshape(-1), P, 0)
        rng = np.random.default_rng(P + 1)
        done = np.zeros(n_pool, dtype=bool)
        for n in (1, 3, 16, 100, 256):
            idx = rng.permutation(n_pool)[:n]
            s0, z0 = counters()
            pcs.stamp_ptrs(pool.ptr(idx), P)
            assert pcs.counter(SVC) == s0 + 1
            done[idx] = True
            hdr = pool.pages[:, :8].copy().view(np.uint64).ravel()
            assert np.array_equal(hdr[done], want[done]), n
            assert not hdr[~done].any()
        ok, fb = pcs.validate_ptrs(pool.ptr(np.flatnonzero(done)[:256]), P)
        assert ok.all() and fb is None


def test_service_idle_gaps(service):
    """Requests spaced wider than the idle limit find their kernel gone and
    start the next generation; gaps near the limit may find the old one
    leaving; results stay exact."""
    P = 4096
    with stamped_pool(64, P, 0x5E2) as pool:
        for gap in (0.0, 0.002, 0.0, 0.01, 0.0005, 0.0007, 0.0008, 0.0009, 0.001, 0.0011, 0.0, 0.0):
            time.sleep(gap)
            pool.pages[7, 10] ^= 0x01
            s0, _ = counters()
            ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(16)), P)
            assert fb == 7 and ok.sum() == 15 and pcs.counter(SVC) == s0 + 1
            pool.pages[7, 10] ^= 0x01


def test_service_declines_what_it_cannot_serve(service):
    P = 4096
    with stamped_pool(512, P, 0x5E9) as pool:
        idx = np.arange(300)  # more than 256 pages
        pool.pages[idx[257], 10] ^= 0xFF
        s0, z0 = counters()
        ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
        assert fb == 257 and ok.sum() == 299
        assert counters() == (s0, z0 + 1)
        pool.pages[idx[257], 10] ^= 0xFF
        s0, _ = counters()
        pcs.stamp_ptrs(pool.ptr(np.arange(16)), P, pcs.XXH64)
        ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(16)), P, pcs.XXH64)
        assert ok.all() and fb is None and pcs.counter(SVC) == s0
    pages = [bytearray(oracle.fill_pages(P, 1, 0x5EA + i).tobytes()) for i in range(8)]
    for pg in pages:
        pcs.set_checksum(pg)
    s0, _ = counters()
    ok, fb = pcs.validate_checksums(pages, P)
    assert ok == [1] * 8 and fb is None and pcs.counter(SVC) == s0


@pytest.fixture
def no_gate():
    """The contention gate off (PCS_TUNE_SERVICE_MAX_CALLERS = 0), so
    concurrent callers still reach the service's one request line."""
    pcs.set_tuning(pcs.TUNE_SERVICE_MAX_CALLERS, 0)
    try:
        yield
    finally:
        pcs.set_tuning(pcs.TUNE_SERVICE_MAX_CALLERS, 2)


def test_service_under_threads(service, no_gate):
    """Four threads validating at once, every request carrying a corrupted
    page of its own at a random slot (low slots included: those addresses
    come with the polled request words): one request at a time goes through
    the service, a call that finds it busy takes the launch path, and each
    thread gets exactly its own batch's verdicts and first_bad.  A request
    served with another request's page addresses would report the wrong
    slot (or none)."""
    P, T, per = 4096, 4, 256
    with stamped_pool(T * per, P, 0x5EB) as pool:
        errors = []

        def worker(t):
            rng = np.random.default_rng(100 + t)
            try:
                for _ in range(80):
                    n = int(rng.integers(1, 64))
                    idx = t * per + rng.permutation(per)[:n]
                    k = int(rng.integers(0, min(n, 14))) if rng.random() < 0.7 else int(rng.integers(0, n))
                    pool.pages[idx[k], 8 + int(rng.integers(0, P - 8))] ^= 0x10
                    ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                    want = np.ones(n, dtype=bool)
                    want[k] = False
                    if fb != k or not np.array_equal(ok.astype(bool), want):
                        errors.append((t, n, k, fb))
                    pcs.stamp_ptrs(pool.ptr(idx[k:k + 1]), P)  # heal: restamp the flipped page
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        s0, z0 = counters()
        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        s1, z1 = counters()
        assert s1 - s0 + z1 - z0 == 2 * T * 80 and s1 > s0


def test_service_alternating_page_sets(service):
    """Back-to-back requests from one thread whose page sets alternate
    (A, B, A, ...) in the polled slots 0-11 and beyond, with a corrupted page
    in a low slot on every other request: every request's verdicts belong
    to its own pages (a poll pairing the new seq with the previous request's
    addresses would validate the wrong set)."""
    P = 4096
    with stamped_pool(512, P, 0x5F0) as pool:
        rng = np.random.default_rng(7)
        s0, _ = counters()
        calls = 0
        for n in (5, 12, 13, 40):
            sets = [rng.permutation(256)[:n], 256 + rng.permutation(256)[:n]]
            for i in range(60):
                idx = sets[i % 2]
                k = None
                if i % 4 in (1, 2):
                    k = (i // 4) % min(n, 12)
                    pool.pages[idx[k], 777] ^= 0x02
                ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                calls += 1
                want = np.ones(n, dtype=bool)
                if k is not None:
                    want[k] = False
                    pool.pages[idx[k], 777] ^= 0x02
                assert fb == k and np.array_equal(ok.astype(bool), want), (n, i, k, fb)
        assert pcs.counter(SVC) == s0 + calls


@pytest.mark.parametrize("lines,wpl", [(4, 2), (8, 1)])
def test_service_lines_under_threads(lines, wpl, no_gate):
    """pcs_service_start_ex: several request lines, each served by its own
    workgroups.  Four threads, each request with a corrupted page of its own
    (low slots mostly): exact verdicts and first_bad on whichever line or
    path served it; the served share shows the lines were used."""
    P, T, per = 4096, 4, 256
    with stamped_pool(T * per, P, 0x5F6 + lines) as pool, pcs.ValidateService(wpl, 1000, lines):
        errors = []

        def worker(t):
            rng = np.random.default_rng(500 + t)
            try:
                for _ in range(80):
                    n = int(rng.integers(1, 40))
                    idx = t * per + rng.permutation(per)[:n]
                    k = int(rng.integers(0, min(n, 12)))
                    pool.pages[idx[k], 8 + int(rng.integers(0, P - 8))] ^= 0x04
                    ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                    want = np.ones(n, dtype=bool)
                    want[k] = False
                    if fb != k or not np.array_equal(ok.astype(bool), want):
                        errors.append((t, n, k, fb))
                    pcs.stamp_ptrs(pool.ptr(idx[k:k + 1]), P)
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        s0, z0 = counters()
        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        s1, z1 = counters()
        assert s1 - s0 + z1 - z0 == 2 * T * 80
        assert s1 - s0 > (z1 - z0), (s1 - s0, z1 - z0)  # with a line per thread, the service takes most calls


def test_service_lines_torn_drill_and_async(no_gate):
    """Four lines: the torn-line drill on every line in turn (two threads'
    worth of async batches in flight at once, each on its own line) and
    exact verdicts throughout."""
    P = 4096
    with stamped_pool(512, P, 0x5F7) as pool, pcs.ValidateService(1, 1000, 4):
        torn0 = pcs.counter(pcs.COUNTER_SERVICE_TORN_REQUESTS)
        pcs.set_tuning(pcs.TUNE_SERVICE_TEAR_TEST, 30)
        b1, b2 = pcs.Batch(), pcs.Batch()
        try:
            for i in range(24):
                i1, i2 = np.arange(i, i + 6), 256 + np.arange(3 * i, 3 * i + 20)
                k1, k2 = i % 6, (5 * i) % 20
                pool.pages[i1[k1], 100] ^= 0x01
                pool.pages[i2[k2], 200] ^= 0x01
                s0, _ = counters()
                b1.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(i1), P)
                b2.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(i2), P)
                b2.wait()
                b1.wait()
                assert pcs.counter(SVC) == s0 + 2, i  # both served, each on a line of its own
                ok1, fb1 = b1.result()
                ok2, fb2 = b2.result()
                pool.pages[i1[k1], 100] ^= 0x01
                pool.pages[i2[k2], 200] ^= 0x01
                assert fb1 == k1 and ok1.count(0) == 1 and fb2 == k2 and ok2.count(0) == 1, (i, fb1, fb2)
        finally:
            pcs.set_tuning(pcs.TUNE_SERVICE_TEAR_TEST, 0)
            b1.close()
            b2.close()
        assert pcs.counter(pcs.COUNTER_SERVICE_TORN_REQUESTS) - torn0 >= 24


def test_service_torn_line_drill(service):
    """PCS_TUNE_SERVICE_TEAR_TEST posts seq first and writes the request
    words 30 us later, so the waiting kernel's polls see the new seq beside
    the previous request's page addresses and count.  The check word must
    make the kernel ignore every such poll: verdicts stay exact for
    alternating page sets, and the kernel reports the torn lines it saw
    (PCS_COUNTER_SERVICE_TORN_REQUESTS)."""
    P = 4096
    with stamped_pool(256, P, 0x5F1) as pool:
        sets = [np.arange(0, 6), np.arange(100, 110)]
        torn0 = pcs.counter(pcs.COUNTER_SERVICE_TORN_REQUESTS)
        s0, _ = counters()
        pcs.set_tuning(pcs.TUNE_SERVICE_TEAR_TEST, 30)
        try:
            for i in range(40):
                idx = sets[i % 2]
                k = i % len(idx) if i % 2 else None
                if k is not None:
                    pool.pages[idx[k], 9] ^= 0x80
                ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                want = np.ones(len(idx), dtype=bool)
                if k is not None:
                    want[k] = False
                    pool.pages[idx[k], 9] ^= 0x80
                assert fb == k and np.array_equal(ok.astype(bool), want), (i, k, fb)
        finally:
            pcs.set_tuning(pcs.TUNE_SERVICE_TEAR_TEST, 0)
        assert pcs.counter(SVC) == s0 + 40
        torn = pcs.counter(pcs.COUNTER_SERVICE_TORN_REQUESTS) - torn0
        assert torn >= 20, torn  # most requests found a waiting kernel polling through the gap


def test_service_stamps_under_threads(service, no_gate):
    """Stamps from four threads on disjoint pages, served by the service or
    the launch path: every stamped header matches the oracle and the pages
    no request named keep their zero header."""
    P, T, per = 4096, 4, 128
    with pcs.PagePool(T * per, P) as pool:
        pool.pages[:] = oracle.fill_pages(P, T * per, 0x5F2).reshape(T * per, P)
        pool.pages[:, :8] = 0
        want = oracle.pages_digest(pool.pages.reshape(-1), P, 0)
        named = np.zeros(T * per, dtype=bool)
        errors = []

        def worker(t):
            rng = np.random.default_rng(300 + t)
            try:
                for _ in range(40):
                    n = int(rng.integers(1, 24))
                    idx = t * per + rng.permutation(per - 8)[:n]  # the last 8 pages of each range stay unnamed
                    named[idx] = True
                    pcs.stamp_ptrs(pool.ptr(idx), P)
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        s0, _ = counters()
        th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:5]
        hdr = pool.pages[:, :8].copy().view(np.uint64).ravel()
        assert np.array_equal(hdr[named], want[named])
        assert not hdr[~named].any()
        assert pcs.counter(SVC) > s0


def test_service_native_threads_and_gate():
    """tests/cpp/service_threads_test.cpp: eight native threads (Python
    threads serialise on the GIL between calls and never keep eight calls in
    flight): sync and async validates with a corrupted page of their own in
    every request, exact verdicts and first_bad on either path; stamps of
    disjoint pages against the oracle; the contention gate at its default
    serving every call of one thread and declining nearly all of eight."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "service_threads_test")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "service threads ok" in r.stdout, r.stdout + r.stderr
    print(r.stdout)


def test_service_soak_under_restarts():
    """tests/cpp/service_threads_test.cpp --soak: eight native threads mix
    sync validates, async validates and stamps while a controller thread
    stops and restarts the service with other line / workgroup / idle
    shapes, flips the gate knob and runs torn-line and re-post drills under
    them: every verdict, first_bad and header exact on whichever path served
    it."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "service_threads_test")
    r = subprocess.run([exe, "--soak", "12"], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "service soak ok" in r.stdout, r.stdout + r.stderr
    print(r.stdout)


@pytest.mark.parametrize("departure", ["0", "1"])
def test_service_soak_departure_modes(departure):
    """The soak (6 s) with the kernels' departure words off and on
    (PCS_TUNE_SERVICE_DEPARTURE): waiting requests learn that their line's
    workgroups left from the runtime every 50 us, or from the words the
    workgroups store as they leave (the runtime then every 1 ms).  Restarts,
    gate flips, torn-line and re-post drills: every result exact either way."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "service_threads_test")
    env = dict(os.environ, PCS_DEPARTURE=departure)
    r = subprocess.run([exe, "--soak", "6"], capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0 and "service soak ok" in r.stdout, r.stdout + r.stderr
    print(r.stdout)


def test_stamp_done_bytes_under_threads():
    """The launch path alone (no service): eight native threads stamping
    small batches of their own zeroed pages, synchronously and through
    pcs_batch, so every call completes from per-page done bytes (zero-copy
    XXH3 stamps of up to PCS_TUNE_ZC_STAMP_POLL_PAGES pages).  Every header,
    and every digest an async batch returns, must be in place when the call
    returns.  With a non-temporal header store behind a release
    fence, ~1 header in 10^5 landed after its done byte
    (profiles/r05/soak_bisect_before_fix.txt); the header and the done byte
    are now system-scope stores."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "service_threads_test")
    env = dict(os.environ, PCS_SOAK_OPS="12", PCS_SOAK_CTL="0", PCS_SOAK_START="off")
    r = subprocess.run([exe, "--soak", "6"], capture_output=True, text=True, timeout=100, env=env)
    assert r.returncode == 0 and "service soak ok" in r.stdout, r.stdout + r.stderr
    assert " 0 served" in r.stdout, r.stdout
    print(r.stdout)


def two_generations(pool, P, idle_us=1000):
    """Serve two requests an idle period apart, so the service has queued at
    least two generations (the re-post drill needs generation gen - 1)."""
    for _ in range(2):
        ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(500, 504)), P)
        assert ok.all() and fb is None
        time.sleep(3 * idle_us / 1e6)


@pytest.mark.parametrize("lines,wpl", [(1, 1), (2, 2), (4, 4)])
def test_service_repost_rearms_stale_verdicts(lines, wpl):
    """a request re-posted to a newer generation must be
    re-armed, or verdicts an older generation left count as answers and a
    lagging workgroup can write into the line's next request.  The drill
    (PCS_TUNE_SERVICE_REPOST_TEST) posts each request as an earlier
    generation would have left it: under generation gen - 1, which no
    waiting kernel serves, with a stale answer in the verdict words of pages
    16 and up (validate 0, stamp 1).  Every such request must come back
    through one re-post (PCS_COUNTER_SERVICE_REPOSTS) with the oracle's
    verdicts, first_bad and headers, and the next, undrilled request on the
    same line must be exact too.  With one workgroup per line, page 16 is
    hashed after page 0 by the same lanes, so a host that did not re-arm
    would collect the stale 0 before it is overwritten."""
    P = 4096
    with stamped_pool(512, P, 0x5F8 + lines) as pool, pcs.ValidateService(wpl, 1000, lines):
        two_generations(pool, P)
        rng = np.random.default_rng(lines)
        rep = pcs.COUNTER_SERVICE_REPOSTS
        try:
            for n, k in ((17, 3), (24, 20), (32, 0), (40, 16), (100, 99), (256, 7)):
                idx = rng.permutation(256)[:n]
                pool.pages[idx[k], 1234] ^= 0x08
                r0, s0 = pcs.counter(rep), pcs.counter(SVC)
                pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 1)
                ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                assert pcs.get_tuning(pcs.TUNE_SERVICE_REPOST_TEST) == 0  # consumed by this request
                want = np.ones(n, dtype=bool)
                want[k] = False
                assert fb == k and np.array_equal(ok.astype(bool), want), (n, k, fb, np.flatnonzero(~ok.astype(bool)))
                assert pcs.counter(rep) == r0 + 1 and pcs.counter(SVC) == s0 + 1
                pool.pages[idx[k], 1234] ^= 0x08
                # the next request on the line (another page set): exact
                other = 256 + rng.permutation(256)[:n]
                ok, fb = pcs.validate_ptrs(pool.ptr(other), P)
                assert ok.all() and fb is None and pcs.counter(rep) == r0 + 1
            # stamps: a stale done word must not stand for a header never written
            idx = np.arange(300, 340)
            pool.pages[idx, :8] = 0
            r0 = pcs.counter(rep)
            pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 1)
            pcs.stamp_ptrs(pool.ptr(idx), P)
            want = oracle.pages_digest(pool.pages[idx].reshape(-1), P, 0)
            assert np.array_equal(pool.pages[idx, :8].copy().view(np.uint64).ravel(), want)
            assert pcs.counter(rep) == r0 + 1
            # and asynchronously
            b = pcs.Batch()
            try:
                idx = np.arange(100, 160)
                pool.pages[idx[30], 99] ^= 0x01
                pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 1)
                b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
                b.wait()
                ok, fb = b.result()
                pool.pages[idx[30], 99] ^= 0x01
                assert fb == 30 and sum(ok) == len(idx) - 1 and pcs.counter(rep) == r0 + 2
            finally:
                b.close()
        finally:
            pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 0)


def test_service_restart_with_fewer_lines_falls_back():
    """four async batches in flight, one on each line of a
    4-line service, none answered (the re-post drill posts each under the
    previous generation, with stale verdicts on pages 16 and up).  The
    service stops and restarts with ONE line.  At their first check, the
    three batches whose lines the new service does not serve re-run on the
    launch path (pcs_capi.cpp: r.k >= lines, no re-post); the one on line 0
    is re-armed and re-posted to the new service.  All four come back with
    the oracle's verdicts and first_bad, and the restarted service serves
    the next request."""
    P = 4096
    with stamped_pool(512, P, 0x5FA) as pool:
        sets = [np.arange(40 * i, 40 * i + 20 + i) for i in range(4)]
        bad = [3, 17, 5, 19]
        batches = [pcs.Batch() for _ in range(4)]
        rep = pcs.COUNTER_SERVICE_REPOSTS
        try:
            pcs._call("pcs_service_start_ex", 4, 2, 1000)
            two_generations(pool, P)
            for i, idx in enumerate(sets):
                pool.pages[idx[bad[i]], 500] ^= 0x20
            r0, (s0, z0) = pcs.counter(rep), counters()
            pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 4)
            for b, idx in zip(batches, sets):
                b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
            assert pcs.get_tuning(pcs.TUNE_SERVICE_REPOST_TEST) == 0  # all four posted to the service
            pcs._call("pcs_service_stop")
            pcs._call("pcs_service_start_ex", 1, 2, 1000)
            for i, b in enumerate(batches):
                b.wait()
                ok, fb = b.result()
                assert fb == bad[i] and sum(ok) == len(sets[i]) - 1 and ok[bad[i]] == 0, (i, fb)
            # one re-post (line 0) served by the new service; three launches
            assert pcs.counter(rep) == r0 + 1
            assert counters() == (s0 + 1, z0 + 3)
            for i, idx in enumerate(sets):
                pool.pages[idx[bad[i]], 500] ^= 0x20
            s0, _ = counters()
            ok, fb = pcs.validate_ptrs(pool.ptr(sets[2]), P)
            assert ok.all() and fb is None and pcs.counter(SVC) == s0 + 1
        finally:
            pcs.set_tuning(pcs.TUNE_SERVICE_REPOST_TEST, 0)
            for b in batches:
                b.close()
            pcs._call("pcs_service_stop")


def test_gate_counts_only_service_shaped_calls():
    """the contention gate counts only calls the service could
    take (XXH3, 1-256 pages, page size on the 256-byte grid).  Four threads
    hammering XXH64 validates (always the launch path) beside one thread of
    small XXH3 validates on a one-line service with the gate at its default:
    the XXH64 traffic must not close the gate, so the XXH3 thread stays
    served (round 4 counted every call and closed it)."""
    P = 4096
    assert pcs.get_tuning(pcs.TUNE_SERVICE_MAX_CALLERS) == 2
    with stamped_pool(512, P, 0x5FB) as pool, pcs.ValidateService(4, 1000, 1):
        x64 = np.arange(256, 320)
        pcs.stamp_ptrs(pool.ptr(x64), P, pcs.XXH64)
        stop = threading.Event()
        errors = []

        def hammer():
            try:
                while not stop.is_set():
                    ok, fb = pcs.validate_ptrs(pool.ptr(x64), P, pcs.XXH64)
                    if not ok.all():
                        errors.append("xxh64 verdicts")
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        th = [threading.Thread(target=hammer) for _ in range(4)]
        for x in th:
            x.start()
        try:
            time.sleep(0.05)
            s0 = pcs.counter(SVC)
            calls = 0
            t_end = time.perf_counter() + 0.5
            while time.perf_counter() < t_end:
                ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(6)), P)
                assert ok.all() and fb is None
                calls += 1
            served = pcs.counter(SVC) - s0
        finally:
            stop.set()
            for x in th:
                x.join()
        assert not errors, errors[:3]
        assert calls > 50 and served >= 0.9 * calls, (served, calls)


def test_service_async_batches(service):
    """ChecksumBatch (pcs_batch_*) validate and stamp batches posted to the
    service: submit returns at once, poll watches the verdict words;
    verdicts, first_bad and stamped headers against the oracle; the service
    counter shows they were served and no launch happened."""
    P = 4096
    with stamped_pool(512, P, 0x5F4) as pool:
        b = pcs.Batch()
        try:
            for n, k in ((6, 4), (32, 0), (128, 100), (256, 255)):
                idx = np.random.default_rng(n).permutation(512)[:n]
                pool.pages[idx[k], 3000] ^= 0x40
                s0, z0 = counters()
                b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
                polls = 0
                while not b.poll():
                    polls += 1
                ok, fb = b.result()
                pool.pages[idx[k], 3000] ^= 0x40
                assert fb == k and sum(ok) == n - 1 and ok[k] == 0, (n, fb)
                assert counters() == (s0 + 1, z0), n
                assert b.path() & pcs.PATH_SERVED and not b.path() & pcs.PATH_LAUNCHED, b.path()
            idx = np.arange(300, 340)
            pool.pages[idx, :8] = 0
            s0, z0 = counters()
            b.submit_ptrs(pcs.Batch.STAMP, pool.ptr(idx), P)
            b.wait()
            assert counters() == (s0 + 1, z0)
            want = oracle.pages_digest(pool.pages[idx].reshape(-1), P, 0)
            assert np.array_equal(pool.pages[idx, :8].copy().view(np.uint64).ravel(), want)
            assert b.result() == [int(x) for x in want]
        finally:
            b.close()


def test_service_stop_with_async_batch_in_flight():
    """Stopping the service while an asynchronous batch is posted to it: the
    batch notices the service is gone and re-runs its pages on the launch
    path by itself (exact verdicts); a restarted service serves again."""
    P = 4096
    with stamped_pool(256, P, 0x5F5) as pool:
        idx = np.arange(10, 50)
        pool.pages[idx[17], 64] ^= 0x08
        b = pcs.Batch()
        try:
            for _ in range(6):
                pcs._call("pcs_service_start", 4, 1000)
                b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
                pcs._call("pcs_service_stop")
                b.wait()
                ok, fb = b.result()
                assert fb == 17 and sum(ok) == len(idx) - 1
            pcs._call("pcs_service_start", 4, 1000)
            s0, _ = counters()
            b.submit_ptrs(pcs.Batch.VALIDATE, pool.ptr(idx), P)
            b.wait()
            assert b.result()[1] == 17 and pcs.counter(SVC) == s0 + 1
        finally:
            b.close()
            pcs._call("pcs_service_stop")


def test_resident_kernel_does_not_hold_up_device_sync(service):
    """Right after a request the kernel is still resident and polling; a
    device-synchronising call elsewhere (unregistering another pool chunk)
    comes back once it leaves (1 ms idle), also while another thread keeps
    requests coming (2 ms of life at most)."""
    P = 4096
    with stamped_pool(64, P, 0x5EE) as pool:
        other = pcs.PagePool(16, P)
        ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(8)), P)
        assert ok.all()
        t0 = time.perf_counter()
        other.close()  # hipHostUnregister
        assert time.perf_counter() - t0 < 0.5
        ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(8)), P)  # still served afterwards
        assert ok.all() and fb is None

        stop = threading.Event()
        served = []

        def traffic():
            k = 0
            while not stop.is_set():
                ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(8)), P)
                k += int(ok.all() and fb is None)
            served.append(k)

        th = threading.Thread(target=traffic)
        th.start()
        try:
            time.sleep(0.05)
            for _ in range(3):
                other = pcs.PagePool(16, P)
                t0 = time.perf_counter()
                other.close()
                assert time.perf_counter() - t0 < 0.5
        finally:
            stop.set()
            th.join()
        assert served and served[0] > 10


def test_service_lifecycle():
    P = 4096
    for bad in ((0, 0), (257, 0), (4, 100), (4, 2000000)):
        with pytest.raises(pcs.PcsError):
            pcs._call("pcs_service_start", *bad)
    for bad in ((0, 1, 0), (9, 1, 0), (4, 65, 0), (2, 0, 0), (2, 2, 100)):
        with pytest.raises(pcs.PcsError):
            pcs._call("pcs_service_start_ex", *bad)
    with stamped_pool(64, P, 0x5EC) as pool:
        ptrs = pool.ptr(np.arange(8))
        for _round in range(2):  # start, serve, stop, and again
            pcs._call("pcs_service_start", 2, 0)
            try:
                with pytest.raises(pcs.PcsError):
                    pcs._call("pcs_service_start", 2, 0)  # already running
                s0, _ = counters()
                ok, fb = pcs.validate_ptrs(ptrs, P)
                assert ok.all() and fb is None and pcs.counter(SVC) == s0 + 1
            finally:
                pcs._call("pcs_service_stop")
            s0, z0 = counters()
            ok, fb = pcs.validate_ptrs(ptrs, P)  # after stop: the launch path
            assert ok.all() and counters() == (s0, z0 + 1)
            assert pcs.lib().pcs_last_path() == pcs.PATH_LAUNCHED
        pcs._call("pcs_service_stop")  # stopping a stopped service is fine


def test_service_left_running_at_exit():
    """A process that exits with its service on (no pcs_service_stop): the
    atexit handler ends the resident kernel before the HIP runtime tears
    down, so the process exits promptly and cleanly."""
    import os
    import subprocess
    import sys
    code = (
        "import numpy as np, eloqstore_amd as pcs, oracle\n"
        "P = 4096\n"
        "pool = pcs.PagePool(32, P)\n"
        "pool.pages[:] = oracle.fill_pages(P, 32, 7).reshape(32, P)\n"
        "pcs.stamp_ptrs(pool.ptr(np.arange(32)), P)\n"
        "pcs._call('pcs_service_start', 4, 1000000)\n"  # 1 s idle: only the exit hook ends it early
        "ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(8)), P)\n"
        "assert ok.all() and fb is None and pcs.counter(pcs.COUNTER_SERVICE_BATCHES) == 1\n"
        "print('served', flush=True)\n"
    )
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "-c", code], cwd=root, capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "served" in r.stdout
    assert time.perf_counter() - t0 < 60


def test_service_toggled_under_threads(no_gate):
    """Start and stop the service 20 times while four threads keep
    validating: every call lands on the service or the launch path with the
    oracle's verdicts (one corrupted page per batch), none hangs."""
    P = 4096
    with stamped_pool(512, P, 0x5EF) as pool:
        bad_page = 300
        pool.pages[bad_page, 50] ^= 0x04
        stop = threading.Event()
        errors, calls = [], [0] * 4

        def worker(t):
            rng = np.random.default_rng(200 + t)
            try:
                while not stop.is_set():
                    n = int(rng.integers(1, 48))
                    idx = rng.permutation(512)[:n]
                    ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                    want = idx != bad_page
                    if not np.array_equal(ok.astype(bool), want):
                        errors.append((t, n))
                    exp_fb = None if want.all() else int(np.flatnonzero(~want)[0])
                    if fb != exp_fb:
                        errors.append((t, n, fb, exp_fb))
                    calls[t] += 1
            except Exception as e:  # noqa: BLE001
                errors.append((t, repr(e)))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        s0 = pcs.counter(SVC)
        try:
            for _ in range(20):
                pcs._call("pcs_service_start", 4, 1000)
                time.sleep(0.01)
                pcs._call("pcs_service_stop")
                time.sleep(0.005)
        finally:
            stop.set()
            for x in th:
                x.join()
        assert not errors, errors[:5]
        assert min(calls) > 20 and pcs.counter(SVC) > s0
        assert pcs.lib().pcs_service_running() == 0


@pytest.mark.parametrize("mode", ["--slow-stop", "--slow-timeout"])
def test_poll_never_waits_on_a_slow_service_exit(mode):
    """ChecksumBatch::Poll / pcs_batch_poll must never block
    (shard.cpp:118-125: one poll that blocks stalls every coroutine of the
    shard).  tests/cpp/service_threads_test.cpp with the service kernel made
    a slow leaver (PCS_TUNE_SERVICE_SLOW_EXIT_TEST: it serves nothing and
    stays after it is told to leave).
    --slow-stop: another thread's pcs_service_stop waits ~300 ms for the
    kernel while this thread polls an async batch posted to it.  A slow
    poll (> 100 us) is the host's, not the library's, when a control thread
    that only reads the clock stalled at the same time, or when the polling
    thread was preempted during it (the kernel's per-thread switch counts:
    involuntary and no voluntary one).  At most 3 of the millions of polls
    may be slow and the library's, none of them over 5 ms (round 5 held the
    service's lock through the drain: polls waited the whole 300 ms).  The
    stop really took the 300 ms, and the batch comes back exact through the
    launch path.
    --slow-timeout: nobody stops it; the request gives up after 5 s (polls
    bounded the same way), re-runs exact on the launch path, and its line is
    quarantined until the kernel has left: a request meanwhile is launched,
    and the line serves again afterwards."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(__file__), "cpp", "service_threads_test")
    r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and f"{mode[2:]} ok" in r.stdout, r.stdout + r.stderr
    print(r.stdout)


def test_thread_prepare():
    """pcs_thread_prepare (eloqstore::PrepareChecksumThread): idempotent, and
    a prepared thread's first small host batch is served exactly."""
    P = 4096
    with stamped_pool(64, P, 0x5FC) as pool:
        errors = []

        def worker():
            try:
                for _ in range(2):
                    pcs._call("pcs_thread_prepare")
                pool.pages[3, 99] ^= 0x01
                ok, fb = pcs.validate_ptrs(pool.ptr(np.arange(8)), P)
                pool.pages[3, 99] ^= 0x01
                if fb != 3 or ok.sum() != 7:
                    errors.append((fb, ok))
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        th = threading.Thread(target=worker)
        th.start()
        th.join()
        assert not errors, errors


def test_service_with_sleeping_sync_waits(service):
    """PCS_TUNE_SYNC_SPIN_US = 1: a synchronous call through the service spins
    1 us, then sleeps between checks.  Validates with a
    corrupted page and stamps of 1-256 pages stay exact and served."""
    P = 4096
    saved = pcs.get_tuning(pcs.TUNE_SYNC_SPIN_US)
    pcs.set_tuning(pcs.TUNE_SYNC_SPIN_US, 1)
    try:
        with stamped_pool(512, P, 0x5FD) as pool:
            rng = np.random.default_rng(9)
            for n in (1, 7, 64, 256):
                idx = rng.permutation(512)[:n]
                k = int(rng.integers(n))
                pool.pages[idx[k], 2000] ^= 0x04
                s0 = pcs.counter(SVC)
                ok, fb = pcs.validate_ptrs(pool.ptr(idx), P)
                pool.pages[idx[k], 2000] ^= 0x04
                assert fb == k and ok.sum() == n - 1 and pcs.counter(SVC) == s0 + 1, n
                assert pcs.lib().pcs_last_path() & pcs.PATH_SERVED
            idx = np.arange(400, 500)
            pool.pages[idx, :8] = 0
            pcs.stamp_ptrs(pool.ptr(idx), P)
            want = oracle.pages_digest(pool.pages[idx].reshape(-1), P, 0)
            assert np.array_equal(pool.pages[idx, :8].copy().view(np.uint64).ravel(), want)
    finally:
        pcs.set_tuning(pcs.TUNE_SYNC_SPIN_US, saved)
