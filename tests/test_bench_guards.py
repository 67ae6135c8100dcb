"""bench.py cannot lose its line (VERDICT r02 Next #1): every optional leg
(config 1, host-inclusive, sweep entries) is guarded and wall-budgeted.  CPU
checks of the guards themselves; the GPU halves are in test_gpu_bench.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

import bench  # noqa: E402


def test_guarded_records_error_and_passes_results():
    def boom():
        raise RuntimeError("disk full")

    r = bench.guarded("config1", boom)
    assert r == {"error": "config1: RuntimeError: disk full"}
    assert bench.guarded("x", lambda a, b=0: {"v": a + b}, 1, b=2) == {"v": 3}
    assert "error" in bench.guarded("config1", lambda: None)


def test_sweep_past_deadline_skips_every_entry_without_touching_the_gpu():
    out = bench.sweep("cuda:0", 3, 1, deadline=0.0)
    assert [e["key"] for e in out] == [s[0] for s in bench.SWEEP]
    assert all("skipped" in e for e in out)


def test_config1_workdir_prefers_the_tree_and_reports_space(tmp_path):
    assert bench.config1_workdir(1 << 20, str(tmp_path)) == str(tmp_path)
    with pytest.raises(RuntimeError, match="no room"):
        bench.config1_workdir(1 << 62, str(tmp_path))


def test_config1_failure_still_prints_the_line():
    """--config 1 with the leg forced to raise: exit 0, one JSON line carrying
    the error (the default N=1 run prints its headline the same way:
    test_gpu_bench.py::test_bench_line_survives_failing_config1)."""
    env = dict(os.environ, PCS_BENCH_FAIL_CONFIG1="1")
    r = subprocess.run([sys.executable, "bench.py", "--config", "1"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert "PCS_BENCH_FAIL_CONFIG1" in d["error"] and d["value"] is None


def test_parity_ok_needs_every_check():
    """A rank passes only with zero digest mismatches, zero content
    mismatches (pages at its global indices) and a passing drill; bench.py
    exits 3 after the line when any rank does not."""
    good = {"mismatches": 0, "content_mismatches": 0}
    assert bench.parity_ok(good, {"pass": True})
    assert bench.parity_ok({"mismatches": 0}, {"pass": True})  # descriptor batches: no content check
    assert not bench.parity_ok(dict(good, mismatches=1), {"pass": True})
    assert not bench.parity_ok(dict(good, content_mismatches=2), {"pass": True})
    assert not bench.parity_ok(good, {"pass": False})
    assert not bench.parity_ok(None, {"pass": True}) and not bench.parity_ok(good, None)


def test_fill_pages_at_matches_contiguous_generator():
    from workload import fill_pages, fill_pages_at
    import numpy as np
    idx = np.array([5, 0, 4096, 77, 8191], dtype=np.int64)
    whole = fill_pages(0x5EED0005, 0, 8192, 256)
    assert np.array_equal(fill_pages_at(0x5EED0005, idx, 256), whole[idx])


def test_settle_runs_whole_batches_for_at_least_the_time(monkeypatch):
    """bench.settle: untimed steps in batches of 8, synchronised after each
    batch, until at least `ms` have passed; 0 ms runs nothing."""
    import time

    calls = {"step": 0, "sync": 0}

    class FakeWorkload:
        def step(self, mode):
            assert mode == "digest"
            calls["step"] += 1
            time.sleep(0.0005)

    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda: calls.__setitem__("sync", calls["sync"] + 1))
    assert bench.settle(FakeWorkload(), "digest", 0) == 0 and calls["step"] == 0
    t0 = time.perf_counter()
    n = bench.settle(FakeWorkload(), "digest", 30)
    assert time.perf_counter() - t0 >= 0.030
    assert n == calls["step"] and n % 8 == 0 and n >= 8 and calls["sync"] == n // 8
