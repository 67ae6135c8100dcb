"""Runs INTEGRATION.md's call-site snippets on the GPU (built by
tests/cpp/gen_integration.py in the build container, where the reference's
page.h exists; the binary travels with the tree).

The binary drives the ReadPages validate loop (sync and async, registered pool
and heap pages, a corrupted page at index 77, skip_verify_checksum), and the
WritePage / FlushBatchPages stamping in append and non-append mode, with the
CPU oracle checking every stamped header.  Both sides of the batch-size gate
(kGpuChecksumMinBatchBytes) run: a 128-page read batch and a 256-page write
batch on the GPU, a 6-page scan-prefetch batch (types.h:31) and a 10-page
write tail on page.cpp's CPU loop, told apart by call counters and
pcs_counter().  Manifest records below and above kGpuManifestMinBytes go
through Finalize, ValidateChecksum and the replay check (replayer.cpp:92),
with a flipped byte rejected.  With the validate service on, the async
snippet and straight ChecksumBatch batches (6 and 32 pages, stamps) are
served by it, and a service stopped under an in-flight batch re-runs it on
the launch path.  An injected GPU failure (PCS_TUNE_FAIL_INJECT) makes the
sync and async read snippets and the flush snippet fall back to page.cpp's
loop, which still finds the corrupted page."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "integration_snippets")

pytestmark = pytest.mark.gpu


def test_integration_snippets_run():
    assert os.path.exists(BIN), "tests/cpp/integration_snippets missing: run __graft_entry__.build() with the reference tree present"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "integration ok" in r.stdout
    assert "read path source=registered: ok" in r.stdout and "read path source=heap: ok" in r.stdout
    assert "write path append=1: 256 pages stamped (GPU batch)" in r.stdout
    assert "write path append=1: 10 pages stamped (reference loop)" in r.stdout
    assert "write path append=0: 40 pages stamped (reference loop)" in r.stdout
    # between the read gate (32 pages) and the write gate (48): the loop; at 48: the GPU
    assert "write path append=1: 40 pages stamped (reference loop)" in r.stdout
    assert "write path append=1: 48 pages stamped (GPU batch)" in r.stdout
    assert "6-page scan batch on the reference loop" in r.stdout
    assert "read path with the validate service: ok (32 and 128 pages served, 6 on the reference loop" in r.stdout
    assert "async batch of 6 pages through the service: ok" in r.stdout
    assert "async batch of 32 pages through the service: ok" in r.stdout
    assert "stop during an async batch re-runs it" in r.stdout
    assert "GPU failure fallback: ok" in r.stdout
    assert r.stdout.count("manifest record") == 2
    assert "(reference loop)" in r.stdout.split("manifest record")[1] and "(GPU)" in r.stdout.split("manifest record")[2]
