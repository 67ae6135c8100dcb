"""CPU-side checks of the native boundary (no GPU needed, no compute calls).

- libeloqstore_pcs.so loads and exports every pcs_* symbol include/eloqstore_pcs.h
  declares, plus the C++ drop-in symbols of include/eloqstore/page_checksum.h;
- without a GPU every compute entry point fails loudly (PCS_ERR_NO_DEVICE),
  never silently falling back to a CPU path;
- argument validation and the pure host logic (shard ranges);
- the CLI's usage / IO error contract (tools/page_checksum_tool.cpp:47-99).
"""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import eloqstore_amd as pcs

HAVE_GPU = pcs.device_count() > 0


def test_library_exports_every_header_symbol():
    funcs = pcs.header_functions()
    assert len(funcs) >= 20
    so = pcs.lib()
    for f in funcs:
        assert hasattr(so, f), f
    # and the binding covers exactly the header
    assert set(funcs) == set(pcs._SIGS)


SINGLE_PAGE = ("eloqstore::SetChecksum(std::basic_string_view<char, std::char_traits<char> >)",
               "eloqstore::ValidateChecksum(std::basic_string_view<char, std::char_traits<char> >)")


def _exports(path):
    return subprocess.run(["nm", "-D", "-C", "--defined-only", path], capture_output=True, text=True,
                          check=True).stdout


def test_cpp_dropin_symbols_exported():
    """The batch library exports the batched C++ forms but NOT page.h's two
    single-page names (include/storage/page.h:25-26): those live only in the
    opt-in libeloqstore_pcs_dropin.so, so linking the batch library can never
    interpose on page.cpp's definitions, whatever the link or DSO order."""
    out = _exports(pcs.LIB_PATH)
    for sym in ("eloqstore::ValidateChecksums(", "eloqstore::SetChecksums(", "eloqstore::PageDigests(",
                "eloqstore::TryValidateChecksums(", "eloqstore::TrySetChecksums(", "eloqstore::LastChecksumError()",
                "eloqstore::ChecksumBatch::Poll()", "eloqstore::ChecksumBatch::TryPoll()",
                "eloqstore::ChecksumBatch::TrySubmitValidate(", "eloqstore::ManifestChecksum(",
                "eloqstore::ValidateManifestRecord(", "eloqstore::RegisterPagePool(", "eloqstore::UnregisterPagePool("):
        assert sym in out, sym
    for sym in SINGLE_PAGE:
        assert sym not in out, sym
    drop = _exports(pcs.DROPIN_LIB_PATH)
    for sym in SINGLE_PAGE:
        assert sym in drop, sym
    assert "eloqstore::ValidateChecksums(" not in drop


@pytest.mark.parametrize("order", ["ref_first", "pcs_first"])
def test_single_page_calls_resolve_to_page_cpp_in_any_link_order(order):
    """A shared object defining page.cpp's SetChecksum / ValidateChecksum
    (tests/cpp/ref_page_stub.cpp, as an EloqStore embedded as a DSO would
    carry them) linked beside the batch library in both orders: every
    single-page call reaches it (its call counter), and without a GPU the
    non-aborting batch form reports PCS_ERR_NO_DEVICE instead of aborting.
    The GPU half (tests/test_gpu_parity.py) runs the batched API beside it."""
    exe = os.path.join(os.path.dirname(__file__), "cpp", f"linkorder_{order}")
    args = [exe] + (["--gpu"] if HAVE_GPU else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "linkorder ok" in r.stdout, r.stdout + r.stderr


def test_fail_inject_knob_fails_host_batches_loudly():
    """PCS_TUNE_FAIL_INJECT (test only): the next k host-batch calls fail with
    PCS_ERR_HIP before touching the GPU, so call sites can prove their
    fallback to the reference loop."""
    so = pcs.lib()
    pages = [bytearray(4096) for _ in range(3)]
    arr, _keep = pcs._page_ptrs(pages)
    okb = (ctypes.c_uint8 * 3)()
    fbv = ctypes.c_uint64()
    try:
        pcs.set_tuning(pcs.TUNE_FAIL_INJECT, 2)
        assert pcs.get_tuning(pcs.TUNE_FAIL_INJECT) == 2
        assert so.pcs_pages_validate_host(arr, 4096, 3, 0, okb, ctypes.byref(fbv)) == pcs.PCS_ERR_HIP
        assert b"injected failure" in so.pcs_last_error()
        assert so.pcs_pages_stamp_host(arr, 4096, 3, 0) == pcs.PCS_ERR_HIP
        assert pcs.get_tuning(pcs.TUNE_FAIL_INJECT) == 0
        # skip_verify computes nothing, so it never fails
        assert so.pcs_pages_validate_host_ex(arr, 4096, 3, 0, okb, ctypes.byref(fbv), 1) == pcs.PCS_OK
    finally:
        pcs.set_tuning(pcs.TUNE_FAIL_INJECT, 0)


def test_version_string():
    assert "gfx950" in pcs.version()


def test_abi_version_matches_header():
    """the library reports the header revision it was built
    from; callers compare it with PCS_ABI_VERSION at start-up."""
    import re
    text = open(pcs.HEADER_PATH).read()
    want = int(re.search(r"#define PCS_ABI_VERSION (\d+)", text).group(1))
    assert pcs.abi_version() == want == pcs.ABI_VERSION


@pytest.mark.skipif(HAVE_GPU, reason="checks the no-GPU failure path")
def test_no_gpu_fails_loudly():
    so = pcs.lib()
    rc = so.pcs_pages_digest_dev(0, 4096, 1, 0, 0, 0)
    assert rc == pcs.PCS_ERR_NO_DEVICE
    assert b"no usable HIP device" in so.pcs_last_error()
    for fn, args in (("pcs_pages_validate_dev", (0, 4096, 1, 0, 0, 0, 0)),
                     ("pcs_pages_stamp_dev", (0, 4096, 1, 0, 0)),
                     ("pcs_desc_digest_dev", (0, 0, 0, 1, 0, 0, 0)),
                     ("pcs_xxh3_64_ranges_dev", (0, 0, 0, 1, 0, 0)),
                     ("pcs_gen_pages_dev", (0, 4096, 1, 0, 0, 0)),
                     ("pcs_host_register", (4096, 4096))):
        assert getattr(so, fn)(*args) == pcs.PCS_ERR_NO_DEVICE, fn
    with pytest.raises(pcs.PcsError):
        pcs.validate_checksum(bytearray(4096))


def test_shard_range_partitions_exactly():
    for n in (0, 1, 7, 1 << 20, (1 << 26) + 3):
        for world in (1, 2, 3, 4, 8):
            spans = [pcs.shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            for (b0, e0), (b1, e1) in zip(spans, spans[1:]):
                assert e0 == b1
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_rank():
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    assert pcs.lib().pcs_shard_range(10, 2, 2, ctypes.byref(b), ctypes.byref(e)) == pcs.PCS_ERR_INVALID
    assert pcs.lib().pcs_shard_range(10, 0, 0, ctypes.byref(b), ctypes.byref(e)) == pcs.PCS_ERR_INVALID


def run_tool(*args):
    return subprocess.run([pcs.TOOL_PATH, *args], capture_output=True, text=True)


def test_cli_usage_errors(tmp_path):
    assert os.access(pcs.TOOL_PATH, os.X_OK)
    r = run_tool()
    assert r.returncode == 1 and "Usage:" in r.stderr
    r = run_tool("a", "b", "c", "d")
    assert r.returncode == 1 and "Usage:" in r.stderr
    f = tmp_path / "f.bin"
    f.write_bytes(b"\0" * 8192)
    for bad in ("x12", "12x", "", "0x"):
        r = run_tool(str(f), bad)
        assert r.returncode == 1 and "Invalid offset" in r.stderr, bad
    r = run_tool(str(f), "0", "0")
    assert r.returncode == 1 and "Invalid page size: 0" in r.stderr
    r = run_tool(str(f), "4097")
    assert r.returncode == 1 and "Requested range [4097, 8193) exceeds file size 8192" in r.stderr
    r = run_tool(str(f), "0x1001", "0x1000")
    assert r.returncode == 1 and "Requested range [4097, 8193)" in r.stderr
    r = run_tool(str(tmp_path / "missing.bin"), "0")
    assert r.returncode == 1 and "Failed to open" in r.stderr


@pytest.mark.skipif(HAVE_GPU, reason="checks the no-GPU failure path")
def test_cli_without_gpu_fails_loudly(tmp_path):
    f = tmp_path / "f.bin"
    f.write_bytes(b"\0" * 8192)
    r = run_tool(str(f), "010")  # octal 8, as std::stoull(base 0) parses it
    assert r.returncode not in (0, 2)
    assert "no usable HIP device" in r.stderr


def test_counters_and_tuning_defaults():
    assert pcs.counter(pcs.COUNTER_ZERO_COPY_LAUNCHES) >= 0
    assert pcs.lib().pcs_counter(99) == 0
    assert pcs.get_tuning(pcs.TUNE_ZERO_COPY) == 1
    assert pcs.get_tuning(5) == -1  # retired (in-place stamp width)
    assert pcs.get_tuning(pcs.TUNE_XXH3_SPLIT_PAGES) == 8192
    assert pcs.get_tuning(pcs.TUNE_INLINE_LIST) == 1
    assert pcs.get_tuning(pcs.TUNE_SERVICE_MAX_CALLERS) == 2
    assert pcs.get_tuning(pcs.TUNE_SERVICE_TEAR_TEST) == 0
    assert pcs.get_tuning(pcs.TUNE_FAIL_INJECT) == 0
    assert pcs.lib().pcs_counter(pcs.COUNTER_SERVICE_TORN_REQUESTS) == 0
    assert pcs.get_tuning(pcs.TUNE_SERVICE_REPOST_TEST) == 0
    assert pcs.lib().pcs_counter(pcs.COUNTER_SERVICE_REPOSTS) == 0


def test_skip_verify_flag_needs_no_gpu():
    """PCS_FLAG_SKIP_VERIFY mirrors KvOptions::skip_verify_checksum
    (kv_options.h:41): the reference skips the validate loop entirely
    (async_io_manager.cpp:239, 353), so nothing is hashed: every verdict is 1,
    first_bad is UINT64_MAX, and the call succeeds even without a GPU.  The
    arguments are still checked."""
    pages = [bytearray(4096) for _ in range(5)]  # all-zero pages never validate
    ok, fb = pcs.validate_checksums(pages, 4096, skip_verify=True)
    assert ok == [1] * 5 and fb is None
    ok, fb = pcs.validate_ptrs(np.zeros(0, dtype=np.uint64), 4096, skip_verify=True)
    assert len(ok) == 0 and fb is None
    so = pcs.lib()
    arr, _keep = pcs._page_ptrs(pages)
    okb = (ctypes.c_uint8 * 5)()
    fbv = ctypes.c_uint64()
    assert so.pcs_pages_validate_host_ex(arr, 4096, 5, 7, okb, ctypes.byref(fbv), 1) == pcs.PCS_ERR_INVALID
    assert so.pcs_pages_validate_host_ex(arr, 4, 5, 0, okb, ctypes.byref(fbv), 1) == pcs.PCS_ERR_INVALID
    assert so.pcs_pages_validate_host_ex(arr, 4096, 5, 0, okb, ctypes.byref(fbv), 2) == pcs.PCS_ERR_INVALID
    assert b"unknown flag" in so.pcs_last_error()
    nulls = (ctypes.c_void_p * 2)(arr[0], None)
    assert so.pcs_pages_validate_host_ex(nulls, 4096, 2, 0, okb, ctypes.byref(fbv), 1) == pcs.PCS_ERR_INVALID
