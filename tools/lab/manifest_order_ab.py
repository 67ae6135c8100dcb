#!/usr/bin/env python3
"""Manifest checksum (pcs_manifest_checksum_dev, wide form) with the block-sum
kernel's workgroups in dispatch order against the chunked tile order
(a temporary tuning key 25, removed once the chunked order was kept),
interleaved in one process; result words compared.  Not part of the product.

    python tools/lab/manifest_order_ab.py [bytes ...]
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import eloqstore_amd as pcs  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [64 << 20, 256 << 20, 1 << 30, 4 << 30]
R, K = 7, 20
for L in sizes:
    buf = torch.empty(L, dtype=torch.uint8, device="cuda:0")
    pcs.gen_pages(buf, 4096, L // 4096, 99, 0)
    d_out = torch.empty(1, dtype=torch.int64, device="cuda:0")
    res, times = {}, {0: [], 1: []}
    for r in range(R):
        for v in ((0, 1) if r % 2 == 0 else (1, 0)):
            pcs.set_tuning(25, v + 1)
            s = torch.cuda.current_stream()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                pcs._call("pcs_manifest_checksum_dev", buf.data_ptr(), L, d_out.data_ptr(), pcs._stream(None))
            a.record(s)
            for _ in range(K):
                pcs._call("pcs_manifest_checksum_dev", buf.data_ptr(), L, d_out.data_ptr(), pcs._stream(None))
            b.record(s)
            b.synchronize()
            times[v].append(a.elapsed_time(b) / K * 1e3)
            res.setdefault(v, int(d_out.item()))
    pcs.set_tuning(25, 2)
    assert res[0] == res[1]
    for v, name in ((0, "dispatch"), (1, "chunked")):
        t = statistics.median(times[v])
        print(f"manifest {L >> 20:6d} MiB {name:9s} {t:9.1f} us  {L / t / 1e6:6.2f} TB/s", flush=True)
    del buf
