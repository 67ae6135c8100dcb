#!/usr/bin/env python3
"""alloc_lab.py — does the same kernel over the same byte count run at a
different rate depending on where its buffer landed in HBM?

tools/lab/drift_lab.py (profiles/r02/drift_lab.txt) showed each resident
buffer timing stable to +-0.3 % over minutes and positions, but config 5's
32 GiB buffer at 0.81 of peak on one box and 0.93 on others.  This allocates
several buffers of one size in a row, by torch (hipMalloc) and by
hipExtMallocWithFlags(hipDeviceMallocContiguous), fills each with the same
synthetic pages, and times k_xxh3_fixed<4096> (pcs_pages_digest_dev) and the
plain streaming read (pcs_stream_read_dev) on each, interleaved over rounds.

    python tools/lab/alloc_lab.py [--gib 32] [--count 3] [--rounds 3]
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import eloqstore_amd as pcs  # noqa: E402

P = 4096
HIP_DEVICE_MALLOC_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=int, default=32)
    ap.add_argument("--count", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    nbytes = args.gib << 30
    n = nbytes // P
    bufs = []
    for i in range(args.count):
        t = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
        bufs.append((f"torch#{i}", t.data_ptr(), t))
    for i in range(args.count):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, HIP_DEVICE_MALLOC_CONTIGUOUS)
        if rc != 0:
            print(f"# contiguous#{i}: hipExtMallocWithFlags rc={rc}", flush=True)
            continue
        bufs.append((f"contig#{i}", p.value, None))
    out = torch.empty(n, dtype=torch.int64, device="cuda:0")
    scratch = torch.empty((nbytes + 4095) // 4096, dtype=torch.int64, device="cuda:0")
    for name, ptr, _ in bufs:
        pcs.gen_pages(ptr, P, n, 0x5EED0005, 0)
    torch.cuda.synchronize()
    ref = None
    for name, ptr, _ in bufs:
        pcs.pages_digest(ptr, P, n, 0, out=out)
        torch.cuda.synchronize()
        h = int(out[::4099].sum().item())
        ref = h if ref is None else ref
        print(f"# {name}: ptr {ptr:#x} digest-sample-sum {'ok' if h == ref else 'MISMATCH'}", flush=True)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 1e3 / args.steps

    res = {}
    n4 = min(n, (4 << 30) // P)  # the buffer's first 4 GiB alone
    for r in range(args.rounds):
        for name, ptr, _ in bufs:
            td = timed(lambda: pcs.pages_digest(ptr, P, n, 0, out=out))
            ts = timed(lambda: pcs.stream_read(ptr, nbytes, scratch))
            t4 = timed(lambda: pcs.pages_digest(ptr, P, n4, 0, out=out))
            res.setdefault(name, []).append((td, ts, t4))
            print(f"round {r} {name:10s} digest {td * 1e3:8.3f} ms {(nbytes + 8 * n) / td / 1e12:6.3f} TB/s   "
                  f"stream {ts * 1e3:8.3f} ms {nbytes / ts / 1e12:6.3f} TB/s   "
                  f"first 4 GiB {n4 * (P + 8) / t4 / 1e12:6.3f} TB/s", flush=True)
    print("# buffer      digest TB/s (med)   stream TB/s (med)   first-4-GiB digest TB/s (med)")
    for name, v in res.items():
        d = statistics.median((nbytes + 8 * n) / x[0] / 1e12 for x in v)
        s = statistics.median(nbytes / x[1] / 1e12 for x in v)
        f4 = statistics.median(n4 * (P + 8) / x[2] / 1e12 for x in v)
        print(f"# {name:10s}  {d:8.3f}            {s:8.3f}            {f4:8.3f}")
    for name, ptr, t in bufs:
        if t is None:
            hip.hipFree(ctypes.c_void_p(ptr))


if __name__ == "__main__":
    main()
