#!/usr/bin/env python3
"""kernel_lab.py — interleaved A/B of the product kernels under tuning knobs.

Not part of the product.  Times pcs_pages_digest_dev / pcs_desc_digest_dev
(through the C ABI) for each variant in interleaved rounds within one process
(cdna_hip_programming.md §5.4 rule 24) and prints median / best GB/s.

    python tools/lab/kernel_lab.py [--rounds 7] [--configs 2,4,3] [--algos xxh3,xxh64]
"""
import argparse
import ctypes
import os
import sys

if "--system-hip" in sys.argv:  # load ROCm's own HIP runtime before torch's bundled one
    ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7", mode=ctypes.RTLD_GLOBAL)

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import eloqstore_amd as pcs  # noqa: E402
from workload import mixed_layout  # noqa: E402

if "--lib" in sys.argv:  # A/B against another build of the library (e.g. an older commit)
    _path = os.path.abspath(sys.argv[sys.argv.index("--lib") + 1])
    _probe = ctypes.CDLL(_path)
    pcs.LIB_PATH = _path
    pcs._SIGS = {k: v for k, v in pcs._SIGS.items() if hasattr(_probe, k)}


def set_tuning_if_known(key, value):
    try:
        pcs.set_tuning(key, value)
    except pcs.PcsError:
        pass  # an older library without this knob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--configs", default="2,4,3")
    ap.add_argument("--algos", default="xxh3,xxh64")
    ap.add_argument("--bpc", default="1048576,8,32")  # 1048576 = uncapped (one block per 16 pages)
    ap.add_argument("--nt", default="0,1")
    ap.add_argument("--system-hip", action="store_true")
    ap.add_argument("--x64-layouts", default="0,1")
    ap.add_argument("--rt-batch", default="1", help="XXH3 run-time-size kernels: 1 = 4-block batches, 0 = one block")
    ap.add_argument("--split", default="8192", help="XXH3 split-page thresholds to compare (0 = group per page)")
    ap.add_argument("--sort", default="0", help="descriptor tile sort by size (XXH3 rt batch 1 only)")
    ap.add_argument("--dsplit", default="0", help="XXH3 descriptor pages in 4 KiB slices (1) or not (0, the product default)")
    ap.add_argument("--x64-sort", default="0", help="XXH64 descriptor tiles sorted by size (1) or not (0)")
    ap.add_argument("--x64-waves", default="4", help="XXH64 LDS kernel waves per workgroup (PCS_TUNE_XXH64_WAVES)")
    ap.add_argument("--b2b", type=int, default=0, help="time K back-to-back launches per sample (0 = one launch)")
    ap.add_argument("--lib", default=None, help="library to load instead of eloqstore_amd/libeloqstore_pcs.so")
    ap.add_argument("--raw-alloc", action="store_true", help="pages from a plain hipMalloc, not torch's allocator")
    args = ap.parse_args()
    dev = "cuda:0"
    print("torch", torch.__version__, "hip runtime:", [l for l in open("/proc/self/maps").read().split() if "amdhip64" in l][:1])
    bpcs = [int(x) for x in args.bpc.split(",")]
    nts = [int(x) for x in args.nt.split(",")]

    for cfg in [int(c) for c in args.configs.split(",")]:
        if cfg == 3:
            n = 1 << 20
            offs, lens, total = mixed_layout(0x5EED0003, 0, n)
            pages = torch.empty(total, dtype=torch.uint8, device=dev)
            d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
            d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
            pcs.gen_desc(pages, d_off, d_len, n, 0x5EED0003, 0)
            nbytes = total
            P = None
        else:
            # 6/7/8: 4 GiB of 8/16/32 KiB pages (not BASELINE configs; page-size sweeps)
            P, n = {2: (4096, 1 << 20), 4: (65536, 1 << 18), 5: (4096, 1 << 23), 6: (8192, 1 << 19),
                    7: (16384, 1 << 18), 8: (32768, 1 << 17)}[cfg]
            if args.raw_alloc:
                hip = ctypes.CDLL("libamdhip64.so.7")
                ptr = ctypes.c_void_p()
                assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(n * P)) == 0
                pages = ptr.value
            else:
                pages = torch.empty(n * P, dtype=torch.uint8, device=dev)
            pcs.gen_pages(pages, P, n, 0x5EED0000 + cfg, 0)
            nbytes = n * P
        out = torch.empty(n, dtype=torch.int64, device=dev)
        ref = {}
        variants = []
        for algo_name in args.algos.split(","):
            algo = pcs.XXH3_64 if algo_name == "xxh3" else pcs.XXH64
            key = pcs.TUNE_XXH3_BLOCKS_PER_CU if algo == 0 else pcs.TUNE_XXH64_BLOCKS_PER_CU
            layouts = [int(x) for x in (args.x64_layouts if algo == 1 else args.rt_batch).split(",")]
            splits = [int(x) for x in args.split.split(",")] if algo == 0 else [0]
            sorts = ([(a, b) for a in [int(x) for x in args.sort.split(",")] for b in [int(x) for x in args.dsplit.split(",")]]
                     if algo == 0 else [(a, w) for a in [int(x) for x in args.x64_sort.split(",")]
                                        for w in [int(x) for x in args.x64_waves.split(",")]])
            for lay in layouts:
                for sp in [(a, b) for a in splits for b in sorts]:
                    for bpc in bpcs:
                        for nt in nts:
                            tag = (f" lay={lay}" + (f" sort{sp[1][0]}" if sp[1][0] else "") + f" w={sp[1][1]}" if algo == 1 else f" rtb={lay}" + (f" split={sp[0]}" if sp[0] else "")
                                   + (" sort" if sp[1][0] else "") + (" dsplit" if sp[1][1] else ""))
                            variants.append((f"{algo_name}{tag} bpc={bpc} nt={nt}", algo, key, bpc, nt, "hash",
                                             (lay, sp)))
        has_desc_ceiling = "pcs_read_ceiling_desc_dev" in pcs._SIGS
        if P in (4096, 65536) or (P is None and has_desc_ceiling):
            for nt in nts:
                variants.append((f"read-ceiling bpc=0 nt={nt}", 0, pcs.TUNE_XXH3_BLOCKS_PER_CU, 0, nt, "ceil", (1, (8192, (0, 1)))))

        def run(v):
            _, algo, key, bpc, nt, kind, (lay, (sp, (srt, dsp))) = v
            pcs.set_tuning(key, bpc)
            pcs.set_tuning(pcs.TUNE_XXH3_SPLIT_PAGES, sp if sp >= 0 else 0)
            pcs.set_tuning(pcs.TUNE_DESC_SORT, srt if algo == 0 else 0)
            set_tuning_if_known(pcs.TUNE_XXH64_DESC_SORT, srt if algo == 1 else 0)
            pcs.set_tuning(pcs.TUNE_DESC_SPLIT, dsp if algo == 0 else 0)
            set_tuning_if_known(pcs.TUNE_XXH64_WAVES, dsp if algo == 1 and dsp else 4)
            if algo == 1:
                pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, lay)
            else:
                pcs.set_tuning(pcs.TUNE_XXH3_RT_BATCH, lay)
            if algo == 1 and lay == 1:
                pcs.set_tuning(pcs.TUNE_XXH64_NT_LOADS, nt)
            else:
                pcs.set_tuning(pcs.TUNE_NT_LOADS, nt)
            if kind == "ceil" and P is None:
                pcs.read_ceiling_desc(pages, d_off, d_len, n, out)
            elif kind == "ceil":
                pcs.read_ceiling(pages, P, n, out)
            elif P is None:
                pcs.desc_digest(pages, d_off, d_len, n, algo, out=out)
            else:
                pcs.pages_digest(pages, P, n, algo, out=out)

        times = {v[0]: [] for v in variants}
        for v in variants:  # warm + parity across variants
            run(v)
            torch.cuda.synchronize()
            if v[5] == "hash":
                d = out.clone()
                if v[1] in ref:
                    assert torch.equal(ref[v[1]], d), f"variant {v[0]} changed the digests"
                else:
                    ref[v[1]] = d
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.rounds):
            for v in variants:
                if args.b2b:  # K launches back to back, like bench.py's timed loop
                    torch.cuda.synchronize()
                    ev0.record()
                    for _k in range(args.b2b):
                        run(v)
                    ev1.record()
                    torch.cuda.synchronize()
                    times[v[0]].append(ev0.elapsed_time(ev1) / args.b2b)
                    continue
                torch.cuda._sleep(1_000_000)  # keep the GPU busy while the launch is enqueued
                ev0.record()
                run(v)
                ev1.record()
                torch.cuda.synchronize()
                times[v[0]].append(ev0.elapsed_time(ev1))
        print(f"== config {cfg}: {n} pages, {nbytes / 2**30:.2f} GiB", flush=True)
        for name, t in times.items():
            t = sorted(t)
            med = t[len(t) // 2]
            print(f"  {name:28s} med {med:8.4f} ms  {nbytes / med / 1e6:8.1f} GB/s  best {nbytes / t[0] / 1e6:8.1f}",
                  flush=True)
        if not isinstance(pages, int):
            del pages
        del out
        torch.cuda.empty_cache()
    pcs.set_tuning(pcs.TUNE_XXH3_BLOCKS_PER_CU, 0)
    pcs.set_tuning(pcs.TUNE_XXH64_BLOCKS_PER_CU, 0)
    pcs.set_tuning(pcs.TUNE_NT_LOADS, 1)
    pcs.set_tuning(pcs.TUNE_XXH64_NT_LOADS, 0)
    pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, 0)


if __name__ == "__main__":
    main()
