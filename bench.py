#!/usr/bin/env python3
"""bench.py — device-resident batched page checksum throughput on MI355X.

Metric (BASELINE.json): GiB/s of device-resident batched page XXH3-64 over
4 KiB pages on 1/2/4/8 MI355X.  A "step" is one pass of the hot path
(pcs_pages_digest_dev -> the XXH3 page kernel) over one batch of synthetic
pages already resident in HBM; value = page bytes hashed by ALL ranks per
second (GiB/s, 2^30), per-GPU work fixed (weak scaling: every rank owns its
own disjoint page range, no collective on the data path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5|6|7]

Default (N=1) = BASELINE config 2: 1,048,576 x 4 KiB pages (4 GiB) per GPU.
Configs 6/7 are the north star's 8/16 KiB page-size sweep (4 GiB per GPU).
Multi-GPU: launched by torch.distributed.run, one process per GPU; gloo is the
control plane (barrier + max over ranks of the timed region).

Also reported, on the same line:
  roofline      dominant kernel's algorithmic bytes per launch / average launch
                time (HIP events on the launch stream) vs 8 TB/s HBM peak;
                traffic = PMC-measured HBM bytes per launch when a matching
                rocprofv3 summary is committed under profiles/ (else null).
  read_ceiling  the same load pattern with the hash removed (achievable rate).
  cpu_baseline  the reference's own xxHash (oracle/_ref, one XXH3_64bits call
                per page like page.cpp:18-31) on ONE host core over a bounded
                sample of the same pages; its digests double as a parity check.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import eloqstore_amd as pcs  # noqa: E402

METRIC = "GiB/s device-resident batched page XXH3-64, 4 KiB pages, 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X spec 8.0 TB/s (MI355X_MICROARCH.md chip table)
GIB = float(1 << 30)

CONFIGS = {
    # name: (page_size or None for mixed, pages per GPU, seed, description)
    2: (4096, 1 << 20, 0x5EED0002, "config2: 4 KiB pages, 1M-page device-resident batch per GPU"),
    3: (None, 1 << 20, 0x5EED0003, "config3: mixed 4/8/16 KiB pages, 1M pages per GPU, packed + descriptors"),
    4: (65536, 1 << 18, 0x5EED0004, "config4: 64 KiB chunks, 256K chunks device-resident per GPU"),
    5: (4096, 1 << 23, 0x5EED0005, "config5: 4 KiB pages, 8M pages per GPU (64M over 8 GPUs)"),
    # page-size sweep named in BASELINE.json's north_star (4 / 16 / 64 KiB batches), not numbered
    # BASELINE configs: 4 GiB per GPU like config 2 (same numbering as tools/lab/kernel_lab.py)
    6: (8192, 1 << 19, 0x5EED0006, "sweep: 8 KiB pages, 512K-page device-resident batch per GPU"),
    7: (16384, 1 << 18, 0x5EED0007, "sweep: 16 KiB pages, 256K-page device-resident batch per GPU"),
}


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def init_dist(world: int):
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        return dist
    return None


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


class Workload:
    """Device-resident pages of this rank's shard plus the timed step."""

    def __init__(self, cfg: int, algo: int, rank: int, pages_per_gpu: int | None, dev: str):
        P, n, seed, desc = CONFIGS[cfg]
        self.cfg, self.algo, self.seed, self.desc = cfg, algo, seed, desc
        self.n = pages_per_gpu or n
        self.first = rank * self.n  # disjoint global page range of this rank
        self.P = P
        self.dev = dev
        if P is not None:
            self.bytes = self.n * P
            self.pages = torch.empty(self.bytes, dtype=torch.uint8, device=dev)
            pcs.gen_pages(self.pages, P, self.n, seed, self.first)
            self.out = torch.empty(self.n, dtype=torch.int64, device=dev)
        else:
            from workload import mixed_layout
            offs, lens, total = mixed_layout(seed, self.first, self.n)
            self.offs, self.lens = offs, lens
            self.bytes = total
            self.pages = torch.empty(total, dtype=torch.uint8, device=dev)
            self.d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
            self.d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
            pcs.gen_desc(self.pages, self.d_off, self.d_len, self.n, seed, self.first)
            self.out = torch.empty(self.n, dtype=torch.int64, device=dev)
        self.ok = torch.empty(self.n, dtype=torch.uint8, device=dev)
        self.fb = torch.empty(1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()

    def step(self, mode: str = "digest"):
        if self.P is not None:
            if mode == "digest":
                pcs.pages_digest(self.pages, self.P, self.n, self.algo, out=self.out)
            elif mode == "validate":
                pcs.pages_validate(self.pages, self.P, self.n, self.algo, ok=self.ok, first_bad=self.fb)
            else:
                pcs.pages_stamp(self.pages, self.P, self.n, self.algo)
        else:
            if mode == "digest":
                pcs.desc_digest(self.pages, self.d_off, self.d_len, self.n, self.algo, out=self.out)
            elif mode == "validate":
                pcs.desc_validate(self.pages, self.d_off, self.d_len, self.n, self.algo, ok=self.ok, first_bad=self.fb)
            else:
                pcs.desc_stamp(self.pages, self.d_off, self.d_len, self.n, self.algo)

    def corruption_drill(self, every: int = 1000):
        """Untimed self-check (persist.cpp:241-246 style): stamp every page,
        validate (all pass), flip byte 10 of every `every`-th page, validate:
        exactly those must fail and the first bad index must be 0."""
        if self.P is None:
            return None
        pcs.pages_stamp(self.pages, self.P, self.n, self.algo)
        pcs.pages_validate(self.pages, self.P, self.n, self.algo, ok=self.ok, first_bad=self.fb)
        clean = int(self.ok.sum().item())
        pcs.flip_byte(self.pages, self.P, self.n, every=every, byte_offset=10)
        pcs.pages_validate(self.pages, self.P, self.n, self.algo, ok=self.ok, first_bad=self.fb)
        flipped = (self.n + every - 1) // every
        detected = int((self.ok == 0).sum().item())
        first = int(self.fb.item())
        pcs.flip_byte(self.pages, self.P, self.n, every=every, byte_offset=10)  # restore
        return {"pages": self.n, "valid_after_stamp": clean, "flipped": flipped, "detected": detected,
                "first_bad": first, "pass": clean == self.n and detected == flipped and first == 0}

    def algorithmic_bytes(self, mode: str = "digest") -> int:
        # every page byte read once (the 8-byte header shares the first line) + the result written:
        # 8 B digest (digest), 1 B verdict (validate), 8 B into the page (stamp)
        return self.bytes + (1 if mode == "validate" else 8) * self.n

    def read_ceiling(self, reps: int) -> float | None:
        scratch = torch.empty_like(self.out)  # keep self.out = the digests of the timed steps
        if self.P is None:  # mixed sizes: the descriptor kernel's load pattern
            def run():
                pcs.read_ceiling_desc(self.pages, self.d_off, self.d_len, self.n, scratch)
        elif self.P in (256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536):
            def run():
                pcs.read_ceiling(self.pages, self.P, self.n, scratch)
        else:
            return None
        run()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(reps):
            run()
        ev[1].record()
        torch.cuda.synchronize()
        t = ev[0].elapsed_time(ev[1]) / 1e3 / reps
        return self.algorithmic_bytes() / t / 1e9

    def sample_pages_host(self, max_bytes: int):
        """(host uint8 array, page size, gpu digests) for a leading sample of the batch."""
        if self.P is not None:
            k = max(1, min(self.n, max_bytes // self.P))
            host = self.pages[: k * self.P].cpu().numpy()
            return host, self.P, self.out[:k].cpu().numpy().view(np.uint64)
        return None


def cpu_baseline(w: Workload, target_s: float):
    """Reference xxHash on one host core over a bounded sample of the same pages."""
    import oracle  # test/baseline infrastructure only (see oracle/__init__.py)

    if w.P is None:
        from workload import fill_desc
        k = 16384
        host = fill_desc(w.seed, w.first, w.offs[:k], w.lens[:k], int(w.offs[k - 1]) + int(w.lens[k - 1]))
        gpu = w.out[:k].cpu().numpy().view(np.uint64)
        ref = oracle.ref_desc_digest(host, w.offs[:k], w.lens[:k], w.algo) is not None
        fn = oracle.ref_desc_digest if ref else oracle.desc_digest
        t0 = time.perf_counter()
        reps = 0
        while True:
            want = fn(host, w.offs[:k], w.lens[:k], w.algo)
            reps += 1
            if time.perf_counter() - t0 >= target_s:
                break
        dt = time.perf_counter() - t0
        what = ("reference external/xxhash.c v0.8.3 (gcc -O2, SSE2 path), one call per page" if ref
                else "oracle C restatement, one call per page")
        return {"value": reps * host.nbytes / dt / GIB, "unit": "GiB/s", "cores": 1,
                "kind": "reference" if ref else "port",
                "sample": f"first {k} mixed pages ({host.nbytes / 2**20:.0f} MiB) of the batch x {reps} passes; {what}"}, \
            {"pages": k, "mismatches": int((want != gpu).sum())}
    host, P, gpu = w.sample_pages_host(256 << 20)
    fn = oracle.ref_pages_digest if oracle.ref_lib() is not None else None
    kind = "reference" if fn else "port"
    if fn is None:
        fn = oracle.pages_digest
    want = fn(host, P, w.algo)
    t0 = time.perf_counter()
    reps = 0
    while True:
        fn(host, P, w.algo)
        reps += 1
        if time.perf_counter() - t0 >= target_s:
            break
    dt = time.perf_counter() - t0
    what = ("reference external/xxhash.c v0.8.3 (gcc -O2, SSE2 path), one XXH3_64bits call per page"
            if kind == "reference" else "oracle C restatement, one call per page")
    if w.algo == pcs.XXH64:
        what = what.replace("XXH3_64bits", "XXH64")
    return {"value": reps * host.nbytes / dt / GIB, "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": f"first {host.nbytes // P} pages ({host.nbytes >> 20} MiB) of the batch x {reps} passes; {what}"}, \
        {"pages": int(host.nbytes // P), "mismatches": int((want != gpu).sum())}


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_all_cores(w: Workload, target_s: float):
    """The same reference loop on several host threads (disjoint page ranges of
    the sample), for context: BASELINE.md's all-cores CPU figure."""
    import threading

    import oracle  # baseline infrastructure only

    if w.P is None or oracle.ref_lib() is None:
        return None
    host, P, _ = w.sample_pages_host(256 << 20)
    k = host.nbytes // P
    nthreads = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    parts = [host[i * k // nthreads * P:(i + 1) * k // nthreads * P] for i in range(nthreads)]
    done = [0] * nthreads
    stop = time.perf_counter() + target_s

    def run(i):
        while time.perf_counter() < stop:
            oracle.ref_pages_digest(parts[i], P, w.algo)
            done[i] += parts[i].nbytes

    t0 = time.perf_counter()
    th = [threading.Thread(target=run, args=(i,)) for i in range(nthreads)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(sum(done) / dt / GIB, 2), "unit": "GiB/s", "cores": nthreads, "kind": "reference",
            "cpu": cpu_model(), "sample": f"{k} pages split over {nthreads} threads, ~{target_s:.0f} s"}


def host_inclusive(w: Workload, max_pages: int = 1 << 18):
    """Pages starting in host memory: H2D + kernel + D2H of digests, through
    pcs_pages_digest_host.  (a) one contiguous pinned run -> direct DMA;
    (b) pageable pages -> gather into pinned staging.  Not the headline value."""
    if w.P is None:
        return None
    k = min(w.n, max_pages)
    nbytes = k * w.P
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(w.pages[:nbytes])
    pageable = pinned.numpy().copy()
    digests = np.empty(k, dtype=np.uint64)
    res = {"pages": k, "page_size": w.P, "bytes": nbytes}
    for name, base in (("direct_pinned", pinned.data_ptr()), ("gather_pageable", pageable.ctypes.data)):
        ptrs = (np.arange(k, dtype=np.uint64) * np.uint64(w.P) + np.uint64(base))
        fn = pcs.lib().pcs_pages_digest_host
        rc = fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)  # warm (allocates staging)
        assert rc == 0, pcs.lib().pcs_last_error()
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 2.0:
            fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        res[f"{name}_GiBps"] = round(nbytes / dt / GIB, 2)
        res[f"{name}_digests_match_device"] = bool(np.array_equal(digests, w.out[:k].cpu().numpy().view(np.uint64)))
    # Scattered pool pages (a random permutation, like pages spread over
    # PagesPool chunks): (c) unregistered -> gather; (d) registered pool ->
    # zero-copy, one launch reading the pages in place.
    perm = np.random.default_rng(7).permutation(k).astype(np.uint64)
    want = w.out[:k].cpu().numpy().view(np.uint64)[perm]
    with pcs.PagePool(k, w.P) as pool:
        pool.pages.reshape(-1)[:] = pageable
        for name, base in (("gather_scattered", pageable.ctypes.data), ("zero_copy_scattered", pool.base)):
            ptrs = perm * np.uint64(w.P) + np.uint64(base)
            fn = pcs.lib().pcs_pages_digest_host
            rc = fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)
            assert rc == 0, pcs.lib().pcs_last_error()
            reps, t0 = 0, time.perf_counter()
            while reps < 3 or time.perf_counter() - t0 < 2.0:
                fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)
                reps += 1
            dt = (time.perf_counter() - t0) / reps
            res[f"{name}_GiBps"] = round(nbytes / dt / GIB, 2)
            res[f"{name}_digests_match_device"] = bool(np.array_equal(digests, want))
        res["batch_latency_us"] = batch_latency(pool, pageable, w)
    return res


def batch_latency(pool, pageable, w: Workload):
    """Median wall time of one validate call over a read-path-sized batch
    (max_read_pages_batch = 128, kv_options.h:18-19; write batches <= 256),
    scattered pages: staged (gather) vs zero-copy (registered pool), and the
    async form (submit + poll spin) on the registered pool."""
    out = {}
    rng = np.random.default_rng(11)
    for nb in (1, 16, 128, 256):
        idx = rng.permutation(pool.n)[:nb].astype(np.uint64)
        row = {}
        for name, base in (("gather", pageable.ctypes.data), ("zero_copy", pool.base)):
            ptrs = idx * np.uint64(w.P) + np.uint64(base)
            ok = np.empty(nb, dtype=np.uint8)
            fb = ctypes.c_uint64()
            fn = pcs.lib().pcs_pages_validate_host
            ts = []
            for _ in range(200):
                t0 = time.perf_counter()
                fn(ptrs.ctypes.data, w.P, nb, w.algo, ok.ctypes.data, ctypes.byref(fb), 0)
                ts.append(time.perf_counter() - t0)
            row[name] = round(float(np.median(ts[20:])) * 1e6, 1)
        b = pcs.Batch()
        ptrs = idx * np.uint64(w.P) + np.uint64(pool.base)
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            b.submit_ptrs(pcs.Batch.VALIDATE, ptrs, w.P, w.algo)
            while not b.poll():
                pass
            ts.append(time.perf_counter() - t0)
        b.close()
        row["zero_copy_async"] = round(float(np.median(ts[20:])) * 1e6, 1)
        out[str(nb)] = row
    return out


def committed_traffic(cfg: int, algo: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        key = f"config{cfg}_{'xxh3' if algo == 0 else 'xxh64'}"
        if key in d.get("traffic_bytes_per_launch", {}):
            best = (d["traffic_bytes_per_launch"][key], os.path.relpath(path, ROOT))
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--algo", choices=["xxh3", "xxh64"], default="xxh3")
    ap.add_argument("--pages-per-gpu", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["digest", "validate", "stamp"], default="digest",
                    help="digest (metric), validate (read path), stamp (write path)")
    ap.add_argument("--all-cores", action="store_true", help="also time the CPU reference on all host threads")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="also time the host-memory path (pinned direct DMA and pageable gather)")
    args = ap.parse_args()

    world, rank, local = dist_env()
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dist = init_dist(world)
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # 1:1 on a full node; ranks share a GPU only in a rehearsal
    torch.cuda.set_device(gpu)
    if pcs.lib().pcs_set_device(gpu) != 0:
        raise pcs.PcsError("pcs_set_device", -2, pcs.lib().pcs_last_error().decode())
    dev = f"cuda:{gpu}"
    algo = pcs.XXH3_64 if args.algo == "xxh3" else pcs.XXH64

    w = Workload(args.config, algo, rank, args.pages_per_gpu, dev)
    if args.mode == "validate":  # the read path checks stamped pages (mostly valid)
        w.step("stamp")
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        w.step(args.mode)
    torch.cuda.synchronize()

    # Two HIP events on the launch stream (torch's current stream) bracket the
    # K steps: the average launch duration is their span / K.  Events around
    # every launch would add a timestamp packet between consecutive kernels,
    # ~7 us per step (tools/lab/tail_lab.hip, profiles/r01/tail_lab.txt); the
    # bracketed average includes the dependent-kernel boundary (~2 us), so it
    # is an upper bound on the kernel time rocprofv3 reports.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        w.step(args.mode)
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(dist)
    elapsed = max_over_ranks(dist, t1 - t0)
    avg_launch = ev0.elapsed_time(ev1) / 1e3 / args.steps
    total_bytes = sum_over_ranks(dist, float(w.bytes)) * args.steps
    value = total_bytes / elapsed / GIB

    if args.mode != "digest":  # leave self.out holding this batch's digests for the parity leg
        w.step("digest")
        torch.cuda.synchronize()
    ceiling = w.read_ceiling(max(3, args.steps // 5))
    cpu, parity, allcores = (None, None, None)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, parity = cpu_baseline(w, args.cpu_seconds)
        if cpu is not None:
            cpu["cpu"] = cpu_model()
        if args.all_cores:
            allcores = cpu_all_cores(w, min(args.cpu_seconds, 5.0))
    drill = w.corruption_drill() if rank == 0 else None
    hostinc = host_inclusive(w) if args.host_inclusive and rank == 0 else None

    if rank == 0:
        achieved = w.algorithmic_bytes(args.mode) / avg_launch / 1e9
        traffic = committed_traffic(args.config, algo) if args.mode == "digest" else None
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: splitmix64 page words generated on device (pcs_gen_pages_dev)",
            "config": {
                "workload": w.desc,
                "page_size": w.P if w.P is not None else "4/8/16 KiB mixed",
                "pages_per_gpu": w.n,
                "bytes_per_gpu": w.bytes,
                "algo": "xxh3_64" if algo == 0 else "xxh64",
                "mode": f"{args.mode} ({'pcs_pages' if w.P else 'pcs_desc'}_{args.mode}_dev)",
                "parallelism": f"page shards x{world}, no collective",
            },
            # whole-job rate against the aggregate HBM peak of all ranks (north_star: "fraction of
            # the aggregate HBM-read roofline"); roofline below is rank 0's dominant kernel
            "per_gpu_GiBps": round(value / world, 2),
            "aggregate_roofline": {"GBps": round(value * GIB / 1e9, 1), "peak_GBps": HBM_PEAK_GBPS * world,
                                   "frac": round(value * GIB / 1e9 / (HBM_PEAK_GBPS * world), 4)},
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None,
                "algorithmic_bytes_per_launch": w.algorithmic_bytes(args.mode),
                "avg_launch_ms": round(avg_launch * 1e3, 4),
                "launch_timing": f"HIP events bracketing the {args.steps} timed steps on the launch stream",
            },
            "read_ceiling_GBps": round(ceiling, 1) if ceiling else None,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        line["corruption_drill"] = drill
        if allcores is not None:
            line["cpu_all_cores"] = allcores
        if hostinc is not None:
            line["host_inclusive"] = hostinc
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
