#!/usr/bin/env python3
"""bench.py — device-resident batched page checksum throughput on MI355X.

Metric (BASELINE.json): GiB/s of device-resident batched page XXH3-64 over
4 KiB pages on 1/2/4/8 MI355X.  A "step" is one pass of the hot path
(pcs_pages_digest_dev -> the XXH3 page kernel) over one batch of synthetic
pages already resident in HBM; value = page bytes hashed by ALL ranks per
second (GiB/s, 2^30), per-GPU work fixed (weak scaling: every rank owns its
own disjoint page range, no collective on the data path).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1|2|3|4|5|6|7]

Workload: N=1 defaults to BASELINE config 2 (1,048,576 x 4 KiB pages, 4 GiB);
N>1 (torch.distributed.run, one process per GPU) defaults to BASELINE config 5
(8 M x 4 KiB pages = 32 GiB per GPU, 64 M pages over 8 GPUs); gloo is the
control plane (barrier + max over ranks of the timed region).  Configs 6/7 are
the north star's 8/16 KiB page-size sweep (4 GiB per GPU).  --config 1 runs
only the CPU reference over the 1 GiB file (BASELINE configs[0]).

Also reported, on the same line:
  roofline      dominant kernel's algorithmic bytes per launch / average launch
                time (HIP events on the launch stream) vs 8 TB/s HBM peak;
                traffic = PMC-measured HBM bytes per launch: at the default
                config, two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE)
                over the headline kernel in this run (traffic_live); else, or
                if those fail, the committed summary under profiles/.
  ceiling       the measured streaming-read ceiling: pcs_stream_read_dev
                (the headline kernel's structure without the hash, at its
                measured-best occupancy) and the hash kernel alternated under
                one protocol; stream_read_GBps, and roofline.frac_of_ceiling =
                achieved / that ceiling.
  cold          the caller's exact protocol (W warmup + K timed steps) run at
                process start, before the 1.5 s settle the headline uses.
  host_inclusive (N = 1, default) pages starting in host memory, 1 GiB: pinned
                hipMemcpyAsync H2D -> kernel -> D2H, gather, and a registered
                zero-copy pool; GiB/s, fraction of PCIe Gen5 x16, digest parity
                per leg, with cpu_ref_inmem_all_cores beside them.
  cpu_baseline  BASELINE config 1: the reference's own xxHash (oracle/_ref) on
                ONE host thread, reading every page of a 1 GiB file of 4 KiB
                pages and validating it like page_checksum_tool / page.cpp:25-31;
                cpu_all_cores: the same over all usable host cores;
                cpu_ref_inmem: the reference's xxhash.c over the same pages
                already in memory, one thread (no pread per page);
                cpu_ref_inmem_all_cores: the same on every usable core (the
                node rate for host-resident pages); cpu_port:
                the repo's C restatement likewise; cli_scan: this repo's GPU
                CLI (--scan) over the same file.
  parity        sampled GPU digests (every 4096th page, first/last 64) against
                the reference xxHash on the host, and the sampled page bodies
                against the generator at their global page indices; with the
                corruption drill, run on EVERY rank over its own shard
                (parity_per_rank / drill_per_rank at N>1); the process exits
                3 after printing the line if any rank fails either.
  sweep         (N=1) every other BASELINE config and mode, one entry each:
                config 3 (XXH3 and XXH64), config 4, config 5, config 7 (16 KiB),
                config 2 validate (read path) and stamp (write path), each with
                its avg launch time, roofline frac, parity sample and
                corruption drill.
  sweep_multi   (N>1) the north star's 16 KiB (config 7 sizes) and 64 KiB
                (config 4) page batches on every rank, weak scaling like the
                headline: aggregate and per-GPU GiB/s, the aggregate roofline,
                rank 0's launch time and frac, parity and drill per rank.
  scaling_detail (N>1) per-rank wall and kernel-event times, and
                concurrent_over_solo = per-GPU rate / rank 0's rate on the same
                shard run alone (an interference check; scaling efficiency is
                the driver's, from the per-N values).
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
    """gloo for the barrier and the max/sum over ranks (no data-path
    collective).  gloo's connection messages ("[Gloo] Rank r is connected to
    ...") are written to stdout by the C++ library; they are moved to stderr
    here so that stdout carries only rank 0's JSON line."""
    if world > 1:
        import torch.distributed as dist
        sys.stdout.flush()
        saved = os.dup(1)
        try:
            os.dup2(2, 1)
            dist.init_process_group("gloo")
            dist.barrier()  # every rank connected before stdout is restored
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
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
            return self._desc_drill(every)
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

    def _desc_drill(self, every: int):
        pcs.desc_stamp(self.pages, self.d_off, self.d_len, self.n, self.algo)
        pcs.desc_validate(self.pages, self.d_off, self.d_len, self.n, self.algo, ok=self.ok, first_bad=self.fb)
        clean = int(self.ok.sum().item())
        idx = self.d_off[::every] + 10
        self.pages[idx] ^= 0xFF
        pcs.desc_validate(self.pages, self.d_off, self.d_len, self.n, self.algo, ok=self.ok, first_bad=self.fb)
        flipped = int(idx.numel())
        detected = int((self.ok == 0).sum().item())
        first = int(self.fb.item())
        self.pages[idx] ^= 0xFF  # restore
        return {"pages": self.n, "valid_after_stamp": clean, "flipped": flipped, "detected": detected,
                "first_bad": first, "pass": clean == self.n and detected == flipped and first == 0}

    def free(self):
        for k in ("pages", "out", "ok", "fb", "d_off", "d_len"):
            if hasattr(self, k):
                delattr(self, k)

    def algorithmic_bytes(self, mode: str = "digest") -> int:
        # every page byte read once (the 8-byte header shares the first line) + the result written:
        # 8 B digest (digest), 1 B verdict (validate), 8 B into the page (stamp)
        return self.bytes + (1 if mode == "validate" else 8) * self.n

    def ceiling_ab(self, rounds: int = 7, per: int = 20, settle_ms: float = 200.0):
        """The streaming-read ceiling against the hash kernel
        under ONE protocol: pcs_stream_read_dev (k_stream_read: the headline
        kernel's structure and loads, no hash) and the digest step alternate
        in `rounds` rounds of `per` launches each, every round bracketed by
        HIP events on the launch stream, after `settle_ms` of both; medians.
        Both move the same bytes (every page byte read, 8 B per 4 KiB page
        written), so their GB/s are directly comparable and frac_of_ceiling
        = hash / ceiling.  Round 5 timed the reader alone for 3 launches
        right after host-side work (the part idling), so it read ~4 % below
        the hash kernel it was meant to bound."""
        import statistics
        scratch = torch.empty((self.bytes + 4095) // 4096, dtype=torch.int64, device=self.dev)

        def read():
            pcs.stream_read(self.pages, self.bytes, scratch)

        def hash_():
            self.step("digest")

        t_end = time.perf_counter() + settle_ms / 1e3
        while time.perf_counter() < t_end:
            for _ in range(4):
                read()
                hash_()
            torch.cuda.synchronize()
        times = {"read": [], "hash": []}
        for r in range(rounds):
            order = (("read", read), ("hash", hash_)) if r % 2 == 0 else (("hash", hash_), ("read", read))
            for name, fn in order:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
                for _ in range(per):
                    fn()
                ev1.record()
                torch.cuda.synchronize()
                times[name].append(ev0.elapsed_time(ev1) / 1e3 / per)
        moved = self.bytes + 8 * ((self.bytes + 4095) // 4096)
        read_gbps = moved / statistics.median(times["read"]) / 1e9
        hash_gbps = self.algorithmic_bytes("digest") / statistics.median(times["hash"]) / 1e9
        return {"stream_read_GBps": round(read_gbps, 1), "hash_GBps": round(hash_gbps, 1),
                "frac_of_ceiling": round(hash_gbps / read_gbps, 4),
                "protocol": f"{rounds} alternating rounds of {per} launches each (HIP events per round), "
                            f"after {settle_ms:.0f} ms of both; medians; the same bytes moved by both"}

    def sample_pages_host(self, max_bytes: int):
        """(host uint8 array, page size, gpu digests) for a leading sample of the batch."""
        if self.P is not None:
            k = max(1, min(self.n, max_bytes // self.P))
            host = self.pages[: k * self.P].cpu().numpy()
            return host, self.P, self.out[:k].cpu().numpy().view(np.uint64)
        return None


def parity_sample(w: Workload, mode: str = "digest"):
    """Sampled parity against the reference xxHash on the host:
    pages 0..63, every 4096th page and the last 64.  digest/validate: the
    GPU's digests of those pages (w.out, written by a digest step); stamp: the
    8-byte headers the stamp wrote into the pages."""
    import oracle  # checker only

    idx = np.unique(np.concatenate([np.arange(min(64, w.n)), np.arange(0, w.n, 4096),
                                    np.arange(max(0, w.n - 64), w.n)])).astype(np.int64)
    tidx = torch.from_numpy(idx).to(w.dev)
    if w.P is not None:
        host = w.pages.view(w.n, w.P).index_select(0, tidx).cpu().numpy()
        fn = oracle.ref_pages_digest if oracle.ref_lib() is not None else oracle.pages_digest
        want = fn(host.reshape(-1), w.P, w.algo)
    else:
        offs, lens = w.offs[idx], w.lens[idx]
        parts = [w.pages[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
        host = torch.cat(parts).cpu().numpy()
        new_off = np.zeros(len(idx), dtype=np.uint64)
        np.cumsum(lens[:-1], dtype=np.uint64, out=new_off[1:])
        want = oracle.ref_desc_digest(host, new_off, lens, w.algo)
        if want is None:
            want = oracle.desc_digest(host, new_off, lens, w.algo)
    if mode == "stamp":
        if w.P is not None:
            got = host[:, :8].copy().view(np.uint64).ravel()
        else:
            got = np.array([host[int(o):int(o) + 8].view(np.uint64)[0] for o in new_off], dtype=np.uint64)
    else:
        got = w.out.index_select(0, tidx).cpu().numpy().view(np.uint64)
    checker = "reference external/xxhash.c (oracle/_ref)" if oracle.ref_lib() is not None else "oracle C restatement"
    res = {"pages": int(len(idx)), "mismatches": int((want != got).sum()), "checker": checker,
           "what": "headers written by the stamp" if mode == "stamp" else "GPU digests"}
    if w.P is not None:
        # the sampled pages' bodies are the generator's pages at this rank's
        # GLOBAL indices (first + i): the shard covers its own range
        from workload import fill_pages_at
        gen = fill_pages_at(w.seed, w.first + idx, w.P)
        res["content_mismatches"] = int((gen[:, 8:] != host[:, 8:]).any(axis=1).sum())
        res["global_pages"] = [int(w.first), int(w.first + w.n)]
    return res


def gather_checks(dist, world: int, rank: int, parity, drill):
    """Every rank's parity sample and drill, gathered on every rank (gloo):
    ([{"rank", "parity", "corruption_drill"}, ...] in rank order, all pass)."""
    checks = [{"rank": rank, "parity": parity, "corruption_drill": drill}]
    if dist is not None:
        checks = [None] * world
        dist.all_gather_object(checks, {"rank": rank, "parity": parity, "corruption_drill": drill})
    return checks, all(parity_ok(c["parity"], c["corruption_drill"]) for c in checks)


def parity_ok(par, drill) -> bool:
    return bool(par and drill and par.get("mismatches") == 0 and par.get("content_mismatches", 0) == 0
                and drill.get("pass"))


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def usable_cores() -> int:
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)


def cpu_threads() -> int:
    """One thread per core this process may actually use: the affinity
    mask, capped by a cgroup CPU quota when one is set (a GPU box shows every
    core of the host but grants a share of them)."""
    quota = cgroup_cpu_quota()
    return usable_cores() if quota is None else max(1, min(usable_cores(), int(quota)))


def cgroup_cpu_quota():
    """CPUs this process may use per the cgroup v2 quota (None if unlimited)."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


CONFIG1_SEED = 0x5EED0001
CONFIG1_PAGES = 1 << 18  # 1 GiB of 4 KiB pages (BASELINE configs[0])


CONFIG1_DIR = os.path.join(ROOT, ".bench_tmp")  # git- and gpurun-ignored; not gpurun_out/ (1 GiB)


def config1_workdir(need_bytes: int, workdir: str | None = None) -> str:
    """A directory with room for the config-1 file: the working tree first
    (the GPU box's scratch copy), then the system temp dir.  Raises with the
    free space of each candidate if none has `need_bytes` plus 256 MiB."""
    import shutil
    import tempfile

    cands = [workdir] if workdir else [CONFIG1_DIR, tempfile.gettempdir()]
    seen = []
    for c in cands:
        try:
            os.makedirs(c, exist_ok=True)
            free = shutil.disk_usage(c).free
        except OSError as e:
            seen.append(f"{c}: {e}")
            continue
        if free >= need_bytes + (256 << 20):
            return c
        seen.append(f"{c}: {free >> 20} MiB free")
    raise RuntimeError(f"no room for the {need_bytes >> 20} MiB config-1 file ({'; '.join(seen)})")


def config1(target_s: float, all_cores_s: float | None, workdir: str | None = None):
    """BASELINE config 1: the reference checksum over a 1 GiB file of 4 KiB
    pages on ONE host thread (tools/page_checksum_tool.cpp reads a page from
    the file and calls ValidateChecksum, page.cpp:25-31).

    The file (splitmix64 pages, seed 0x5EED0001, stamped) is written by this
    repo's CLI (`page_checksum_tool --gen`, GPU-stamped).  The timed loop is
    oracle/_ref's ref_scan_file: pread one page, XXH3_64bits from the
    reference's own external/xxhash.c, compare with the stored header; whole
    passes over the file are repeated for ~target_s (page cache warm).  Every
    page must validate: the reference agreeing with the GPU's stamps is a
    parity check of its own.  Also: the same loop on all usable host cores
    (disjoint page ranges, one thread each), and the repo CLI's --scan."""
    import shutil
    import subprocess
    import tempfile
    import threading

    import oracle  # baseline infrastructure only

    if os.environ.get("PCS_BENCH_FAIL_CONFIG1"):  # tests: a failing leg must not lose the line
        raise RuntimeError("PCS_BENCH_FAIL_CONFIG1 set")
    P, n = 4096, CONFIG1_PAGES
    d = tempfile.mkdtemp(prefix="pcs_config1_", dir=config1_workdir(n * P, workdir))
    path = os.path.join(d, "config1.data")
    try:
        r = subprocess.run([pcs.TOOL_PATH, "--gen", path, str(n), str(P), hex(CONFIG1_SEED)],
                           capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise RuntimeError(f"page_checksum_tool --gen failed: {r.stderr.strip()}")
        ref = oracle.ref_lib() is not None and hasattr(oracle.ref_lib(), "ref_scan_file")
        if not ref:
            return None
        oracle.ref_scan_file(path, P, 0, n)  # warm the page cache
        passes, bad, t0 = 0, 0, time.perf_counter()
        while True:
            got, b = oracle.ref_scan_file(path, P, 0, n)
            assert got == n * P
            bad += b
            passes += 1
            if time.perf_counter() - t0 >= target_s:
                break
        dt = time.perf_counter() - t0
        one = {"value": round(passes * n * P / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "reference",
               "sample": f"config 1: {passes} passes over a 1 GiB file of {n} x 4 KiB pages (seed 0x5EED0001, "
                         f"stamped by page_checksum_tool --gen), pread + reference external/xxhash.c v0.8.3 "
                         f"XXH3_64bits (gcc -O2, SSE2) + compare per page on one thread, page cache warm",
               "pages_failed": bad, "cpu": cpu_model()}
        allc = None
        if all_cores_s:
            # one thread per core this process may actually use: the affinity
            # mask, capped by a cgroup CPU quota when one is set (a GPU box
            # shows every core of the host but grants a share of them)
            T = cpu_threads()
            done = [0] * T
            fails = [0] * T
            stop = time.perf_counter() + all_cores_s

            def run(i):
                b0, e0 = i * n // T, (i + 1) * n // T
                while time.perf_counter() < stop:
                    got, b = oracle.ref_scan_file(path, P, b0, e0 - b0)
                    done[i] += got
                    fails[i] += b

            t0 = time.perf_counter()
            th = [threading.Thread(target=run, args=(i,)) for i in range(T)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = time.perf_counter() - t0
            allc = {"value": round(sum(done) / dt / GIB, 2), "unit": "GiB/s", "cores": T, "kind": "reference",
                    "nproc": os.cpu_count(), "usable_cores": usable_cores(), "cgroup_cpu_quota": cgroup_cpu_quota(),
                    "cpu": cpu_model(), "pages_failed": sum(fails),
                    "sample": f"config 1 file, {T} threads (one per usable core: affinity mask capped by the cgroup "
                              f"CPU quota) on disjoint page ranges, "
                              f"~{all_cores_s:.0f} s"}
        # the same pages through this repo's CPU restatement
        # (oracle/xxh_oracle.c), in memory, one thread: the port's own rate
        # and a parity check of it against the stamped headers
        data = np.fromfile(path, dtype=np.uint8)
        want = data.reshape(n, P)[:, :8].copy().view(np.uint64).ravel()
        reps, t0 = 0, time.perf_counter()
        while True:
            got = oracle.pages_digest(data, P, 0)
            reps += 1
            if time.perf_counter() - t0 >= min(3.0, target_s):
                break
        dt = time.perf_counter() - t0
        port = {"value": round(reps * n * P / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"config 1 file in memory, {reps} passes of oracle/xxh_oracle.c (the repo's C restatement, "
                          f"gcc -O2) per page, one thread",
                "pages_failed": int((got != want).sum())}
        # The reference's own xxhash.c over the same pages already in memory
        # (no pread per page): the in-memory anchor beside the pread-bound
        # cpu_baseline, one thread
        reps, t0 = 0, time.perf_counter()
        while True:
            got = oracle.ref_pages_digest(data, P, 0)
            reps += 1
            if time.perf_counter() - t0 >= min(5.0, target_s):
                break
        dt = time.perf_counter() - t0
        inmem = {"value": round(reps * n * P / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "reference",
                 "sample": f"config 1 file in memory (one 1 GiB buffer), {reps} passes of the reference's "
                           f"external/xxhash.c v0.8.3 XXH3_64bits over [8, 4096) of every page (gcc -O2, SSE2, "
                           f"oracle/_ref), one thread",
                 "pages_failed": int((got != want).sum())}
        # The same in-memory pages on every usable core: the
        # reference's ValidateChecksum loop over pages already in the page
        # pool (async_io_manager.cpp:353-366 after ReadPages), one thread per
        # core on disjoint page ranges.  This, not the pread-bound
        # cpu_all_cores, is the node rate a host-resident GPU path competes
        # with.
        inmem_all = None
        if all_cores_s:
            T = cpu_threads()
            done = [0] * T
            fails = [0] * T
            stop = time.perf_counter() + all_cores_s

            def run_mem(i):
                b0, e0 = i * n // T, (i + 1) * n // T
                part, hdr = data[b0 * P:e0 * P], want[b0:e0]
                while time.perf_counter() < stop:
                    got = oracle.ref_pages_digest(part, P, 0)  # ctypes: the GIL is released in the call
                    done[i] += (e0 - b0) * P
                    fails[i] += int((got != hdr).sum())

            t0 = time.perf_counter()
            th = [threading.Thread(target=run_mem, args=(i,)) for i in range(T)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            dt = time.perf_counter() - t0
            inmem_all = {"value": round(sum(done) / dt / GIB, 2), "unit": "GiB/s", "cores": T, "kind": "reference",
                         "usable_cores": usable_cores(), "cgroup_cpu_quota": cgroup_cpu_quota(), "cpu": cpu_model(),
                         "pages_failed": sum(fails),
                         "sample": f"config 1 file in memory (one 1 GiB buffer), {T} threads (one per usable core) "
                                   f"on disjoint page ranges, each running the reference's external/xxhash.c "
                                   f"XXH3_64bits over [8, 4096) of its pages and comparing the header, "
                                   f"~{all_cores_s:.0f} s"}
        del data
        r = subprocess.run([pcs.TOOL_PATH, "--scan", path, str(P)], capture_output=True, text=True, timeout=300)
        scan = {"rc": r.returncode, "line": r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr.strip()}
        return {"cpu_baseline": one, "cpu_all_cores": allc, "cpu_port": port, "cpu_ref_inmem": inmem,
                "cpu_ref_inmem_all_cores": inmem_all, "cli_scan": scan}
    finally:
        shutil.rmtree(d, ignore_errors=True)


PCIE_GEN5_X16_GBPS = 63.0  # PCIe Gen5 x16 per direction, after 128b/130b encoding (≈ 63 GB/s)


def host_inclusive(w: Workload, max_pages: int = 1 << 18):
    """Pages starting in host memory (SURVEY §8d "host-inclusive"; north_star:
    "the rate including pinned hipMemcpyAsync to and from the GPU"), 1 GiB of
    the headline's pages, each leg through pcs_pages_digest_host:
      direct_pinned        one contiguous pinned run: pinned hipMemcpyAsync
                           H2D -> kernel -> D2H of the digests (32 MiB chunks
                           over three streams)
      gather_pageable      pageable pages gathered into pinned staging first
      gather_scattered     pool pages in random order, unregistered: gather
      zero_copy_scattered  the same pages in a registered pool: one launch
                           reading them in place over PCIe (the reference
                           consumer's shape: ReadPages validating host pool
                           pages, async_io_manager.cpp:353-366)
    Each leg's digests are compared with the device-resident run's
    (parity: mismatches), and its rate is given as a fraction of PCIe Gen5
    x16 (63 GB/s).  Not the headline value."""
    if w.P is None:
        return None
    k = min(w.n, max_pages)
    nbytes = k * w.P
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pinned.copy_(w.pages[:nbytes])
    pageable = pinned.numpy().copy()
    digests = np.empty(k, dtype=np.uint64)
    dev_digests = w.out[:k].cpu().numpy().view(np.uint64)
    res = {"pages": k, "page_size": w.P, "bytes": nbytes, "pcie_peak_GBps": PCIE_GEN5_X16_GBPS, "legs": {}}

    def leg(name, ptrs, want, how):
        fn = pcs.lib().pcs_pages_digest_host
        rc = fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)  # warm (allocates staging)
        assert rc == 0, pcs.lib().pcs_last_error()
        reps, t0 = 0, time.perf_counter()
        while reps < 3 or time.perf_counter() - t0 < 2.0:
            rc = fn(ptrs.ctypes.data, w.P, k, w.algo, digests.ctypes.data)
            assert rc == 0, pcs.lib().pcs_last_error()
            reps += 1
        dt = (time.perf_counter() - t0) / reps
        res["legs"][name] = {"GiBps": round(nbytes / dt / GIB, 2), "GBps": round(nbytes / dt / 1e9, 2),
                             "frac_of_pcie": round(nbytes / dt / 1e9 / PCIE_GEN5_X16_GBPS, 4),
                             "calls": reps, "parity_mismatches": int((digests != want).sum()), "how": how}
        res[f"{name}_GiBps"] = res["legs"][name]["GiBps"]

    for name, base, how in (("direct_pinned", pinned.data_ptr(),
                             "pinned hipMemcpyAsync H2D -> XXH3 kernel -> D2H of digests"),
                            ("gather_pageable", pageable.ctypes.data,
                             "memcpy gather into pinned staging, then as direct_pinned")):
        leg(name, np.arange(k, dtype=np.uint64) * np.uint64(w.P) + np.uint64(base), dev_digests, how)
    # Scattered pool pages (a random permutation, like pages spread over
    # PagesPool chunks): unregistered -> gather; registered pool -> zero-copy
    perm = np.random.default_rng(7).permutation(k).astype(np.uint64)
    want = dev_digests[perm]
    with pcs.PagePool(k, w.P) as pool:
        pool.pages.reshape(-1)[:] = pageable
        for name, base, how in (("gather_scattered", pageable.ctypes.data,
                                 "scattered pageable pages gathered into pinned staging"),
                                ("zero_copy_scattered", pool.base,
                                 "scattered pages of a registered pool read in place by one launch")):
            leg(name, perm * np.uint64(w.P) + np.uint64(base), want, how)
        res["batch_latency_us"] = batch_latency(pool, pageable, w)
    res["parity_mismatches"] = sum(v["parity_mismatches"] for v in res["legs"].values())
    return res


def batch_latency(pool, pageable, w: Workload):
    """Median wall time of one validate call over a read-path-sized batch
    (max_read_pages_batch = 128, kv_options.h:18-19; write batches <= 256),
    scattered pages: staged (gather) vs zero-copy (registered pool), the
    async form (submit + poll spin) on the registered pool, and the sync call
    with the validate service on."""
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
                fn(ptrs.ctypes.data, w.P, nb, w.algo, ok.ctypes.data, ctypes.byref(fb))
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
        # the same sync call with the validate service on
        if w.algo == pcs.XXH3_64 and w.P % 256 == 0:
            ok = np.empty(nb, dtype=np.uint8)
            fb = ctypes.c_uint64()
            served0 = pcs.counter(pcs.COUNTER_SERVICE_BATCHES)
            ts = []
            with pcs.ValidateService(4, 1000):
                for _ in range(200):
                    t0 = time.perf_counter()
                    pcs.lib().pcs_pages_validate_host(ptrs.ctypes.data, w.P, nb, w.algo, ok.ctypes.data,
                                                      ctypes.byref(fb))
                    ts.append(time.perf_counter() - t0)
            assert ok.all() and pcs.counter(pcs.COUNTER_SERVICE_BATCHES) - served0 == 200
            row["zero_copy_service"] = round(float(np.median(ts[20:])) * 1e6, 1)
        out[str(nb)] = row
    return out


SETTLE_MS = 1500.0       # the headline, at the start of the process
SWEEP_SETTLE_MS = 200.0  # each sweep entry, later in the same process


def settle(w: Workload, mode: str, ms: float) -> int:
    """Untimed steps, in batches of 8, until at least `ms` of them have run;
    returns how many.  The timed region then starts on a part in its steady
    state.  A fresh process (or 0.1 s of idle) followed by only the driver's
    5 warmup steps (3 ms) timed 20 steps up to 2 % slow
    (profiles/r05/bench_gap_r05y.txt), and for up to ~1 s after a process
    starts -- after another process that used (and freed) a lot of HBM has
    exited, and on some fresh boxes -- steps run ~2 % slower than from then on
    (tools/lab/free_wipe_lab.py, profiles/r05/free_wipe_r05y.txt)."""
    if ms <= 0:
        return 0
    n = 0
    t_end = time.perf_counter() + ms / 1e3
    while n == 0 or time.perf_counter() < t_end:
        for _ in range(8):
            w.step(mode)
        n += 8
        torch.cuda.synchronize()
    return n


def cold_rate(dist, w: Workload, mode: str, steps: int, warmup: int) -> dict:
    """The headline protocol without the settle: `warmup` steps, then
    `steps` steps timed (host clock between barriers, HIP events on the
    launch stream), at the start of the process."""
    for _ in range(warmup):
        w.step(mode)
    torch.cuda.synchronize()
    barrier(dist)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(steps):
        w.step(mode)
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(dist)
    elapsed = max_over_ranks(dist, t1 - t0)
    value = sum_over_ranks(dist, float(w.bytes)) * steps / elapsed / GIB
    avg = ev0.elapsed_time(ev1) / 1e3 / steps
    return {"value": round(value, 2), "unit": "GiB/s", "steps": steps, "warmup": warmup,
            "frac": round(w.algorithmic_bytes(mode) / avg / 1e9 / HBM_PEAK_GBPS, 4),
            "avg_launch_ms": round(avg * 1e3, 4),
            "protocol": "the driver's warmup + timed steps at process start, no settle (rank 0's kernel for frac)"}


def timed_launches(w: Workload, mode: str, steps: int, warmup: int, rounds: int = 1) -> float:
    """Average launch time (s) of `steps` back-to-back steps, bracketed by two
    HIP events on the launch stream (torch's current stream).  With rounds >
    1 the steps run as that many bracketed rounds and the median round's
    per-step time is returned: one host-side stall inside a round (a 1.1 ms
    gap between two launches was seen in a 50-step sweep entry's trace,
    profiles/r03b_sweep.json config 7) then moves one round, not the entry.
    The garbage collector is held off while launches are timed."""
    import gc
    import statistics

    for _ in range(warmup):
        w.step(mode)
    torch.cuda.synchronize()
    per = max(1, steps // max(1, rounds))
    times = []
    gc_on = gc.isenabled()
    gc.disable()
    try:
        for _ in range(max(1, rounds)):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
            for _ in range(per):
                w.step(mode)
            ev1.record()
            torch.cuda.synchronize()
            times.append(ev0.elapsed_time(ev1) / 1e3 / per)
    finally:
        if gc_on:
            gc.enable()
    return statistics.median(times)


# (entry key, BASELINE config, algo, mode): every BASELINE config and mode the
# headline line does not cover, run by the default N=1 bench.
SWEEP = (
    ("config3_xxh3", 3, 0, "digest"),
    ("config3_xxh64", 3, 1, "digest"),
    ("config4_xxh3", 4, 0, "digest"),
    ("config5_xxh3", 5, 0, "digest"),
    ("config7_xxh3", 7, 0, "digest"),
    ("config2_xxh3_validate", 2, 0, "validate"),
    ("config2_xxh3_stamp", 2, 0, "stamp"),
)
SWEEP_ROUNDS = 5  # a sweep entry's steps run as this many bracketed rounds; the median round counts
PHASE_GAP_S = 0.1  # idle gap between phases: tools/summarize_sweep.py splits the kernel trace on it


def sweep(dev: str, steps: int, warmup: int, head: Workload | None = None, scale: int = 1,
          deadline: float | None = None, settle_ms: float = SWEEP_SETTLE_MS):
    """Each entry on a device-resident workload that stays allocated until the
    sweep ends: config 2 entries reuse the headline's batch (`head`), config 3
    XXH64 reuses config 3's arena.  Nothing is freed between entries: a
    hipFree of a large buffer (torch.cuda.empty_cache) left every other buffer
    of the process reading ~1.5 % slower until another process initialised
    the GPU (tools/lab/degrade_lab.py, profiles/r02/degrade_lab.txt).

    An entry that raises is recorded as {"key", "error"} and the sweep goes
    on; entries that would start after `deadline` (perf_counter seconds) are
    recorded as {"key", "skipped"} so the bench stays inside its wall budget."""
    out = []
    resident: dict[int, Workload] = {}
    if head is not None and head.cfg == 2 and head.n == CONFIGS[2][1] // scale:
        resident[2] = head
    for key, cfg, algo, mode in SWEEP:
        if deadline is not None and time.perf_counter() > deadline:
            out.append({"key": key, "config": cfg, "skipped": "bench wall budget spent"})
            continue
        try:
            out.append(sweep_entry(key, cfg, algo, mode, resident, dev, steps, warmup, scale, settle_ms))
        except Exception as e:  # noqa: BLE001 — recorded in the line, never loses it
            out.append({"key": key, "config": cfg, "error": f"{type(e).__name__}: {e}"[:500]})
        time.sleep(PHASE_GAP_S)
    return out


def sweep_entry(key, cfg, algo, mode, resident, dev, steps, warmup, scale, settle_ms=SWEEP_SETTLE_MS):
    """One sweep entry (see sweep())."""
    if cfg not in resident:
        resident[cfg] = Workload(cfg, algo, 0, max(1, CONFIGS[cfg][1] // scale), dev)
    w = resident[cfg]
    w.algo = algo
    if mode == "validate":
        w.step("stamp")
    torch.cuda.synchronize()
    time.sleep(PHASE_GAP_S)
    settle(w, mode, settle_ms)  # as the headline: the part leaves its idle state before the warmup
    t_wall0 = time.perf_counter()
    rounds = SWEEP_ROUNDS if steps >= 2 * SWEEP_ROUNDS else 1
    avg = timed_launches(w, mode, steps, warmup, rounds)
    t_wall = time.perf_counter() - t_wall0
    time.sleep(PHASE_GAP_S)
    alg = w.algorithmic_bytes(mode)
    if mode != "stamp":
        w.step("digest")  # w.out = this batch's digests for the parity sample
        torch.cuda.synchronize()
    par = parity_sample(w, mode)
    drill = w.corruption_drill()
    traffic = committed_traffic_key(key)
    e = {"key": key, "config": cfg, "workload": w.desc, "algo": "xxh3_64" if algo == 0 else "xxh64",
         "mode": mode, "pages": w.n, "bytes": w.bytes, "steps": steps, "warmup": warmup,
         "avg_launch_ms": round(avg * 1e3, 4), "GiBps": round(w.bytes / avg / GIB, 1),
         "achieved_GBps": round(alg / avg / 1e9, 1), "frac": round(alg / avg / 1e9 / HBM_PEAK_GBPS, 4),
         "algorithmic_bytes_per_launch": alg, "wall_s": round(t_wall, 3),
         "timing": f"median of {rounds} rounds of {max(1, steps // rounds)} steps, each bracketed by HIP events",
         "traffic": traffic[0] if traffic else None, "traffic_source": traffic[1] if traffic else None,
         "parity": par, "corruption_drill": drill}
    return e


def min_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


# N > 1: the north star's 16 KiB and 64 KiB page batches at every GPU count,
# beside the 4 KiB headline (config 5): the same weak-scaling timing
MULTI_SWEEP = (("config7_xxh3", 7), ("config4_xxh3", 4))


def multi_rank_sweep(dist, world: int, rank: int, dev: str, algo: int, steps: int, warmup: int, scale: int,
                     settle_ms: float = SWEEP_SETTLE_MS, deadline: float | None = None):
    """Each entry on every rank: its own shard of the config (global page
    indices rank * n ...), `steps` launches timed between barriers, value =
    bytes of all ranks / the max-over-ranks wall time, then parity and the
    drill on every rank.  Every rank reaches every collective: a local
    failure (build, settle, warmup, the timed launches, parity, drill) is
    recorded, never raised, and the ranks agree on success (min over ranks)
    before and after the timed section, so no rank waits on a rank that has
    failed.  Entries past the wall deadline (on any rank) are skipped."""
    out = []
    for key, cfg in MULTI_SWEEP:
        late = deadline is not None and time.perf_counter() > deadline
        if min_over_ranks(dist, 0.0 if late else 1.0) < 1.0:
            out.append({"key": key, "config": cfg, "skipped": "bench wall budget spent"})
            continue
        w, err = None, None
        try:
            w = Workload(cfg, algo, rank, max(1, CONFIGS[cfg][1] // scale), dev)
            settle(w, "digest", settle_ms)
            for _ in range(warmup):
                w.step("digest")
            torch.cuda.synchronize()
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:300]
        if min_over_ranks(dist, 0.0 if err else 1.0) < 1.0:
            out.append({"key": key, "config": cfg, "error": err or "another rank failed to build or warm its shard"})
            if w is not None:
                w.free()
            continue
        barrier(dist)
        t0 = t1 = time.perf_counter()
        avg = None
        try:
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            ev0.record()
            for _ in range(steps):
                w.step("digest")
            ev1.record()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            avg = ev0.elapsed_time(ev1) / 1e3 / steps
        except Exception as e:  # noqa: BLE001
            err = f"{type(e).__name__}: {e}"[:300]
        barrier(dist)
        if min_over_ranks(dist, 0.0 if err else 1.0) < 1.0:
            out.append({"key": key, "config": cfg, "error": err or "another rank failed in the timed section"})
            w.free()
            continue
        elapsed = max_over_ranks(dist, t1 - t0)
        total = sum_over_ranks(dist, float(w.bytes)) * steps
        par = guarded_check(parity_sample, w)
        drill = guarded_check(w.corruption_drill)
        checks, ok = gather_checks(dist, world, rank, par, drill)
        value = total / elapsed / GIB
        alg = w.algorithmic_bytes("digest")
        out.append({"key": key, "config": cfg, "workload": w.desc, "pages_per_gpu": w.n, "bytes_per_gpu": w.bytes,
                    "steps": steps, "warmup": warmup, "value": round(value, 2), "unit": "GiB/s",
                    "per_gpu_GiBps": round(value / world, 2),
                    "aggregate_roofline": {"GBps": round(value * GIB / 1e9, 1), "peak_GBps": HBM_PEAK_GBPS * world,
                                           "frac": round(value * GIB / 1e9 / (HBM_PEAK_GBPS * world), 4)},
                    "rank0_avg_launch_ms": round(avg * 1e3, 4) if rank == 0 else None,
                    "rank0_frac": round(alg / avg / 1e9 / HBM_PEAK_GBPS, 4) if rank == 0 else None,
                    "checks_all_ranks_pass": ok,
                    "parity_per_rank": [dict(c["parity"], rank=c["rank"]) for c in checks],
                    "drill_per_rank": [dict(c["corruption_drill"], rank=c["rank"]) for c in checks]})
        w.free()
        del w
        time.sleep(PHASE_GAP_S)
    return out


def committed_traffic_key(key: str):
    """HBM bytes per launch for a sweep entry from the committed summary."""
    best = None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*sweep*.json"))):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for e in d.get("entries", []):
            if e.get("key") == key and e.get("traffic_bytes_per_launch"):
                best = (e["traffic_bytes_per_launch"], os.path.relpath(path, ROOT))
    return best


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
    if cfg == 2 and algo == 0:
        best = committed_traffic_key("headline") or best
    return best


LIVE_KERNEL = "pcs::k_xxh3_fixed<4096, 0, "  # the headline's dominant kernel (config 2, XXH3 digest)


def pmc_child() -> None:
    """--pmc-child: the headline workload's kernel, 4 launches, nothing else
    timed; run under rocprofv3 --pmc by live_traffic()."""
    torch.cuda.set_device(0)
    w = Workload(2, pcs.XXH3_64, 0, None, "cuda:0")
    for _ in range(4):
        w.step("digest")
    torch.cuda.synchronize()
    print("pmc child ok", flush=True)


def live_traffic(timeout_s: int = 90):
    """roofline.traffic measured on THIS box in THIS run: rocprofv3 --pmc
    FETCH_SIZE and --pmc WRITE_SIZE in separate passes (their TCC counters do
    not fit one pass on gfx950) over a child process running the headline
    kernel (bench.py --pmc-child), corrected as MI355X_MICROARCH.md's HBM
    section prescribes for gfx950: read = FETCH_SIZE (KiB) * 1024 * 2 (it
    counts half the bytes of a wide streaming read), write = WRITE_SIZE (KiB) *
    1024; median over the kernel's dispatches.  Each pass runs under
    `timeout -s KILL` (a --pmc run that asks for more counters than the
    hardware has hangs)."""
    import csv
    import shutil
    import statistics
    import subprocess
    import tempfile

    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None
    per = {}
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="pcs_pmc_")
        try:
            cmd = ["timeout", "-s", "KILL", str(timeout_s), prof, "--pmc", counter, "-d", d, "-o", counter.lower(),
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--pmc-child"]
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s + 30, env=env, cwd=ROOT)
            if r.returncode != 0 or "pmc child ok" not in r.stdout:
                raise RuntimeError(f"rocprofv3 --pmc {counter}: rc {r.returncode}: {(r.stderr or r.stdout)[-300:]}")
            vals = []
            for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                with open(path) as f:
                    for row in csv.DictReader(f):
                        if LIVE_KERNEL in row["Kernel_Name"] and row["Counter_Name"] == counter:
                            vals.append(float(row["Counter_Value"]))
            if not vals:
                raise RuntimeError(f"rocprofv3 --pmc {counter}: no dispatch of {LIVE_KERNEL}")
            per[counter] = (statistics.median(vals), len(vals))
        finally:
            shutil.rmtree(d, ignore_errors=True)
    rd = per["FETCH_SIZE"][0] * 1024 * 2
    wr = per["WRITE_SIZE"][0] * 1024
    return {"traffic": round(rd + wr), "read_bytes": round(rd), "write_bytes": round(wr),
            "dispatches": {k: v[1] for k, v in per.items()},
            "source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --pmc-child in this run "
                      "(read = FETCH_SIZE*1024*2, write = WRITE_SIZE*1024, median over dispatches)"}


def guarded_check(fn, *a, **kw):
    """A parity sample or drill that raises becomes a failing record
    ({"error", "pass": False}) instead of an exception."""
    try:
        return fn(*a, **kw)
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc(file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}"[:300], "pass": False}


def guarded(name: str, fn, *a, **kw):
    """fn(*a, **kw), or {"error": ...} if it raises (the traceback goes to
    stderr): an optional leg never takes the headline line down with it."""
    try:
        r = fn(*a, **kw)
        return r if r is not None else {"error": f"{name}: no result (reference build absent)"}
    except Exception as e:  # noqa: BLE001
        import traceback
        traceback.print_exc(file=sys.stderr)
        return {"error": f"{name}: {type(e).__name__}: {e}"[:500]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=None, choices=[1] + sorted(CONFIGS),
                    help="default: 2 on one GPU, 5 (8M pages per GPU) when WORLD_SIZE > 1")
    ap.add_argument("--algo", choices=["xxh3", "xxh64"], default="xxh3")
    ap.add_argument("--pages-per-gpu", type=int, default=None)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["digest", "validate", "stamp"], default="digest",
                    help="digest (metric), validate (read path), stamp (write path)")
    ap.add_argument("--no-all-cores", action="store_true", help="skip the all-cores CPU reference run")
    ap.add_argument("--no-sweep", action="store_true", help="headline only (no per-config sweep)")
    ap.add_argument("--sweep-steps", type=int, default=50)
    ap.add_argument("--sweep-warmup", type=int, default=5)
    ap.add_argument("--sweep-scale", type=int, default=1,
                    help="divide every sweep workload's page count (tests only; default 1 = the BASELINE sizes)")
    ap.add_argument("--host-inclusive", action="store_true",
                    help="(default at N=1) time the host-memory paths too")
    ap.add_argument("--no-host-inclusive", action="store_true",
                    help="skip the host-memory legs (pinned H2D -> kernel -> D2H, gather, zero-copy)")
    ap.add_argument("--no-live-traffic", action="store_true",
                    help="take roofline.traffic from the committed profiles/ summary instead of two rocprofv3 "
                         "--pmc passes in this run")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--settle-ms", type=float, default=SETTLE_MS,
                    help="untimed steps for at least this long before the W warmup steps (0: none)")
    ap.add_argument("--wall-budget", type=float, default=360.0,
                    help="seconds from start after which the optional legs (config 1, host-inclusive, "
                         "sweep entries) are skipped and recorded as such; the headline line always prints")
    args = ap.parse_args()
    if args.pmc_child:
        pmc_child()
        return
    t_start = time.perf_counter()
    deadline = t_start + args.wall_budget

    world, rank, local = dist_env()
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    if args.config == 1:  # BASELINE configs[0]: CPU reference only, runs without a GPU
        if rank == 0:
            c1 = guarded("config1", config1, args.cpu_seconds,
                         None if args.no_all_cores else min(args.cpu_seconds, 5.0))
            one = c1.get("cpu_baseline") or {}
            print(json.dumps({"metric": "GiB/s page_checksum_tool-style validate over a 1 GiB file of 4 KiB pages, "
                                        "reference xxHash on one host thread",
                              "value": one.get("value"), "unit": "GiB/s", "n_gpus": 0, "higher_is_better": True,
                              "dtype": "u64", "data": "synthetic (splitmix64 pages, seed 0x5EED0001)",
                              "config": {"workload": "config1: 1 GiB file, 4 KiB pages, single host thread"},
                              **c1}), flush=True)
        return
    cfg = args.config if args.config is not None else (5 if world > 1 else 2)
    dist = init_dist(world)
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # 1:1 on a full node; ranks share a GPU only in a rehearsal
    torch.cuda.set_device(gpu)
    if pcs.lib().pcs_set_device(gpu) != 0:
        raise pcs.PcsError("pcs_set_device", -2, pcs.lib().pcs_last_error().decode())
    dev = f"cuda:{gpu}"
    algo = pcs.XXH3_64 if args.algo == "xxh3" else pcs.XXH64

    w = Workload(cfg, algo, rank, args.pages_per_gpu, dev)
    if args.mode == "validate":  # the read path checks stamped pages (mostly valid)
        w.step("stamp")
        torch.cuda.synchronize()

    # The trace's phase gap goes BEFORE the warmup, never between it and the
    # timed steps: 0.1 s of idle GPU there cost the driver's short run
    # (--steps 20 --warmup 5) 2.1 % (6,725 vs 6,872 GiB/s, medians of 10 in one
    # process) and 0.15 % at 400 steps (tools/lab/bench_gap_lab.py,
    # profiles/r05/bench_gap_r05y.txt): the part slows down while idle, and the
    # warmup exists to bring it back before the clock starts.
    time.sleep(PHASE_GAP_S)
    # The driver's own protocol first, with no settle: W
    # warmup steps, then K timed steps, on the part as the process finds it.
    cold = cold_rate(dist, w, args.mode, min(args.steps, 400), args.warmup)
    time.sleep(PHASE_GAP_S)
    settle_steps = settle(w, args.mode, args.settle_ms)
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
    import gc
    gc.disable()  # no collector pause between two timed launches
    barrier(dist)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        w.step(args.mode)
    ev1.record()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    gc.enable()
    barrier(dist)
    elapsed = max_over_ranks(dist, t1 - t0)
    avg_launch = ev0.elapsed_time(ev1) / 1e3 / args.steps
    total_bytes = sum_over_ranks(dist, float(w.bytes)) * args.steps
    value = total_bytes / elapsed / GIB
    time.sleep(PHASE_GAP_S)

    scaling = None
    if dist is not None:
        # Per-rank evidence, then rank 0 alone on its own shard (the others wait
        # at the barrier): concurrent per-GPU rate / solo rate, an interference
        # check (the driver computes scaling efficiency from the per-N lines).
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "gpu": gpu, "wall_s": round(t1 - t0, 5),
                                          "kernel_event_ms_per_step": round(avg_launch * 1e3, 4),
                                          "GiBps": round(w.bytes * args.steps / (t1 - t0) / GIB, 1)})
        solo = None
        barrier(dist)
        if rank == 0:
            torch.cuda.synchronize()
            s0 = time.perf_counter()
            for _ in range(args.steps):
                w.step(args.mode)
            torch.cuda.synchronize()
            solo = w.bytes * args.steps / (time.perf_counter() - s0) / GIB
        barrier(dist)
        if rank == 0:
            scaling = {"per_rank": per_rank, "solo_rank0_GiBps": round(solo, 1),
                       "concurrent_over_solo": round(value / world / solo, 4),
                       "concurrent_over_solo_def": "per-GPU rate of the concurrent run / rank 0's rate on the "
                                                   "same shard run alone in this job",
                       "shared_gpus": ndev < world}
        time.sleep(PHASE_GAP_S)

    if args.mode != "digest":  # leave self.out holding this batch's digests for the parity leg
        w.step("digest")
        torch.cuda.synchronize()
    # Parity and the corruption drill on EVERY rank, each over its own shard
    # (SURVEY §8d "parity in every run", §8e partitioning); rank 0's line
    # carries them all and the run fails if any rank's does.
    # Each guarded per rank: a rank whose check raises records
    # it as failed and still reaches the gather, so no rank waits forever.
    parity = guarded_check(parity_sample, w)
    ceiling = guarded("ceiling", w.ceiling_ab) if args.mode == "digest" and w.P == 4096 else None
    time.sleep(PHASE_GAP_S)
    drill = guarded_check(w.corruption_drill)
    time.sleep(PHASE_GAP_S)
    per_rank_checks, checks_ok = gather_checks(dist, world, rank, parity, drill)
    # Optional legs, each guarded: a failure is recorded under its key and the
    # headline line (roofline, parity, drill) still prints.  The sweep runs
    # before config 1: with config 1 first (its CLI processes initialise the
    # GPU beside this one), one box measured config 3 XXH3 at 0.82 instead of
    # 0.89 (gpurun_out r03a, profiles/r03a_sweep.json).  Sweep entries past
    # the wall budget are skipped, and config 1 is skipped when the time left
    # cannot hold it.
    hostinc = None
    if not args.no_host_inclusive and rank == 0 and world == 1:
        hostinc = guarded("host_inclusive", host_inclusive, w) if time.perf_counter() < deadline else \
            {"skipped": "bench wall budget spent"}
    multi_entries = None
    if world > 1 and not args.no_sweep:
        multi_entries = multi_rank_sweep(dist, world, rank, dev, algo, args.sweep_steps, args.sweep_warmup,
                                         max(1, args.sweep_scale), min(args.settle_ms, SWEEP_SETTLE_MS), deadline)
        checks_ok = checks_ok and all(e.get("checks_all_ranks_pass") for e in multi_entries if "skipped" not in e)
    sweep_entries = None
    if rank == 0 and world == 1 and not args.no_sweep:
        sweep_entries = guarded("sweep", sweep, dev, args.sweep_steps, args.sweep_warmup,
                                head=w if algo == 0 else None, scale=max(1, args.sweep_scale), deadline=deadline,
                                settle_ms=min(args.settle_ms, SWEEP_SETTLE_MS))
    c1 = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        all_s = None if args.no_all_cores else min(args.cpu_seconds, 5.0)
        need = args.cpu_seconds + 2 * (all_s or 0) + 3.0 + 30.0  # + port leg + gen/scan/warm margin
        if time.perf_counter() + need > deadline:
            c1 = {"skipped": f"bench wall budget: {deadline - time.perf_counter():.0f} s left, ~{need:.0f} s needed"}
        else:
            c1 = guarded("config1", config1, args.cpu_seconds, all_s)

    live = None
    if (rank == 0 and world == 1 and cfg == 2 and algo == pcs.XXH3_64 and args.mode == "digest"
            and args.pages_per_gpu is None and not args.no_live_traffic):
        live = guarded("live_traffic", live_traffic) if time.perf_counter() + 60 < deadline else \
            {"skipped": "bench wall budget spent"}

    if rank == 0:
        achieved = w.algorithmic_bytes(args.mode) / avg_launch / 1e9
        traffic = committed_traffic(cfg, algo) if args.mode == "digest" else None
        if live and live.get("traffic"):
            traffic = (live["traffic"], live["source"])
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle": {"ms": args.settle_ms, "steps": settle_steps},
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
                # achieved / the measured streaming-read ceiling of the same bytes (ceiling_ab)
                "frac_of_ceiling": round(achieved / ceiling["stream_read_GBps"], 4)
                if ceiling and ceiling.get("stream_read_GBps") else None,
                "traffic": traffic[0] if traffic else None,
                "traffic_source": traffic[1] if traffic else None,
                "traffic_live": live,
                "algorithmic_bytes_per_launch": w.algorithmic_bytes(args.mode),
                "avg_launch_ms": round(avg_launch * 1e3, 4),
                "launch_timing": f"HIP events bracketing the {args.steps} timed steps on the launch stream",
            },
            "stream_read_GBps": ceiling.get("stream_read_GBps") if ceiling else None,
            "ceiling": ceiling,
            "cold": cold,
            "cpu_baseline": c1.get("cpu_baseline") if c1 else None,
            "parity": parity,
        }
        line["corruption_drill"] = drill
        if world > 1:
            line["parity_per_rank"] = [dict(c["parity"], rank=c["rank"]) for c in per_rank_checks]
            line["drill_per_rank"] = [dict(c["corruption_drill"], rank=c["rank"]) for c in per_rank_checks]
        line["checks_all_ranks_pass"] = checks_ok
        if c1 is not None:
            for k in ("cpu_all_cores", "cpu_port", "cpu_ref_inmem", "cpu_ref_inmem_all_cores", "cli_scan"):
                line[k] = c1.get(k)
            for k in ("error", "skipped"):
                if k in c1:
                    line[f"config1_{k}"] = c1[k]
        line["bench_wall_s"] = round(time.perf_counter() - t_start, 1)
        if scaling is not None:
            line["scaling_detail"] = scaling
        if hostinc is not None:
            if c1 and c1.get("cpu_ref_inmem_all_cores") and not hostinc.get("error"):
                ref = c1["cpu_ref_inmem_all_cores"]
                hostinc["cpu_ref_inmem_all_cores"] = {k: ref.get(k) for k in ("value", "unit", "cores")}
            line["host_inclusive"] = hostinc
        if sweep_entries is not None:
            line["sweep"] = sweep_entries
        if multi_entries is not None:
            line["sweep_multi"] = multi_entries
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if not checks_ok:
        bad = [c["rank"] for c in per_rank_checks if not parity_ok(c["parity"], c["corruption_drill"])]
        bad_sweep = [e["key"] for e in (multi_entries or []) if "skipped" not in e and not e.get("checks_all_ranks_pass")]
        print(f"bench: parity or corruption drill failed: headline rank(s) {bad}, sweep_multi {bad_sweep}",
              file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
