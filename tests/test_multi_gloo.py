"""Multi-rank sharding on CPU (gloo, world size 2): the N>1 path of bench.py
without a GPU.

Each rank takes its page range from pcs_shard_range (the native library's
host logic), hashes its shard with the oracle (CPU stand-in for the kernel,
which the GPU tests cover), and the gathered digests must equal the
single-process result.  Also exercises bench.py's barrier / max / sum helpers
under a real process group.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_PAGES, P, SEED = 1000, 4096, 0x5EED0005


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank: int, world: int, port: int, out_dir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    import eloqstore_amd as pcs
    import oracle
    from workload import fill_pages

    b, e = pcs.shard_range(N_PAGES, world, rank)
    pages = fill_pages(SEED, b, e - b, P).reshape(-1)
    dig = oracle.pages_digest(pages, P).view(np.int64)
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([e - b]))
    maxn = int(max(s.item() for s in sizes))
    buf = torch.zeros(maxn, dtype=torch.int64)
    buf[: e - b] = torch.from_numpy(dig)
    parts = [torch.zeros(maxn, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, buf)
    gathered = torch.cat([parts[r][: int(sizes[r].item())] for r in range(world)])

    bench.barrier(dist)
    mx = bench.max_over_ranks(dist, float(rank + 1))
    sm = bench.sum_over_ranks(dist, float(e - b))
    # bench.py's per-rank parity gather: rank 1 reports a mismatch, so the
    # gathered verdict must fail on every rank and name rank 1
    par = {"pages": e - b, "mismatches": int(rank == 1), "content_mismatches": 0}
    checks, ok = bench.gather_checks(dist, world, rank, par, {"pass": True})
    if rank == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), gathered.numpy())
        with open(os.path.join(out_dir, "stats.txt"), "w") as f:
            f.write(f"{mx} {sm}\n")
        with open(os.path.join(out_dir, "checks.txt"), "w") as f:
            bad = [c["rank"] for c in checks if not bench.parity_ok(c["parity"], c["corruption_drill"])]
            f.write(f"{[c['rank'] for c in checks]} {ok} {bad}\n")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_rank_shards_match_single_process(tmp_path, world):
    mp.spawn(worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    import oracle
    from workload import fill_pages

    gathered = np.load(tmp_path / "gathered.npy").view(np.uint64)
    single = oracle.pages_digest(fill_pages(SEED, 0, N_PAGES, P).reshape(-1), P)
    assert np.array_equal(gathered, single)
    mx, sm = open(tmp_path / "stats.txt").read().split()
    assert float(mx) == world and float(sm) == N_PAGES
    assert open(tmp_path / "checks.txt").read().strip() == f"{list(range(world))} False [1]"


GLOO_STDOUT_SCRIPT = r'''
import sys
sys.path.insert(0, {root!r})
import bench
world, rank, local = bench.dist_env()
dist = bench.init_dist(world)
mx = bench.max_over_ranks(dist, float(rank))
bench.barrier(dist)
if rank == 0:
    print('{{"max_rank": %d}}' % mx, flush=True)
'''


def test_init_dist_keeps_stdout_to_the_json_line(tmp_path):
    """Under torch.distributed.run, gloo's C++ connection messages go to
    stdout by default; bench.init_dist moves them to stderr, so the driver
    reads exactly one line (rank 0's JSON) from a multi-rank bench run."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "gloo_stdout.py"
    script.write_text(GLOO_STDOUT_SCRIPT.format(root=root))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(script)],
                       capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines() == ['{"max_rank": 2}'], r.stdout


def sweep_worker(rank: int, world: int, port: int, out_dir: str):
    """bench.multi_rank_sweep under gloo with a stand-in workload (no GPU):
    rank 1 raises inside config 7's TIMED launches.  Both ranks must leave
    the sweep (no rank left waiting in a collective), record config 7 as an
    error, and still run config 4."""
    import json

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench

    class Ev:
        def record(self):
            pass

        def elapsed_time(self, other):
            return 1.0

    class FakeWorkload:
        def __init__(self, cfg, algo, rank_, n, dev):
            self.cfg, self.n, self.bytes, self.desc, self.calls = cfg, n, n * 4096, f"fake config{cfg}", 0

        def step(self, mode):
            self.calls += 1
            if self.cfg == 7 and rank == 1 and self.calls > 1:  # past the one warmup step
                raise RuntimeError("fault in the timed launches")

        def algorithmic_bytes(self, mode):
            return self.bytes

        def corruption_drill(self):
            return {"pass": True}

        def free(self):
            pass

    torch.cuda.synchronize = lambda *a: None
    torch.cuda.Event = lambda enable_timing=True: Ev()
    bench.Workload = FakeWorkload
    bench.settle = lambda w, mode, ms: 0
    bench.parity_sample = lambda w, mode="digest": {"pages": 1, "mismatches": 0}
    out = bench.multi_rank_sweep(dist, world, rank, "cpu", 0, 3, 1, 1, 0.0, None)
    late = bench.multi_rank_sweep(dist, world, rank, "cpu", 0, 3, 1, 1, 0.0, 0.0)
    with open(os.path.join(out_dir, f"sweep{rank}.json"), "w") as f:
        json.dump({"out": out, "late": late}, f)
    dist.destroy_process_group()


def test_multi_rank_sweep_survives_a_failing_rank(tmp_path):
    import json

    mp.spawn(sweep_worker, args=(2, free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        d = json.load(open(tmp_path / f"sweep{r}.json"))
        assert [e["key"] for e in d["out"]] == ["config7_xxh3", "config4_xxh3"]
        assert "error" in d["out"][0] and "checks_all_ranks_pass" not in d["out"][0]
        assert d["out"][1]["checks_all_ranks_pass"] and d["out"][1]["value"] > 0
        assert all("skipped" in e for e in d["late"])
