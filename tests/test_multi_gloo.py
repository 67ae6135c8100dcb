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
