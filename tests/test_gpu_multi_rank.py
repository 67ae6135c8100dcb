"""The N>1 path on a GPU: two ranks, one process each, sharing cuda:0 of the
one-GPU box (bench.py maps rank -> device modulo the device count; on a full
node the map is 1:1).

- Each rank hashes its own page shard with the HIP kernel, checks it against
  the oracle, and the digests gathered over gloo equal the single-process
  oracle result: sharding by pcs_shard_range loses and duplicates nothing.
- bench.py launched the way the driver launches it (torch.distributed.run,
  127.0.0.1 rendezvous) prints one weak-scaling line from rank 0.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_PAGES, P, SEED = 3001, 4096, 0x5EED0005


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank: int, world: int, port: int, out_dir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import eloqstore_amd as pcs
    import oracle

    torch.cuda.set_device(0)
    b, e = pcs.shard_range(N_PAGES, world, rank)
    pages = torch.empty((e - b) * P, dtype=torch.uint8, device="cuda:0")
    pcs.gen_pages(pages, P, e - b, SEED, b)  # global page indices b..e-1
    dig = pcs.pages_digest(pages, P, e - b).cpu()
    own_ok = bool(np.array_equal(dig.numpy().view(np.uint64), oracle.pages_digest(pages.cpu().numpy(), P)))
    sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([e - b]))
    maxn = int(max(s.item() for s in sizes))
    buf = torch.zeros(maxn, dtype=torch.int64)
    buf[: e - b] = dig
    parts = [torch.zeros(maxn, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(parts, buf)
    oks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(oks, torch.tensor([int(own_ok)]))
    if rank == 0:
        gathered = torch.cat([parts[r][: int(sizes[r].item())] for r in range(world)])
        np.save(os.path.join(out_dir, "gathered.npy"), gathered.numpy())
        with open(os.path.join(out_dir, "oks.txt"), "w") as f:
            f.write(" ".join(str(int(o.item())) for o in oks))
    dist.destroy_process_group()


def test_two_ranks_gpu_shards_match_oracle(tmp_path):
    world = 2
    mp.spawn(worker, args=(world, free_port(), str(tmp_path)), nprocs=world, join=True)
    import oracle
    from workload import fill_pages

    assert open(tmp_path / "oks.txt").read().split() == ["1"] * world
    gathered = np.load(tmp_path / "gathered.npy").view(np.uint64)
    single = oracle.pages_digest(fill_pages(SEED, 0, N_PAGES, P).reshape(-1), P)
    assert np.array_equal(gathered, single)


def test_bench_two_ranks_torchrun():
    """The driver's scaling launch, rehearsed with 2 ranks on the box's one GPU:
    with no --config, N>1 defaults to BASELINE config 5 (8 M x 4 KiB pages =
    32 GiB per rank, generated in place); rank 0 prints one line with per-rank
    wall/kernel-event times and the concurrent rate against its solo rate."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           "bench.py", "--gpus", "2", "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and r.stdout.strip().splitlines() == lines, r.stdout[-3000:]  # rank 0 only, nothing else
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["steps"] == 3
    assert line["config"]["workload"].startswith("config5")
    assert line["config"]["pages_per_gpu"] == 1 << 23 and line["config"]["bytes_per_gpu"] == 32 << 30
    assert line["value"] > 0 and line["aggregate_roofline"]["peak_GBps"] == 2 * 8000.0
    assert line["corruption_drill"]["pass"] and line["parity"]["mismatches"] == 0
    # parity and the drill on every rank, over its own shard
    assert line["checks_all_ranks_pass"] is True
    assert [p["rank"] for p in line["parity_per_rank"]] == [0, 1]
    assert [d["rank"] for d in line["drill_per_rank"]] == [0, 1]
    for p in line["parity_per_rank"]:
        assert p["mismatches"] == 0 and p["content_mismatches"] == 0 and p["pages"] > 2000
    assert [p["global_pages"] for p in line["parity_per_rank"]] == [[0, 1 << 23], [1 << 23, 2 << 23]]
    assert all(d["pass"] and d["pages"] == 1 << 23 for d in line["drill_per_rank"])
    sd = line["scaling_detail"]
    assert [p["rank"] for p in sd["per_rank"]] == [0, 1]
    assert all(p["kernel_event_ms_per_step"] > 0 and p["wall_s"] > 0 for p in sd["per_rank"])
    assert sd["concurrent_over_solo"] > 0 and sd["solo_rank0_GiBps"] > 0 and sd["shared_gpus"]
    assert "sweep" not in line  # the N=1 sweep
    # the north star's 16 KiB and 64 KiB batches at N > 1, full sizes per rank
    sm = line["sweep_multi"]
    assert [e["key"] for e in sm] == ["config7_xxh3", "config4_xxh3"]
    for e in sm:
        assert "error" not in e, e
        assert e["checks_all_ranks_pass"] and [p["rank"] for p in e["parity_per_rank"]] == [0, 1]
        assert e["value"] > 0 and e["aggregate_roofline"]["peak_GBps"] == 2 * 8000.0 and 0 < e["rank0_frac"] < 1
        n = e["pages_per_gpu"]
        assert [p["global_pages"] for p in e["parity_per_rank"]] == [[0, n], [n, 2 * n]]
    assert [e["bytes_per_gpu"] for e in sm] == [4 << 30, 16 << 30]


def test_bench_four_ranks_torchrun():
    """Four ranks on the box's one GPU (1 M pages per rank, config 5's seed and
    global page indices): every rank's parity and drill come back in rank 0's
    line, each over its own global range."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           "bench.py", "--gpus", "4", "--steps", "3", "--warmup", "1", "--pages-per-gpu", str(1 << 20),
           "--sweep-steps", "3", "--sweep-warmup", "1", "--sweep-scale", "16"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and r.stdout.strip().splitlines() == lines, r.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 4 and line["checks_all_ranks_pass"] is True
    n = 1 << 20
    assert [p["global_pages"] for p in line["parity_per_rank"]] == [[r * n, (r + 1) * n] for r in range(4)]
    assert all(p["mismatches"] == 0 and p["content_mismatches"] == 0 for p in line["parity_per_rank"])
    assert [d["rank"] for d in line["drill_per_rank"]] == [0, 1, 2, 3] and all(d["pass"] for d in line["drill_per_rank"])
    assert [e["key"] for e in line["sweep_multi"]] == ["config7_xxh3", "config4_xxh3"]
    assert all(e["checks_all_ranks_pass"] and len(e["drill_per_rank"]) == 4 for e in line["sweep_multi"])
