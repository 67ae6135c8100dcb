"""Debug: XXH64 LDS kernel, partial last tiles: which pages come out wrong?"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch, eloqstore_amd as pcs, oracle
P = 4096
host_all = np.random.default_rng(65).integers(0, 256, size=(100_032 * P), dtype=np.uint8)
dev_all = torch.from_numpy(host_all).to("cuda:0")
for n in (69, 96, 100, 128 + 32, 1000, 1024 + 32, 10000, 64 * 1563, 100_000, 100_000 - 1, 100_000 + 1, 100_016, 100_032):
    for rep in range(2):
        got = pcs.pages_digest(dev_all, P, n, pcs.XXH64).cpu().numpy().view(np.uint64)
        want = oracle.pages_digest(host_all[: n * P], P, 1)
        bad = np.flatnonzero(got != want)
        print(f"n={n} rep={rep} tiles={(n + 63) // 64} bad={len(bad)} {bad[:8].tolist()}", flush=True)
for wv in (1, 2):
    pcs.set_tuning(pcs.TUNE_XXH64_WAVES, wv)
    for n in (100_000, 100_016):
        got = pcs.pages_digest(dev_all, P, n, pcs.XXH64).cpu().numpy().view(np.uint64)
        want = oracle.pages_digest(host_all[: n * P], P, 1)
        bad = np.flatnonzero(got != want)
        print(f"waves={wv} n={n} bad={len(bad)} {bad[:8].tolist()}", flush=True)
pcs.set_tuning(pcs.TUNE_XXH64_WAVES, 4)
for lay in (2, 3, 4):
    pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, lay)
    got = pcs.pages_digest(dev_all, P, 100_000, pcs.XXH64).cpu().numpy().view(np.uint64)
    want = oracle.pages_digest(host_all[: 100_000 * P], P, 1)
    bad = np.flatnonzero(got != want)
    print(f"layout={lay} n=100000 bad={len(bad)} {bad[:8].tolist()}", flush=True)
pcs.set_tuning(pcs.TUNE_XXH64_LAYOUT, 0)
