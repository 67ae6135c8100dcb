#!/usr/bin/env python3
"""Summarise tools/lab/slowbox_diag.sh output: per kernel of pmc_probe2.py
(config 2 k_xxh3_fixed<4096>, config 3 k_xxh3_desc, 16 KiB k_xxh3_split,
config 7, the plain streaming read), medians over its launches, of

  in flight   TCC_EA0_RDREQ_LEVEL / TCC_BUSY   (L2 -> memory reads outstanding)
  latency     TCC_EA0_RDREQ_LEVEL / TCC_EA0_RDREQ   (cycles, Little's law)
  credit      TCC_EA0_RDREQ_DRAM_CREDIT_STALL / TCC_BUSY
  utcl1 miss  TCP_UTCL1_TRANSLATION_MISS per MiB read (EA read requests x 64 B)
  multi miss  TCP_UTCL1_STALL_MULTI_MISS per MiB
  utcl2 busy  GRBM_UTCL2_BUSY / GRBM_GUI_ACTIVE

    python tools/lab/summarize_slowbox.py gpurun_out/slowbox_TAG ...

Not part of the product."""
import csv
import glob
import os
import statistics
import sys


def by_kernel(path):
    out = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                out.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: statistics.median(v) for c, v in cs.items()} for k, cs in out.items()}


def main():
    for d in sys.argv[1:]:
        print(f"== {d}")
        mode = os.path.join(d, "mode_ab.txt")
        if os.path.exists(mode):
            for ln in open(mode):
                if ln.startswith("config"):
                    print("  " + ln.split("  rounds")[0].strip())
        k = {}
        for sub in ("tcc", "tcp", "grbm"):
            for name, cs in by_kernel(os.path.join(d, sub)).items():
                k.setdefault(name, {}).update(cs)
        for name, c in sorted(k.items()):
            if "gen" in name or "fill" in name:
                continue
            busy = c.get("TCC_BUSY_sum", 0) or 1
            rq = c.get("TCC_EA0_RDREQ_sum", 0) or 1
            lvl = c.get("TCC_EA0_RDREQ_LEVEL_sum", 0)
            mib = rq * 64 / 2**20
            print(f"  {name[:40]:40s} inflight {lvl / busy:8.0f}  lat {lvl / rq:7.0f}  "
                  f"credit {c.get('TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum', 0) / busy:6.3f}  "
                  f"utcl1miss/MiB {c.get('TCP_UTCL1_TRANSLATION_MISS_sum', 0) / mib:8.3f}  "
                  f"multimiss/MiB {c.get('TCP_UTCL1_STALL_MULTI_MISS_sum', 0) / mib:8.3f}  "
                  f"utcl2busy {c.get('GRBM_UTCL2_BUSY', 0) / (c.get('GRBM_GUI_ACTIVE', 0) or 1):6.3f}")


if __name__ == "__main__":
    main()
