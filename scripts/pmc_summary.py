"""Summarise rocprofv3 --pmc counter CSVs per kernel family (the extras' GEMM / norm / attention kernels).

    python scripts/pmc_summary.py gpurun_out/<run>/pmc_mlp1/pmc_counter_collection.csv [more csvs...]

Counters are summed per kernel name over dispatches (several passes merge by kernel name); derived metrics:
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4): a RELATIVE figure only (the two counters are kept
               in different units / per-SE instances on gfx950; compare kernels with it, not with 100 %)
  LDS conflict rate = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per LDS instruction)
  TCC hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  per-dispatch time from the dispatch timestamps.
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    """Kernel name with its template arguments, without the return type, namespaces and parameter list."""
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def main(paths):
    ctr = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(float)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                k = family(r["Kernel_Name"])
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (p, r["Dispatch_Id"])
                if key not in disp[k]:
                    disp[k].add(key)
                    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    rows = []
    for k, c in ctr.items():
        if not re.search(r"gemm|norm|attn|adam|decoder|heads|lstm|transpose|cast", k):
            continue
        busy = c.get("SQ_BUSY_CYCLES", 0.0)
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        lds = c.get("SQ_INSTS_LDS", 0.0)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        n = len(disp[k])
        rows.append((dur[k] / max(n, 1), k, n, mfma / (4 * busy) if busy else float("nan"),
                     conf / lds if lds else float("nan"), hit / (hit + miss) if hit + miss else float("nan"),
                     c.get("SQ_INSTS_VALU_MFMA_BF16", 0.0) / max(n, 1)))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'disp':>5s} {'us/disp':>8s} {'MFMA busy':>9s} {'LDSconf/inst':>12s} {'TCC hit':>8s} {'MFMA/disp':>10s}")
    for us, k, n, mb, lc, th, mf in rows:
        print(f"{k[:60]:60s} {n:5d} {us:8.1f} {mb:9.1%} {lc:12.3f} {th:8.1%} {mf:10.0f}")


if __name__ == "__main__":
    main(sys.argv[1:])
