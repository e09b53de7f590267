"""Summarise rocprofv3 --pmc counter CSVs per kernel family (the extras' GEMM / norm / attention kernels).

    python scripts/pmc_summary.py gpurun_out/<run>/pmc_mlp1/pmc_counter_collection.csv [more csvs...]

Counters are summed per kernel name over dispatches (several passes merge by kernel name); derived metrics:
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4): a RELATIVE figure only (the two counters are kept
               in different units / per-SE instances on gfx950; compare kernels with it, not with 100 %)
  LDS conflict rate = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per LDS instruction)
  TCC hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  wait% = SQ_WAIT_ANY / SQ_WAVE_CYCLES, activ% = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (share of wave-cycles)
  HBM GB/s = FETCH_SIZE / WRITE_SIZE (KB per dispatch) over the dispatch time
  instruction counts per dispatch (SQ_INSTS_*: MFMA bf16, VALU, LDS, VMEM read + write, SALU)
  per-dispatch time from the dispatch timestamps.  Each CSV is one counter pass; counters are averaged per
  dispatch within their pass, then merged by kernel name.
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
    # per file (= one counter pass): counter sums, dispatch count and duration per kernel -> per-dispatch averages,
    # merged over passes (each counter comes from the pass that collected it; durations averaged over passes)
    per = defaultdict(dict)          # kernel -> counter -> per-dispatch value
    us = defaultdict(list)           # kernel -> per-dispatch us of each pass
    ndisp = defaultdict(int)
    for p in paths:
        ctr = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        dur = defaultdict(float)
        with open(p) as f:
            for r in csv.DictReader(f):
                k = family(r["Kernel_Name"])
                ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = r["Dispatch_Id"]
                if key not in disp[k]:
                    disp[k].add(key)
                    dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, c in ctr.items():
            n = max(len(disp[k]), 1)
            for name, v in c.items():
                per[k][name] = v / n
            us[k].append(dur[k] / n)
            ndisp[k] = max(ndisp[k], n)
    nan = float("nan")
    rows = []
    for k, c in per.items():
        if not re.search(r"gemm|norm|attn|adam|decoder|heads|lstm|transpose|cast|ffn", k):
            continue
        t = sum(us[k]) / len(us[k])
        busy = c.get("SQ_BUSY_CYCLES")
        mfma = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        lds = c.get("SQ_INSTS_LDS")
        conf = c.get("SQ_LDS_BANK_CONFLICT")
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        wcyc = c.get("SQ_WAVE_CYCLES")
        wait, act = c.get("SQ_WAIT_ANY"), c.get("SQ_ACTIVE_INST_ANY")
        fetch, write = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        vmem = None if c.get("SQ_INSTS_VMEM_RD") is None else c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_VMEM_WR", 0)
        rows.append(dict(
            k=k, n=ndisp[k], us=t,
            mfma_busy=mfma / (4 * busy) if busy and mfma is not None else nan,
            lds_conf=conf / lds if lds and conf is not None else nan,
            l2_hit=hit / (hit + miss) if hit is not None and miss is not None and hit + miss else nan,
            wait=wait / wcyc if wait is not None and wcyc else nan,
            active=act / wcyc if act is not None and wcyc else nan,
            mfma_i=c.get("SQ_INSTS_VALU_MFMA_BF16", nan), valu_i=c.get("SQ_INSTS_VALU", nan),
            lds_i=lds if lds is not None else nan, vmem_i=vmem if vmem is not None else nan,
            salu_i=c.get("SQ_INSTS_SALU", nan),
            rd_gbs=fetch * 1e3 / (t * 1e3) if fetch is not None else nan,   # KB / us = GB/s
            wr_gbs=write * 1e3 / (t * 1e3) if write is not None else nan))
    rows.sort(key=lambda r: -r["us"])
    hdr = (f"{'kernel':52s} {'disp':>5s} {'us/disp':>8s} {'MFMAbusy':>8s} {'wait%':>6s} {'activ%':>6s} {'LDScf/i':>7s} "
           f"{'L2hit':>6s} {'HBMrdGB/s':>9s} {'HBMwrGB/s':>9s} | per dispatch: {'MFMA':>8s} {'VALU':>9s} {'LDS':>8s} "
           f"{'VMEM':>8s} {'SALU':>8s}")
    print(hdr)
    f = lambda v, fmt: ("-" if v != v else format(v, fmt))  # noqa: E731 (nan -> '-')
    for r in rows:
        print(f"{r['k'][:52]:52s} {r['n']:5d} {r['us']:8.1f} {f(r['mfma_busy'], '8.1%'):>8s} {f(r['wait'], '6.1%'):>6s} "
              f"{f(r['active'], '6.1%'):>6s} {f(r['lds_conf'], '7.3f'):>7s} {f(r['l2_hit'], '6.1%'):>6s} "
              f"{f(r['rd_gbs'], '9.0f'):>9s} {f(r['wr_gbs'], '9.0f'):>9s} | {f(r['mfma_i'], '8.0f'):>22s} "
              f"{f(r['valu_i'], '9.0f'):>9s} {f(r['lds_i'], '8.0f'):>8s} {f(r['vmem_i'], '8.0f'):>8s} "
              f"{f(r['salu_i'], '8.0f'):>8s}")


if __name__ == "__main__":
    main(sys.argv[1:])
