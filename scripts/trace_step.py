"""Per-step kernel breakdown from a rocprofv3 kernel trace (csv): groups one training step's dispatches (between two
optimizer launches) by (kernel, grid) and prints time per group.  python scripts/trace_step.py <kernel_trace.csv>"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adam_fused" in r["Kernel_Name"]]
step = rows[idx[-3] + 1: idx[-2] + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} kernels")
agg = collections.defaultdict(lambda: [0, 0.0])
for r in step:
    name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
    key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:8.1f} us  n={v[0]:2d}  {v[1] / v[0]:6.1f} us/call  {k}")
