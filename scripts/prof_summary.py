import csv, sys
f = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof/bench_kernel_stats.csv'
rows = list(csv.DictReader(open(f)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:n]:
    print(f"{float(r['AverageNs'])/1e3:9.1f}us x{r['Calls']:>6} {float(r['Percentage']):5.1f}% {r['Name'][:100]}")
print('total kernel ms', tot / 1e6, 'kernels', sum(int(r['Calls']) for r in rows))
