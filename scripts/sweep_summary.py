"""One JSON line per sweep run: wall time, trials, trained windows summed over the trials' ``[throughput]`` lines
(train.py), aggregate windows/s over the sweep's wall clock, and any hand-off / xGMI timeout reported by a trial.

    python scripts/sweep_summary.py <sweep_dir> <k> <t0> <t1> <rc>
"""
import json
import re
import sys
from pathlib import Path


def main(d, k, t0, t1, rc):
    d = Path(d)
    wall = float(t1) - float(t0)
    wins, fit, trials, timeouts = 0, 0.0, 0, 0
    for f in sorted(d.glob("job*.out")):
        text = f.read_text(errors="replace")
        m = re.search(r"\[throughput\] train_windows=(\d+) fit_s=([\d.]+)", text)
        if m:
            trials += 1
            wins += int(m.group(1))
            fit += float(m.group(2))
        timeouts += len(re.findall(r"timed out|gave up", text, re.I))
    print(json.dumps({"metric": "sweep trial throughput (18-job thesis grid, 1 GPU)", "jobs_per_device": int(k),
                      "rc": int(rc), "trials_done": trials, "wall_s": round(wall, 2),
                      "train_windows": wins, "windows_per_s_wall": round(wins / wall, 1) if wall > 0 else None,
                      "sum_fit_s": round(fit, 2), "timeout_mentions": timeouts}))


if __name__ == "__main__":
    main(*sys.argv[1:])
