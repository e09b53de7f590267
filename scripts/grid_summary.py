"""Summarise a thesis-grid multirun (scripts/plans/r6_grid*.txt: ``train.py -m`` through the gpu_pool launcher) into
one JSON line per trial plus the best-by-validation trial per loss, as the thesis selects its models
(`/root/reference/tex/diplomski_rad.tex:1106-1126`; results table `:1170`).

    python scripts/grid_summary.py <sweep dir> [<sweep dir> ...] > grid.jsonl
"""
import json
import re
import sys
from pathlib import Path


def grab(pat, text, cast=float):
    m = re.search(pat, text)
    return cast(m.group(1)) if m else None


def overrides(run_dir: Path) -> dict:
    out = {}
    f = run_dir / ".hydra" / "overrides.yaml"
    if f.exists():
        for line in f.read_text().splitlines():
            line = line.strip().lstrip("-").strip().strip("'\"")
            if "=" in line:
                k, v = line.split("=", 1)
                out[k.lstrip("+~")] = v
    return out


def trials(sweep: Path):
    for job in sorted(sweep.glob("job*.out"), key=lambda p: int(re.sub(r"\D", "", p.stem) or 0)):
        num = re.sub(r"\D", "", job.stem)
        text = job.read_text(errors="replace")
        ov = overrides(sweep / num)
        rec = {"sweep": str(sweep), "job": int(num), **ov,
               "best_val_loss": grab(r"Best validation loss: ([-0-9.eE+naninf]+)", text),
               "best_epoch": grab(r"best_epoch=(\d+)", text, int),
               "epochs_run": len(re.findall(r"^\[epoch \d+\]", text, re.M)),
               "test_delta_mse": grab(r"Test ΔMSE: ([-0-9.eE+naninf]+)", text),
               "test_delta_nll": grab(r"Test ΔNLL: ([-0-9.eE+naninf]+)", text),
               "test_mae": grab(r"Test MAE: ([-0-9.eE+naninf]+)", text),
               "test_nll": grab(r"Test NLL: ([-0-9.eE+naninf]+)", text),
               "step_p50_ms": grab(r"step p50 ([0-9.]+) ms", text)}
        if rec["test_delta_mse"] is not None and rec["test_delta_nll"] is not None:
            rec["test_delta_mix"] = rec["test_delta_nll"] + 100.0 * rec["test_delta_mse"]  # mse_weight = 100
        # the mirrored solution (beta -> -beta, SURVEY / BASELINE.md "Sign basin"): its reconstruction is off by
        # ~2 alpha-beta-r_m, the test ΔMSE jumps from ~0.004 to ~1-2
        if rec["test_delta_mse"] is not None:
            rec["mirrored_basin"] = rec["test_delta_mse"] > 0.1
        yield rec


def main(dirs):
    recs = [r for d in dirs for r in trials(Path(d))]
    for r in recs:
        print(json.dumps(r))
    best = {}
    for r in recs:
        loss, v = r.get("loss"), r.get("best_val_loss")
        if loss is None or v is None or v != v:
            continue
        if loss not in best or v < best[loss]["best_val_loss"]:
            best[loss] = r
    print(json.dumps({"best_by_validation": {k: {kk: best[k].get(kk) for kk in (
        "model.hidden_size", "model.num_layers", "model.learning_rate", "seed", "best_val_loss", "best_epoch",
        "test_delta_mse", "test_delta_nll", "test_delta_mix", "mirrored_basin", "sweep", "job")} for k in best}}))


if __name__ == "__main__":
    main(sys.argv[1:])
