"""Collect the thesis-accuracy runs (scripts/gpu_thesis.sh) into one JSON line per (loss, precision)."""
import json
import re
import sys
from pathlib import Path

REF = {  # tex/diplomski_rad.tex:1170 (synthetic; x1e-5 for ΔL_MSE, decimal units, ζ = 1e5) and :1174 (OLS)
    "thesis_delta_mse_x1e5": {"mse": 2.230, "nll": 1.966, "combined": 1.877, "ols_lookback": 1.182},
    "thesis_delta_nll": {"mse": 2.238, "nll": 2.219, "combined": 2.209, "ols_lookback": 1.536},
    "thesis_delta_mix": {"mse": 4.468, "nll": 4.185, "combined": 4.086, "ols_lookback": 2.718},
    # figures at tex/diplomski_rad.tex:1193-1212 (model / OLS / model-vs-OLS)
    "thesis_corr": {"alpha": [-0.0585, 0.0981, 0.3190], "beta": [0.4024, 0.4622, 0.5023],
                    "recon": [0.9733, 0.9694, 0.9790]},
}


def grab(pat, text, cast=float):
    m = re.search(pat, text)
    return cast(m.group(1)) if m else None


def main(d):
    d = Path(d)
    for trf in sorted(d.glob("train_*.log")):
        m = re.fullmatch(r"train_(mse|nll|combined)_(high|highest)(?:_s(\d+))?\.log", trf.name)
        tef = d / trf.name.replace("train_", "test_", 1)
        if not m or not tef.exists():
            continue
        loss, p, seed = m.group(1), m.group(2), int(m.group(3) or 0)
        tr = trf.read_text()
        te = tef.read_text()
        summ = json.loads(re.search(r"\[test-summary\] (\{.*\})", te).group(1))
        rec = {"loss": loss, "matmul_precision": p, "seed": seed, "H": 32, "L": 2, "lr": 1e-3, "windows": 10000,
               "test_delta_mse": grab(r"Test ΔMSE: ([-0-9.eE+]+)", tr),
               "test_delta_nll": grab(r"Test ΔNLL: ([-0-9.eE+]+)", tr),
               "test_mae": grab(r"Test MAE: ([-0-9.eE+]+)", tr),
               "test_nll": grab(r"Test NLL: ([-0-9.eE+]+)", tr),
               "best_val_loss": grab(r"Best validation loss: ([-0-9.eE+]+)", tr),
               "best_epoch": grab(r"best_epoch=(\d+)", tr, int),
               "epochs_run": len(re.findall(r"^\[epoch \d+\]", tr, re.M)),
               **summ}
        if rec["test_delta_mse"] is not None and rec["test_delta_nll"] is not None:
            rec["test_delta_mix"] = rec["test_delta_nll"] + 100.0 * rec["test_delta_mse"]  # mse_weight = 100
        print(json.dumps(rec))
    print(json.dumps({"reference": REF, "units": "code: percent log-returns, Student-t(5) noise (SURVEY Q12/Q13); "
                      "thesis: decimal returns, Normal noise -> absolute ΔL is parity-unpinned, compare orderings "
                      "and the unit-free correlations"}))


if __name__ == "__main__":
    main(sys.argv[1])
