"""``@main`` decorator: the Hydra entry-point contract of the reference.

`train.py:70` and `test.py:147` use ``@hydra.main(version_base=None,
config_path="configs", config_name="config")``.  This decorator reproduces the
CLI (``key=value`` overrides, ``-m/--multirun``, ``--cfg job|hydra|all``,
``-cn``/``-cp``), the run/sweep directories and the launchers:

* ``basic``   – sequential, in-process (Hydra's default launcher);
* ``joblib``  – the reference's ``override hydra/launcher: joblib``
  (`configs/config.yaml:6,17-20`); ``n_jobs: 1`` runs jobs sequentially
  in-process exactly like the reference; ``n_jobs > 1`` runs them as parallel
  child processes;
* ``gpu_pool`` – MI355X addition: every trial is a child process pinned to one
  GPU through ``HIP_VISIBLE_DEVICES`` (``jobs_per_device`` trials per GPU), so
  an 18-trial sweep (`sweeps/experiment_synthetic.sh`) fills an 8-GPU node.

Failure handling of the child-process launchers: a trial that exits non-zero is re-queued up
to ``max_retries`` times with ``resume=auto`` (it continues from its own ``last.ckpt`` when one exists);
``heartbeat_timeout_s > 0`` additionally kills a trial whose heartbeat file (touched by the trainer at
every epoch boundary and every 500 steps, ``MTA_HEARTBEAT_FILE``) went stale — a hung GPU or collective —
and retries it the same way.  ``MTA_RETRY_ATTEMPT`` tells the child which attempt it is.
"""
from __future__ import annotations

import functools
import logging
import os
import subprocess
import sys
import time
from pathlib import Path
from typing import Callable, List, Optional, Sequence

import yaml

from .composer import Override, compose, expand_sweep, override_dirname, parse_override
from .nodes import DictConfig, OmegaConf

log = logging.getLogger("masters_thesis_amd.config")

_ENV_CHILD = "MTA_SWEEP_CHILD"
_ENV_RUN_DIR = "MTA_HYDRA_RUN_DIR"


def _parse_argv(argv: Sequence[str]):
    opts = {"multirun": False, "cfg": None, "config_name": None, "config_path": None, "resolve": False}
    overrides: List[str] = []
    it = iter(argv)
    for a in it:
        if a in ("-m", "--multirun"):
            opts["multirun"] = True
        elif a in ("-c", "--cfg"):
            opts["cfg"] = next(it)
        elif a.startswith("--cfg="):
            opts["cfg"] = a.split("=", 1)[1]
        elif a in ("-cn", "--config-name"):
            opts["config_name"] = next(it)
        elif a in ("-cp", "--config-path"):
            opts["config_path"] = next(it)
        elif a == "--resolve":
            opts["resolve"] = True
        elif a in ("-h", "--help"):
            opts["cfg"] = "help"
        else:
            overrides.append(a)
    return opts, overrides


def _write_hydra_dir(run_dir: Path, job_cfg: DictConfig, hydra_cfg: DictConfig, overrides: Sequence[Override]):
    sub = run_dir / str(hydra_cfg.get("output_subdir", ".hydra"))
    sub.mkdir(parents=True, exist_ok=True)
    OmegaConf.save(job_cfg, sub / "config.yaml")
    try:
        hy = OmegaConf.to_container(hydra_cfg, resolve=True)
    except Exception:  # pragma: no cover - partially resolvable hydra node
        hy = OmegaConf.to_container(hydra_cfg, resolve=False)
    with open(sub / "hydra.yaml", "w") as f:
        yaml.safe_dump({"hydra": hy}, f, sort_keys=False)
    with open(sub / "overrides.yaml", "w") as f:
        yaml.safe_dump([o.text() for o in overrides if not o.key.startswith("hydra")], f)


def _run_job(task_fn, config_dir, config_name, overrides: List[Override], job_num: int, run_dir_key: str,
             sweep_dir: Optional[Path] = None):
    job_cfg, hydra_cfg, _ = compose(config_dir, config_name, overrides)
    if sweep_dir is not None:
        hydra_cfg["job"]["num"] = job_num
    hydra_cfg["job"]["override_dirname"] = override_dirname(overrides)
    hydra_cfg["job"]["name"] = Path(sys.argv[0]).stem or "app"
    if sweep_dir is not None:
        run_dir = sweep_dir / str(hydra_cfg["sweep"]["subdir"])
        hydra_cfg["mode"] = "MULTIRUN"
    else:
        run_dir = Path(str(hydra_cfg["run"]["dir"]))
    # ranks 1..N-1 started by the trainer's own launcher (parallel/launch.py) re-run this script a moment later:
    # they share rank 0's run directory (exported below) and leave its .hydra files and job log to rank 0
    child_rank = int(os.environ.get("RANK", "0")) > 0 and os.environ.get(_ENV_RUN_DIR)
    if child_rank:
        run_dir = Path(os.environ[_ENV_RUN_DIR])
    hydra_cfg["runtime"]["output_dir"] = str(run_dir.resolve())
    os.environ[_ENV_RUN_DIR] = str(run_dir.resolve())
    if not child_rank:
        _write_hydra_dir(run_dir, job_cfg, hydra_cfg, overrides)
        _attach_job_log(run_dir / f"{hydra_cfg['job']['name']}.log")
    if hydra_cfg["job"].get("chdir", False):
        os.chdir(run_dir)
    return task_fn(job_cfg)


def _attach_job_log(path: Path) -> None:
    root = logging.getLogger()
    for h in list(root.handlers):
        if getattr(h, "_mta_job_log", False):
            root.removeHandler(h)
            h.close()
    h = logging.FileHandler(path)
    h._mta_job_log = True  # type: ignore[attr-defined]
    h.setFormatter(logging.Formatter("[%(asctime)s][%(name)s][%(levelname)s] - %(message)s"))
    root.addHandler(h)
    if root.level > logging.INFO or root.level == logging.NOTSET:
        root.setLevel(logging.INFO)


def _visible_gpu_count() -> int:
    env = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    if env:
        return len([x for x in env.split(",") if x.strip() != ""])
    try:  # device_count does not initialise HIP on this image
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


# Trials packed on one MI355X: aggregate throughput of the headline trainer rises to k = 4 (17.9 k samples/s) and
# falls beyond it (k = 5: 14.5 k, k = 8: 12.0 k; profiles/r4_pack_sweep.jsonl) -- with one hardware queue per trial,
# a fifth queue shares a compute pipe with another and the pipelined LSTM's co-resident workgroups then wait on
# each other's time slices.  jobs_per_device is capped at max_jobs_per_device (default 4) unless raised explicitly.
MAX_JOBS_PER_DEVICE = 4


def jobs_per_device(launcher) -> int:
    per = int(launcher.get("jobs_per_device", 1) or 1)
    cap = int(launcher.get("max_jobs_per_device", MAX_JOBS_PER_DEVICE) or MAX_JOBS_PER_DEVICE)
    if per > cap:
        print(f"[gpu_pool] jobs_per_device={per} capped at {cap} (measured optimum; raise max_jobs_per_device to "
              f"override)", file=sys.stderr)
    return max(1, min(per, cap))


def _launch_children(jobs: List[List[Override]], sweep_dir: Path, launcher: DictConfig, script_argv0: str,
                     base_flags: List[str]):
    """Run each job as a child process; gpu_pool pins one GPU per slot."""
    kind = launcher["_target_"]
    if kind == "gpu_pool":
        devices = launcher.get("devices")
        if devices is None:
            devices = list(range(max(_visible_gpu_count(), 1)))
        elif isinstance(devices, int):
            devices = list(range(devices))
        slots = [d for d in devices for _ in range(jobs_per_device(launcher))]
    else:
        n = int(launcher.get("n_jobs", -1) or -1)
        n = os.cpu_count() if n < 0 else n
        slots = [None] * max(1, n)
    max_retries = int(launcher.get("max_retries", 0) or 0)
    hb_timeout = float(launcher.get("heartbeat_timeout_s", 0) or 0)
    pending = [(num, ovs, 0) for num, ovs in enumerate(jobs)]
    running = {}
    results = {}
    free = list(range(len(slots)))
    while pending or running:
        while pending and free:
            slot = free.pop(0)
            num, ovs, attempt = pending.pop(0)
            env = dict(os.environ)
            env[_ENV_CHILD] = "1"
            env["MTA_RETRY_ATTEMPT"] = str(attempt)
            # parallel CPU children must not oversubscribe the cores (spinning OpenMP pools starve each other)
            env.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // len(slots))))
            hb = sweep_dir / f"job{num}.heartbeat"
            env["MTA_HEARTBEAT_FILE"] = str(hb)
            hb.write_text(str(time.time()))
            if slots[slot] is not None:
                env["HIP_VISIBLE_DEVICES"] = str(slots[slot])
                if slots.count(slots[slot]) > 1:
                    # trials sharing a GPU time-slice it: the pipelined LSTM's cross-workgroup waits poll 16x
                    # longer before giving up (bench.py --concurrent does the same; a give-up fails the trial)
                    env.setdefault("MTA_LSTM_SPIN_LIMIT", str(1 << 25))
                    env.setdefault("MTA_ADAM_SPIN_LIMIT", str(1 << 26))
                    env.setdefault("GPU_MAX_HW_QUEUES", "1")  # one hardware queue per trial
            extra = ["resume=auto"] if attempt > 0 else []
            cmd = [sys.executable, script_argv0, *base_flags, *[o.text() for o in ovs], *extra,
                   f"hydra.run.dir={sweep_dir}/{num}", f"hydra.job.num={num}"]
            log_f = open(sweep_dir / f"job{num}.out", "a" if attempt else "w")
            p = subprocess.Popen(cmd, env=env, stdout=log_f, stderr=subprocess.STDOUT)
            running[p] = (slot, num, ovs, attempt, log_f, hb)
            print(f"[launcher:{kind}] job #{num} (attempt {attempt}) on slot {slots[slot]}: "
                  f"{' '.join(o.text() for o in ovs)}", flush=True)
        if hb_timeout > 0:
            now = time.time()
            for p, (slot, num, _, attempt, _, hb) in running.items():
                try:
                    stale = now - hb.stat().st_mtime
                except OSError:
                    stale = 0.0
                if p.poll() is None and stale > hb_timeout:
                    print(f"[launcher:{kind}] job #{num} heartbeat stale for {stale:.0f}s: killing it", flush=True)
                    p.kill()
        done = [p for p in running if p.poll() is not None]
        if not done:
            time.sleep(0.2)
            continue
        for p in done:
            slot, num, ovs, attempt, log_f, hb = running.pop(p)
            log_f.close()
            free.append(slot)
            results[num] = p.returncode
            if p.returncode != 0 and attempt < max_retries:
                print(f"[launcher:{kind}] job #{num} FAILED (exit {p.returncode}); retry {attempt + 1}/{max_retries} "
                      f"with resume=auto", flush=True)
                pending.append((num, ovs, attempt + 1))
            elif p.returncode != 0:
                print(f"[launcher:{kind}] job #{num} FAILED (exit {p.returncode}); see {sweep_dir}/job{num}.out",
                      flush=True)
    return [results[i] for i in range(len(jobs))]


def run(task_fn: Callable[[DictConfig], object], config_path: str, config_name: str, argv: Sequence[str],
        caller_file: Optional[str] = None):
    opts, raw_overrides = _parse_argv(argv)
    base = Path(caller_file).resolve().parent if caller_file else Path.cwd()
    config_dir = Path(opts["config_path"] or config_path)
    if not config_dir.is_absolute():
        config_dir = base / config_dir
    config_name = opts["config_name"] or config_name
    overrides = [parse_override(o) for o in raw_overrides]

    if opts["cfg"] is not None:
        job_cfg, hydra_cfg, _ = compose(config_dir, config_name, overrides, allow_sweep=opts["multirun"])
        if opts["cfg"] == "help":
            print(f"{Path(sys.argv[0]).name} [-m] [--cfg job|hydra|all] key=value ...\n")
            print(OmegaConf.to_yaml(job_cfg))
        elif opts["cfg"] == "hydra":
            print(OmegaConf.to_yaml(hydra_cfg, resolve=opts["resolve"]))
        else:
            print(OmegaConf.to_yaml(job_cfg, resolve=opts["resolve"]))
        return None

    if not opts["multirun"]:
        return _run_job(task_fn, config_dir, config_name, overrides, 0, "run")

    # ---- multirun -------------------------------------------------------
    jobs = expand_sweep(overrides)
    _, hydra_cfg, _ = compose(config_dir, config_name, jobs[0])
    sweep_dir = Path(str(hydra_cfg["sweep"]["dir"]))
    sweep_dir.mkdir(parents=True, exist_ok=True)
    launcher = hydra_cfg["launcher"]
    kind = launcher["_target_"]
    print(f"[{kind}] Launching {len(jobs)} jobs locally")
    with open(sweep_dir / "multirun.yaml", "w") as f:
        yaml.safe_dump({"overrides": [o.text() for o in overrides], "launcher": OmegaConf.to_container(launcher),
                        "jobs": [[o.text() for o in j] for j in jobs]}, f, sort_keys=False)
    parallel = kind == "gpu_pool" or (kind == "joblib" and int(launcher.get("n_jobs", -1) or -1) != 1)
    if parallel and not os.environ.get(_ENV_CHILD):
        flags = []
        if opts["config_name"]:
            flags += ["-cn", opts["config_name"]]
        if opts["config_path"]:
            flags += ["-cp", str(config_dir)]
        codes = _launch_children(jobs, sweep_dir, launcher, sys.argv[0], flags)
        if any(codes):
            raise SystemExit(f"{sum(1 for c in codes if c)} of {len(jobs)} jobs failed")
        return codes
    results = []
    os.environ["MTA_MULTIRUN_INPROC"] = "1"  # the trainer keeps in-process sweep jobs on one device each
    try:
        for num, ovs in enumerate(jobs):
            print(f"\t#{num} : {' '.join(o.text() for o in ovs)}")
            results.append(_run_job(task_fn, config_dir, config_name, ovs, num, "sweep", sweep_dir=sweep_dir))
    finally:
        os.environ.pop("MTA_MULTIRUN_INPROC", None)
    return results


def main(version_base=None, config_path: str = "configs", config_name: str = "config"):
    """Drop-in for ``hydra.main``: ``@main(version_base=None, config_path=..., config_name=...)``."""

    def deco(task_fn):
        caller = sys.modules.get(task_fn.__module__)
        caller_file = getattr(caller, "__file__", None)

        @functools.wraps(task_fn)
        def wrapper(cfg_passthrough: Optional[DictConfig] = None):
            if cfg_passthrough is not None:
                return task_fn(cfg_passthrough)
            return run(task_fn, config_path, config_name, sys.argv[1:], caller_file)

        return wrapper

    return deco
