"""Own multi-GPU launcher: one process per GPU, started by the framework itself.

Reference behaviour: Lightning's ``Trainer()`` with its defaults (``accelerator="auto"``, ``devices="auto"``,
``strategy="auto"``; `/root/reference/train.py:169-180`) re-runs the training script once per extra visible GPU
(its subprocess-script launcher) and turns the original process into rank 0 -- DDP without torchrun.  Here the
same contract is explicit (SURVEY §2.5 "first-class DDP: own launcher, one process per GCD"):

* ``resolve_devices(devices)`` -- ``"auto"`` / ``-1`` = every visible GPU (1 on a CPU host), an int = that many;
* ``launch_script_ranks(n)`` -- called in the ORIGINAL process before it has touched the GPU: starts ranks
  1..n-1 as FRESH child processes re-running the same command line (``subprocess.Popen``: a new program, never an
  exec of this one), with ``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE``/``MASTER_ADDR``/
  ``MASTER_PORT`` set, and makes the current process rank 0 by setting the same variables here;
* a watchdog thread ends the whole job as soon as any rank exits non-zero (the survivors would otherwise sit in
  a collective until its timeout), and at interpreter exit rank 0 waits for its children and exits with the
  first non-zero child status.

Ranks beyond the visible GPUs share them (``parallel.dist``: ``LOCAL_RANK % device_count``), which is how the
multi-rank path is rehearsed on a one-GPU box; the process group is then gloo (RCCL needs one GPU per rank) and
the gradient sync stays the xGMI/IPC kernel.
"""
from __future__ import annotations

import atexit
import os
import socket
import subprocess
import sys
import threading
import time
from typing import Any, List, Optional, Sequence

_CHILDREN: List[subprocess.Popen] = []
_LOCK = threading.Lock()
_WATCHDOG: Optional[threading.Thread] = None
_STOPPING = threading.Event()  # rank 0 itself is ending the job: the watchdog stands down
RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def visible_gpus() -> int:
    """GPUs this process may use, counted WITHOUT initialising HIP (``torch.cuda.device_count`` does not on this
    image; the visibility variables are honoured first)."""
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() not in ("", "-1")])
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # pragma: no cover
        return 0


def resolve_devices(devices: Any = "auto", accelerator: str = "auto") -> int:
    """Number of ranks a ``Trainer(devices=...)`` asks for: ``auto``/``-1``/``None`` = all visible GPUs (at least
    1), an int or digit string = that many, a list = its length (Lightning's device-index form)."""
    if accelerator == "cpu":
        n_vis = 0
    else:
        n_vis = visible_gpus()
    if devices is None or devices == "auto" or devices == -1 or devices == "-1":
        return max(1, n_vis)
    if isinstance(devices, (list, tuple)):
        return max(1, len(devices))
    n = int(devices)
    if n < 1:
        raise ValueError(f"devices must be 'auto', -1 or a positive int, got {devices!r}")
    return n


def in_launched_job() -> bool:
    """True when this process is already one rank of a multi-process job (torchrun, this launcher, a test)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket() as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def _gpu_initialised() -> bool:
    try:
        import torch

        return bool(torch.cuda.is_initialized())
    except Exception:  # pragma: no cover
        return False


def _kill_children() -> None:
    with _LOCK:
        kids = list(_CHILDREN)
    for p in kids:
        if p.poll() is None:
            try:
                p.terminate()
            except OSError:  # pragma: no cover
                pass
    deadline = time.time() + 10
    for p in kids:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()


def _watchdog(poll_s: float = 0.5) -> None:
    """Fail fast: a child rank that exits non-zero takes the whole job down (rank 0 included)."""
    while not _STOPPING.is_set():
        with _LOCK:
            kids = list(_CHILDREN)
        if not kids:
            return
        for i, p in enumerate(kids):
            rc = p.poll()
            if rc is not None and rc != 0 and not _STOPPING.is_set():
                print(f"[launch] rank {i + 1} exited with status {rc}; stopping the job", file=sys.stderr, flush=True)
                _kill_children()
                os._exit(rc if 0 < rc < 256 else 1)
        if all(p.poll() is not None for p in kids):
            return
        time.sleep(poll_s)


def _join_at_exit() -> None:
    """Rank 0's exit: wait for the other ranks; the job's status is the first non-zero one."""
    _STOPPING.set()
    with _LOCK:
        kids = list(_CHILDREN)
    bad = 0
    for i, p in enumerate(kids):
        try:
            rc = p.wait(timeout=float(os.environ.get("MTA_LAUNCH_JOIN_S", "300")))
        except subprocess.TimeoutExpired:
            print(f"[launch] rank {i + 1} still running at rank 0's exit: killing it", file=sys.stderr, flush=True)
            p.kill()
            rc = 1
        if rc and not bad:
            bad = rc
    if bad:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(bad if 0 < bad < 256 else 1)


def launch_script_ranks(n: int, argv: Optional[Sequence[str]] = None, extra_env: Optional[dict] = None,
                        child_stdout=None) -> int:
    """Start ranks 1..n-1 of an ``n``-process job re-running ``argv`` (default: this interpreter + ``sys.argv``) and
    make THIS process rank 0.  Returns ``n``.  Must run before the process initialises the GPU.

    ``child_stdout``: where ranks >= 1 write stdout (default: this process's stderr, so only rank 0's stdout --
    e.g. bench.py's one JSON line -- reaches stdout)."""
    if n <= 1 or in_launched_job():
        return n
    if _gpu_initialised():
        raise RuntimeError("launch_script_ranks: this process already initialised the GPU; the launcher must start "
                           "the other ranks first (start the job earlier, or use torch.distributed.run)")
    if argv is None:
        argv = [sys.executable, *_script_argv()]
    port = int(os.environ.get("MASTER_PORT") or free_port())
    base = dict(MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"), MASTER_PORT=str(port), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    out = sys.stderr if child_stdout is None else child_stdout
    n_vis = visible_gpus()
    if 0 < n_vis < n:
        # ranks time-slicing a GPU: the pipelined LSTM's cross-workgroup waits and the single-launch optimizer's
        # grid-wide norm wait may sit out another process's slice, so they poll longer before giving up (the
        # trial-packing launcher does the same, config/app.py)
        extra_env = dict(extra_env or {})
        for k, v in (("MTA_LSTM_SPIN_LIMIT", str(1 << 25)), ("MTA_ADAM_SPIN_LIMIT", str(1 << 26))):
            if k not in os.environ:
                extra_env.setdefault(k, v)
    for r in range(1, n):
        env = dict(os.environ, **base, RANK=str(r), LOCAL_RANK=str(r), **(extra_env or {}))
        p = subprocess.Popen(list(argv), env=env, stdout=out)
        with _LOCK:
            _CHILDREN.append(p)
    os.environ.update(base, RANK="0", LOCAL_RANK="0", **(extra_env or {}))
    global _WATCHDOG
    _WATCHDOG = threading.Thread(target=_watchdog, name="mta-launch-watchdog", daemon=True)
    _WATCHDOG.start()
    atexit.register(_join_at_exit)
    prev_hook = sys.excepthook

    def _hook(*exc):  # rank 0 failed: the other ranks would wait in a collective until its timeout
        _STOPPING.set()
        prev_hook(*exc)
        sys.stderr.flush()
        _kill_children()

    sys.excepthook = _hook
    print(f"[launch] {n} ranks (1 per GPU, {visible_gpus()} visible): rank 0 = pid {os.getpid()}, children "
          f"{[p.pid for p in _CHILDREN]}, master 127.0.0.1:{port}", file=sys.stderr, flush=True)
    return n


def _script_argv() -> List[str]:
    """The command line that started this interpreter, in re-runnable form (``python -m pkg`` or a script)."""
    main = sys.modules.get("__main__")
    spec = getattr(main, "__spec__", None)
    if spec is not None and spec.name and spec.name != "__main__":
        mod = spec.name[:-len(".__main__")] if spec.name.endswith(".__main__") else spec.name
        return ["-m", mod, *sys.argv[1:]]
    return [os.path.abspath(sys.argv[0]), *sys.argv[1:]]


def children() -> List[subprocess.Popen]:
    with _LOCK:
        return list(_CHILDREN)
