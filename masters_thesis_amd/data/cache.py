"""Dataset-cache file helpers: atomic writes (temporary file + rename) and an advisory file lock, so
concurrent sweep jobs never read a half-written dataset."""
from __future__ import annotations

import contextlib
import os
from pathlib import Path

import torch


def atomic_torch_save(obj, path: Path) -> None:
    tmp = path.with_name(f".{path.name}.tmp{os.getpid()}")
    torch.save(obj, tmp)
    os.replace(tmp, path)


def atomic_write_text(path: Path, text: str) -> None:
    tmp = path.with_name(f".{path.name}.tmp{os.getpid()}")
    tmp.write_text(text)
    os.replace(tmp, path)


@contextlib.contextmanager
def file_lock(path: Path):
    import fcntl

    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "a+") as f:
        fcntl.flock(f.fileno(), fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)


def remove_cached_datasets(datasets_dir: Path) -> None:
    """The reference's ``teardown('cleanup')`` (`src/data.py:246-250`): drop the cached datasets."""
    d = Path(datasets_dir)
    if not d.exists():
        return
    for p in d.glob("dataset*.pt"):
        p.unlink(missing_ok=True)
    (d / "hparams_hash.txt").unlink(missing_ok=True)
    with contextlib.suppress(OSError):
        d.rmdir()
