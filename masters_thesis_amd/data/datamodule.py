"""``FinancialLstmDataModule``: raw series -> windows -> OLS targets -> 70/20/10 splits -> loaders.

Reference: `src/data.py:133-250` (+ the import-time bootstrap of `train.py:15-36`).  Same
hyper-parameters, tensor contract and split; what changes:

* **Lazy, per-source bootstrap** (SURVEY Q6): ``prepare_data`` creates the raw series only for
  the data module in use — synthetic series from the DGP (on the GPU when one is attached),
  real series from the Fama-French CSVs in ``raw_dir`` — next to a ``source.json`` recording
  how they were made (a changed ``n_samples``/``seed`` regenerates them).
* **Dataset build on the device**: windowing is a strided view, features one fused
  elementwise op, the OLS targets one ``csrc/data.hip`` launch for all windows.
* **Race-free cache** (SURVEY Q7): one ``datasets/dataset-<hash>.pt`` per parameter hash
  (windowing parameters + data source), written under a file lock to a temporary file and
  renamed into place; ``hparams_hash.txt`` is kept for layout compatibility.  The file is a
  plain dict of tensors loaded with ``weights_only=True``.  ``cache=False`` keeps everything in
  memory (``bench.py``).
* **Residency** (MI355X, 288 GB HBM): ``device`` keeps the whole split in HBM (1.3 GB for the
  default synthetic set) and the engine gathers batches inside its captured step graph;
  ``stream`` keeps it in pinned host memory behind the native prefetcher (``prefetch.py``).
* **Sharding**: with ``world_size > 1`` the train loader gives each rank an equal share of the
  epoch order; val/test loaders split the windows without padding (metrics are summed
  across ranks).

A batch is ``(X (B, K, T, F), y (B, K, n, 4), factor (B, 2), inv_psi (B, K))`` with
``y`` channels ``[r_stock, r_market, alpha, beta]``.
"""
from __future__ import annotations

import hashlib
import json
from pathlib import Path
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import Tensor

from .cache import atomic_torch_save, atomic_write_text, file_lock, remove_cached_datasets
from .common import add_quadratic_features, append_feature, lookback_target_split
from .dgp import SyntheticLogReturns
from .famafrench import FamaFrench25Portfolios
from .loaders import TensorBatchLoader
from .prefetch import StreamingLoader

__all__ = ["FinancialLstmDataModule", "TensorBatchLoader", "build_windows"]

SPLIT_FRACTIONS = (0.7, 0.9)  # train | val | test boundaries (`src/data.py:225-234`)


def build_windows(r_stocks: Tensor, r_market: Tensor, alphas: Optional[Tensor], betas: Optional[Tensor], *,
                  lookback_window: int, target_window: int, stride: int, prediction_task: bool,
                  interaction_only: bool) -> Dict[str, Tensor]:
    """The dataset tensors of `src/data.py:197-216`, computed where the inputs live."""
    from ..ops.ols import ols_features

    X, y = lookback_target_split(r_stocks, r_market, lookback_window, target_window, stride, prediction_task)
    X = add_quadratic_features(X, interaction_only=interaction_only).contiguous()
    y = y.contiguous()
    t_alphas, t_betas, factor, inv_psi = ols_features(y)
    if alphas is None or betas is None:  # real data: no ground truth, the OLS targets stand in
        alphas, betas = t_alphas, t_betas
    y = append_feature(append_feature(y, alphas.to(y.device)), betas.to(y.device)).contiguous()
    return {"X": X, "y": y, "factor": factor.contiguous(), "inv_psi": inv_psi.contiguous()}


class FinancialLstmDataModule:
    KEYS = ("X", "y", "factor", "inv_psi")

    def __init__(self, data_dir, lookback_window: int = 60, target_window: int = 20, stride: int = 80,
                 prediction_task: bool = True, interaction_only: bool = True, batch_size: int = 1, *,
                 name: str = "synthetic", n_stocks: int = 100, n_samples: int = 1_000_000, seed: int = 0,
                 dgp_variant: str = "no_outliers", raw_dir=None, residency: str = "device", cache: bool = True,
                 device=None, rank: int = 0, world_size: int = 1, prefetch_slots: int = 3,
                 prefetch_threads: int = 4):
        if not prediction_task and target_window > lookback_window:
            raise ValueError("target window must be <= lookback window for reconstruction task")
        if residency not in ("device", "stream"):
            raise ValueError(f"datamodule.residency must be 'device' or 'stream', got {residency!r}")
        self.data_dir = Path(data_dir)
        self.hparams = dict(lookback_window=int(lookback_window), target_window=int(target_window),
                            stride=int(stride), prediction_task=bool(prediction_task),
                            interaction_only=bool(interaction_only), batch_size=int(batch_size))
        self.name = str(name)
        self.n_stocks, self.n_samples, self.seed = int(n_stocks), int(n_samples), int(seed)
        self.dgp_variant = dgp_variant
        self.raw_dir = Path(raw_dir) if raw_dir is not None else self.data_dir.parent / "real_raw"
        self.residency = residency
        self.cache = bool(cache)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.rank, self.world_size = int(rank), int(world_size)
        self.prefetch_slots, self.prefetch_threads = int(prefetch_slots), int(prefetch_threads)
        self.dataset: Optional[List[Tensor]] = None
        self.splits: Dict[str, Tuple[int, int]] = {}
        self._memory: Optional[Dict[str, Tensor]] = None
        self._loaders: List[Any] = []

    @classmethod
    def from_config(cls, cfg, **overrides) -> "FinancialLstmDataModule":
        c = dict(cfg.items()) if hasattr(cfg, "items") else dict(cfg)
        kw = {k: c[k] for k in ("lookback_window", "target_window", "stride", "prediction_task", "interaction_only",
                                "batch_size", "name", "n_stocks", "n_samples", "seed", "dgp_variant", "raw_dir",
                                "residency", "prefetch_slots", "prefetch_threads") if k in c and c[k] is not None}
        kw.update(overrides)
        return cls(c["data_dir"], **kw)

    # ------------------------------------------------------------------ identity / cache paths
    @property
    def is_real(self) -> bool:
        return self.name == "real"

    def source_signature(self) -> Dict[str, Any]:
        if self.is_real:
            return {"kind": "famafrench25", "n_samples": FamaFrench25Portfolios.n_samples,
                    "skip_old_data": FamaFrench25Portfolios.skip_old_data}
        return {"kind": "synthetic", "n_stocks": self.n_stocks, "n_samples": self.n_samples, "seed": self.seed,
                "variant": self.dgp_variant}

    def _compute_hparams_hash(self) -> str:
        h = {k: self.hparams[k] for k in ("lookback_window", "target_window", "stride", "prediction_task",
                                          "interaction_only")}
        h["source"] = self.source_signature()
        return hashlib.sha256(json.dumps(h, sort_keys=True).encode()).hexdigest()

    @property
    def datasets_dir(self) -> Path:
        return self.data_dir / "datasets"

    def dataset_path(self) -> Path:
        return self.datasets_dir / f"dataset-{self._compute_hparams_hash()[:16]}.pt"

    def _stored_source(self) -> Optional[Dict[str, Any]]:
        p = self.data_dir / "source.json"
        if p.exists():
            try:
                return json.loads(p.read_text())
            except ValueError:
                return None
        return None

    # ------------------------------------------------------------------ raw series
    def _build_device(self) -> torch.device:
        return self.device if self.device.type == "cuda" else torch.device("cpu")

    def _raw_series(self, persist: bool):
        """(r_stocks, r_market, alphas|None, betas|None); generated/loaded and optionally saved."""
        d = self.data_dir
        have = (d / "stocks.pt").exists() and (d / "market.pt").exists()
        stored = self._stored_source()
        fresh = have and (stored is None or stored == self.source_signature())
        if persist and fresh:
            load = lambda f: torch.load(d / f, map_location="cpu", weights_only=True)  # noqa: E731
            opt = lambda f: load(f) if (d / f).exists() else None  # noqa: E731
            return load("stocks.pt"), load("market.pt"), opt("alphas.pt"), opt("betas.pt")
        if self.is_real:
            p25, mkt = FamaFrench25Portfolios.load(self.raw_dir)
            series = (p25, mkt, None, None)
        else:
            series = SyntheticLogReturns.generate(self.n_stocks, self.n_samples, device=self._build_device(),
                                                  seed=self.seed, variant=self.dgp_variant)
        if persist:
            d.mkdir(parents=True, exist_ok=True)
            for f, t in zip(("stocks.pt", "market.pt", "alphas.pt", "betas.pt"), series):
                if t is not None:
                    atomic_torch_save(t.detach().cpu().contiguous(), d / f)
            atomic_write_text(d / "source.json", json.dumps(self.source_signature(), sort_keys=True))
        return series

    def _build(self, persist: bool) -> Dict[str, Tensor]:
        r_s, r_m, a, b = self._raw_series(persist)
        dev = self._build_device()
        hp = {k: v for k, v in self.hparams.items() if k != "batch_size"}
        return build_windows(r_s.to(dev), r_m.to(dev), None if a is None else a.to(dev),
                             None if b is None else b.to(dev), **hp)

    # ------------------------------------------------------------------ Lightning-style hooks
    def prepare_data(self) -> None:
        """Create (once) the cached dataset for these parameters (`src/data.py:177-219`)."""
        if not self.cache:
            if self._memory is None:
                self._memory = self._build(persist=False)
            return
        with file_lock(self.data_dir / ".lock"):
            path = self.dataset_path()
            if path.exists():
                print("Dataset parameters unchanged, skipping data preparation")
                return
            ds = self._build(persist=True)
            self.datasets_dir.mkdir(parents=True, exist_ok=True)
            atomic_torch_save({k: ds[k].detach().cpu().contiguous() for k in self.KEYS}, path)
            atomic_write_text(self.datasets_dir / "hparams_hash.txt", self._compute_hparams_hash())

    def _load(self) -> Dict[str, Tensor]:
        if self._memory is not None:
            return self._memory
        if not self.cache:
            self.prepare_data()
            return self._memory
        path = self.dataset_path()
        if not path.exists():
            self.prepare_data()
            path = self.dataset_path()
        ds = torch.load(path, map_location="cpu", weights_only=True)
        return {k: ds[k] for k in self.KEYS}

    def setup(self, stage: Optional[str] = None) -> None:
        ds = self._load()
        tensors = [ds[k] for k in self.KEYS]
        if self.device.type == "cuda":
            if self.residency == "device":
                tensors = [t.to(self.device, non_blocking=True).contiguous() for t in tensors]
            else:
                tensors = [t.cpu().contiguous().pin_memory() for t in tensors]
        else:
            tensors = [t.cpu().contiguous() for t in tensors]
        self._memory = None if self.cache else {k: t for k, t in zip(self.KEYS, tensors)}
        self.dataset = tensors
        n = int(tensors[0].shape[0])
        a, b = int(SPLIT_FRACTIONS[0] * n), int(SPLIT_FRACTIONS[1] * n)
        self.splits = {"train": (0, a), "val": (a, b), "test": (b, n)}

    @property
    def n_windows(self) -> int:
        return 0 if self.dataset is None else int(self.dataset[0].shape[0])

    # ------------------------------------------------------------------ loaders
    def _loader(self, split: str, batch_size: int, shuffle: bool):
        if self.dataset is None:
            self.setup("fit" if split != "test" else "test")
        start, stop = self.splits[split]
        base = TensorBatchLoader(self.dataset, batch_size, shuffle=shuffle, seed=self.seed,
                                 rank=self.rank, world_size=self.world_size, start=start, stop=stop)
        if self.device.type == "cuda" and self.residency == "stream":
            ld = StreamingLoader(base, self.device, slots=self.prefetch_slots, threads=self.prefetch_threads)
            self._loaders.append(ld)
            return ld
        return base

    def train_dataloader(self):
        return self._loader("train", self.hparams["batch_size"], True)

    def val_dataloader(self):
        return self._loader("val", 1, False)

    def test_dataloader(self):
        return self._loader("test", 1, False)

    def teardown(self, stage: Optional[str] = None) -> None:
        for ld in self._loaders:
            ld.close()
        self._loaders.clear()
        if stage == "cleanup":  # explicit opt-in (the reference's is unreachable)
            remove_cached_datasets(self.datasets_dir)
