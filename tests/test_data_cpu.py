"""Data module on the CPU: window counts and the 70/20/10 split, cache reuse / invalidation, loader
sharding and epoch order, DGP moments."""
import math

import pytest
import torch
from hypothesis import given, settings, strategies as st

from masters_thesis_amd.data import FinancialLstmDataModule, SyntheticLogReturns, TensorBatchLoader
from masters_thesis_amd.data.common import lookback_target_split


def _dm(tmp_path, **kw):
    args = dict(lookback_window=60, target_window=30, stride=90, n_stocks=8, n_samples=9000, seed=3)
    args.update(kw)
    return FinancialLstmDataModule(tmp_path / "synthetic", **args)


def test_reference_window_count_and_split():
    # synthetic config: 1e6 days, span = stride = 90 -> 11,111 windows, split 7,777 / 2,222 / 1,112
    rs, rm = torch.zeros(1, 1_000_000), torch.zeros(1_000_000)
    X, y = lookback_target_split(rs, rm, 60, 30, 90, True)
    n = X.shape[0]
    assert n == 11_111 and y.shape[2] == 30
    a, b = int(0.7 * n), int(0.9 * n)
    assert (a, b - a, n - b) == (7_777, 2_222, 1_112)


def test_prepare_setup_shapes_and_channels(tmp_path):
    dm = _dm(tmp_path)
    dm.prepare_data()
    dm.setup("fit")
    X, y, factor, inv_psi = dm.dataset
    W = 9000 // 90
    assert X.shape == (W, 8, 60, 3) and y.shape == (W, 8, 30, 4)
    assert factor.shape == (W, 2) and inv_psi.shape == (W, 8)
    assert dm.splits == {"train": (0, 70), "val": (70, 90), "test": (90, 100)}
    alphas = torch.load(tmp_path / "synthetic/alphas.pt", weights_only=True)
    # y channels 2/3 hold the TRUE coefficients, broadcast over windows and days
    torch.testing.assert_close(y[:, :, :, 2], alphas.view(1, 8, 1).expand(W, 8, 30))
    torch.testing.assert_close(X[..., 2], X[..., 0] * X[..., 1])
    assert torch.isfinite(inv_psi).all() and (inv_psi > 0).all()


def test_cache_reuse_and_invalidation(tmp_path, capsys):
    dm = _dm(tmp_path)
    dm.prepare_data()
    first = dm.dataset_path()
    assert first.exists() and (tmp_path / "synthetic/datasets/hparams_hash.txt").exists()
    _dm(tmp_path).prepare_data()
    assert "skipping data preparation" in capsys.readouterr().out
    # new windowing parameters -> a second cache file next to the first
    other = _dm(tmp_path, stride=45)
    other.prepare_data()
    assert other.dataset_path() != first and first.exists() and other.dataset_path().exists()
    # a different data source regenerates the raw series and the dataset
    bigger = _dm(tmp_path, n_samples=12_000)
    bigger.prepare_data()
    bigger.setup("fit")
    assert bigger.n_windows == 12_000 // 90
    bigger.teardown("cleanup")
    assert not (tmp_path / "synthetic/datasets").exists()


def test_in_memory_mode_writes_nothing(tmp_path):
    dm = _dm(tmp_path, cache=False)
    dm.setup("fit")
    assert dm.n_windows == 100 and not (tmp_path / "synthetic").exists()


def test_reconstruction_task_and_validation(tmp_path):
    dm = _dm(tmp_path, prediction_task=False, target_window=20, stride=60, cache=False)
    dm.setup("fit")
    X, y = dm.dataset[0], dm.dataset[1]
    assert X.shape[2] == 60 and y.shape[2] == 20
    torch.testing.assert_close(y[:, :, :, 0], X[:, :, 40:, 0])
    with pytest.raises(ValueError):
        _dm(tmp_path, prediction_task=False, target_window=70)
    with pytest.raises(ValueError):
        _dm(tmp_path, residency="nowhere")


@pytest.mark.parametrize("world", [2, 3])
def test_train_shards_are_disjoint_and_equal(world):
    X = torch.arange(50.0).view(50, 1)
    shards = [TensorBatchLoader([X], 2, shuffle=True, seed=5, rank=r, world_size=world, start=3, stop=48)
              for r in range(world)]
    rows = [torch.cat([b[0].flatten() for b in ld]).long() for ld in shards]
    assert len({r.numel() for r in rows}) == 1  # equal step counts on every rank
    allr = torch.cat(rows)
    assert allr.unique().numel() == allr.numel() and allr.min() >= 3 and allr.max() < 48
    assert allr.numel() == (45 // world) * world
    # eval shards cover every window exactly once, without padding
    ev = [TensorBatchLoader([X], 1, shuffle=False, rank=r, world_size=world, start=3, stop=48) for r in range(world)]
    assert sorted(torch.cat([torch.cat([b[0].flatten() for b in ld]) for ld in ev]).long().tolist()) == list(range(3, 48))


def test_epoch_order_changes_per_epoch_and_is_reproducible():
    X = torch.arange(20.0).view(20, 1)
    ld = TensorBatchLoader([X], 4, shuffle=True, seed=1)
    e0 = ld.epoch_indices(0)
    assert not torch.equal(e0, ld.epoch_indices(1))
    assert torch.equal(e0, TensorBatchLoader([X], 4, shuffle=True, seed=1).epoch_indices(0))
    assert len(ld) == 5 and sorted(e0.tolist()) == list(range(20))


@settings(max_examples=10, deadline=None)
@given(seed=st.integers(0, 2 ** 31 - 1))
def test_dgp_moments_cpu(seed):
    K, N = 16, 40_000
    r_s, r_m, al, be = SyntheticLogReturns.generate(K, N, seed=seed)
    assert r_s.shape == (K, N) and r_m.shape == (N,) and al.shape == be.shape == (K,)
    mk, idio = SyntheticLogReturns.mkt_params, SyntheticLogReturns.idio_params
    t_var = mk["df"] / (mk["df"] - 2)
    m = r_m.double()
    assert abs(m.mean().item() - mk["loc"]) < 6 * mk["scale"] * math.sqrt(t_var / N)
    eps = r_s.double() - al.double()[:, None] - be.double()[:, None] * m[None]
    assert abs(eps.var().item() / (idio["scale"] ** 2 * t_var) - 1) < 0.1
    again = SyntheticLogReturns.generate(K, N, seed=seed)
    assert torch.equal(again[0], r_s)
