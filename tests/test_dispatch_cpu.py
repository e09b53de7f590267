"""Host-side dispatch rules of round 5 (no GPU): which decoder / encoder path a configuration takes.

* ``ops.losses.train_decoder_fits``: the one-workgroup training decoder only up to ``TRAIN_DECODER_MAX_N`` sequences
  (at N = 800 it cost 185 us a step against the grid decoder path, ``profiles/r5_decoder_maxn_ab.txt``);
* ``ops.extras.mlp_heads_fusable`` / ``mlp_encode_heads``: the alpha / beta heads fuse into the MLP's last norm
  only on the bf16 HIP path with a wide last layer; elsewhere ``mlp_encode_heads`` is the plain composition
  ``heads(encoder(x))`` (checked here on the CPU against the reference MLP + addmm);
* ``ops.extras._gelu_in_norm``: the GELU-on-load widths are exactly the wide-kernel ones.
"""
import torch

from masters_thesis_amd.ops import extras as X
from masters_thesis_amd.ops.losses import TRAIN_DECODER_MAX_N, train_decoder_fits


def test_train_decoder_cap():
    assert TRAIN_DECODER_MAX_N == 256
    assert train_decoder_fits(100, 30, 64)  # the headline: B = 1 window of 100 stocks
    assert train_decoder_fits(200, 30, 64)  # B = 2 keeps the one-launch decoder (and the LSTM's fused step)
    assert not train_decoder_fits(800, 30, 64)  # B = 8: the grid decoder path
    assert not train_decoder_fits(6400, 30, 64)


def test_gelu_in_norm_widths():
    assert [d for d in (128, 256, 512, 1024, 1536, 2048, 4096) if X._gelu_in_norm(d)] == [1024, 2048]


def test_mlp_heads_cpu_is_the_plain_composition():
    from masters_thesis_amd.models.extras import MLPEncoder

    torch.manual_seed(0)
    N, T, F, H, L = 12, 60, 3, 1024, 2
    enc = MLPEncoder(F, T, H, L, 0.0, "layernorm")
    x = torch.randn(N, T, F)
    heads = (torch.randn(1, H) * 0.05, torch.randn(1), torch.randn(1, H) * 0.05, torch.randn(1))
    params = enc.flat_params()
    assert not X.mlp_heads_fusable(x, params, L, "layernorm", "medium")  # CPU tensors: no HIP path
    ab = X.mlp_encode_heads(x, params, enc.seeds, L, "layernorm", 0.0, False, "medium", heads)
    h = X.mlp_reference(x, params, L, "layernorm", 0.0, False)
    ref = torch.addmm(torch.cat([heads[1], heads[3]]), h, torch.cat([heads[0], heads[2]], 0).t())
    assert ab.shape == (N, 2)
    torch.testing.assert_close(ab, ref)
