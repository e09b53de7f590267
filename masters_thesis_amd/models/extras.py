"""North-star extra encoder families (``BASELINE.json`` configs 1-4; not in the reference).

``model.arch=mlp`` / ``model.arch=transformer`` swap the reference's LSTM encoder
(`src/model.py:88-94`) for an MLP over the flattened lookback window or a pre-norm
transformer encoder over its T tokens.  Everything else is the reference model: the two
``Linear(H, 1)`` alpha/beta heads, the MSE / Woodbury-NLL / combined losses and their logging
(`src/model.py:176-331`), Adam/AdamW + ReduceLROnPlateau.  Module classes are
``FinancialMlp{Mse,Nll,Combined}`` and ``FinancialTransformer{Mse,Nll,Combined}``, selected by
``get_model_class(loss.module_class, arch)``.

On the GPU the encoders run as bf16-mixed HIP kernels (``ops.extras``) when the matmul precision the trainer
resolves is "medium" (``trainer.precision=bf16-mixed``, e.g. ``trainer=gpu_fast``), and as the fp32 graph under
``32-true`` (the reference trainers' precision, `configs/trainer/fast.yaml:3`); on the CPU as fp32 PyTorch.  A
model used outside a Trainer defaults to "medium".
"""
from __future__ import annotations

import math

import torch
from torch import Tensor

from ..ops import extras as xops
from ..ops._lib import use_hip
from ..ops.losses import decoder_losses, heads_losses_train, train_decoder_fits
from . import register_model_class
from .lstm import FinancialLstmCombined, FinancialLstmMse, FinancialLstmNll

ARCH_PREFIX = {"mlp": "FinancialMlp", "transformer": "FinancialTransformer"}


def _linear_init(w: Tensor, b: Tensor) -> None:
    # nn.Linear's default init
    torch.nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    bound = 1.0 / math.sqrt(w.shape[1])
    torch.nn.init.uniform_(b, -bound, bound)


class _Linear(torch.nn.Module):
    def __init__(self, fin: int, fout: int):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.empty(fout, fin))
        self.bias = torch.nn.Parameter(torch.empty(fout))
        _linear_init(self.weight, self.bias)


class _Norm(torch.nn.Module):
    def __init__(self, d: int, bias: bool):
        super().__init__()
        self.weight = torch.nn.Parameter(torch.ones(d))
        if bias:
            self.bias = torch.nn.Parameter(torch.zeros(d))


class MLPEncoder(torch.nn.Module):
    """``z = flatten(x)``; per layer ``z = Dropout(Norm(GELU(Linear(z))))`` (no dropout after the last)."""

    def __init__(self, input_size: int, lookback: int, hidden_size: int, num_layers: int, dropout: float,
                 norm: str = "layernorm"):
        super().__init__()
        if norm not in ("layernorm", "rmsnorm"):
            raise ValueError(f"norm must be layernorm or rmsnorm, got {norm}")
        self.num_layers, self.dropout, self.norm = num_layers, float(dropout), norm
        self.layers = torch.nn.ModuleList(
            [_Linear(input_size * lookback if i == 0 else hidden_size, hidden_size) for i in range(num_layers)])
        self.norms = torch.nn.ModuleList([_Norm(hidden_size, norm == "layernorm") for _ in range(num_layers)])
        self.register_buffer("seeds", torch.randint(0, 2 ** 62, (max(num_layers, 1),), dtype=torch.int64),
                             persistent=False)

    def flat_params(self):
        out = []
        for lin, nrm in zip(self.layers, self.norms):
            out += [lin.weight, lin.bias, nrm.weight] + ([nrm.bias] if self.norm == "layernorm" else [])
        return out

    precision = "medium"  # set per call by the owning model (its matmul_precision)

    def forward(self, x: Tensor) -> Tensor:
        return xops.mlp_encode(x, self.flat_params(), self.seeds, self.num_layers, self.norm, self.dropout,
                               self.training, self.precision)


class _Block(torch.nn.Module):
    def __init__(self, d: int, mlp_ratio: int):
        super().__init__()
        self.norm1 = _Norm(d, False)
        self.qkv = _Linear(d, 3 * d)
        self.proj = _Linear(d, d)
        self.norm2 = _Norm(d, False)
        self.fc1 = _Linear(d, mlp_ratio * d)
        self.fc2 = _Linear(mlp_ratio * d, d)

    def flat_params(self):
        return [self.norm1.weight, self.qkv.weight, self.qkv.bias, self.proj.weight, self.proj.bias,
                self.norm2.weight, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias]


class TransformerEncoder(torch.nn.Module):
    """Pre-norm encoder: Linear embed -> [x + Attn(RoPE)(RMSNorm x); x + MLP(RMSNorm x)] x L -> RMSNorm(last token)."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int, num_heads: int, mlp_ratio: int = 4,
                 dropout: float = 0.0):
        super().__init__()
        if hidden_size % num_heads or (hidden_size // num_heads) not in (32, 64):
            raise ValueError("transformer: head dim (hidden_size / num_heads) must be 32 or 64")
        self.num_layers, self.num_heads, self.dropout = num_layers, num_heads, float(dropout)
        self.embed = _Linear(input_size, hidden_size)
        self.blocks = torch.nn.ModuleList([_Block(hidden_size, mlp_ratio) for _ in range(num_layers)])
        self.final_norm = _Norm(hidden_size, False)
        self.register_buffer("seeds", torch.randint(0, 2 ** 62, (max(num_layers, 1),), dtype=torch.int64),
                             persistent=False)

    def flat_params(self):
        out = [self.embed.weight, self.embed.bias]
        for b in self.blocks:
            out += b.flat_params()
        return out + [self.final_norm.weight]

    def forward(self, x: Tensor) -> Tensor:
        if x.shape[1] > 64:
            raise ValueError("transformer encoder supports lookback windows of up to 64 tokens")
        return xops.transformer_encode(x, self.flat_params(), self.seeds, self.num_layers, self.num_heads,
                                       self.dropout, self.training, self.precision)

    precision = "medium"


def _make(base, arch: str):
    prefix = ARCH_PREFIX[arch]
    name = base.__name__.replace("FinancialLstm", prefix)

    if arch == "mlp":
        def __init__(self, input_size: int = 3, hidden_size: int = 256, num_layers: int = 2, dropout: float = 0.1,
                     learning_rate: float = 1e-4, weight_decay: float = 1e-5, mse_weight: float = 1e2, *,
                     lookback: int = 60, norm: str = "layernorm", backend: str = "auto", nll_mode: str = "reference",
                     optimizer: str = "adamw"):
            kw = dict(backend=backend, nll_mode=nll_mode, optimizer=optimizer)
            if base is FinancialLstmCombined:
                base.__init__(self, input_size, 8, 1, 0.0, learning_rate, weight_decay, mse_weight, **kw)
            else:
                base.__init__(self, input_size, 8, 1, 0.0, learning_rate, weight_decay, **kw)
            del self.lstm
            self.encoder = MLPEncoder(input_size, lookback, hidden_size, num_layers, dropout, norm)
            self.alpha_head = torch.nn.Linear(hidden_size, 1)
            self.beta_head = torch.nn.Linear(hidden_size, 1)
            self._hparams.clear()
            self.save_hyperparameters()
            self.matmul_precision = "medium"
    else:
        def __init__(self, input_size: int = 3, hidden_size: int = 128, num_layers: int = 4, dropout: float = 0.1,
                     learning_rate: float = 1e-4, weight_decay: float = 1e-5, mse_weight: float = 1e2, *,
                     num_heads: int = 4, mlp_ratio: int = 4, backend: str = "auto", nll_mode: str = "reference",
                     optimizer: str = "adamw"):
            kw = dict(backend=backend, nll_mode=nll_mode, optimizer=optimizer)
            if base is FinancialLstmCombined:
                base.__init__(self, input_size, 8, 1, 0.0, learning_rate, weight_decay, mse_weight, **kw)
            else:
                base.__init__(self, input_size, 8, 1, 0.0, learning_rate, weight_decay, **kw)
            del self.lstm
            self.encoder = TransformerEncoder(input_size, hidden_size, num_layers, num_heads, mlp_ratio, dropout)
            self.alpha_head = torch.nn.Linear(hidden_size, 1)
            self.beta_head = torch.nn.Linear(hidden_size, 1)
            self._hparams.clear()
            self.save_hyperparameters()
            self.matmul_precision = "medium"

    def encode(self, x: Tensor) -> Tensor:
        self.encoder.precision = self.matmul_precision
        return self.encoder(x)

    def _losses(self, batch, want_nll: bool, acc, coeffs=None):
        """The MLP's bf16 HIP path with the alpha / beta heads fused into its last norm kernels
        (``ops.extras.mlp_encode_heads``: no h / dh round trip, no separate head kernels) and the losses on the
        resulting (N, 2) ``ab`` (``ops.losses.decoder_losses``); every other case: the reference composition."""
        enc = getattr(self, "encoder", None)
        if arch != "mlp" or self.backend == "torch":
            return base._losses(self, batch, want_nll, acc, coeffs)
        context, target, factor, inv_psi, B = self._unpack(batch)
        enc.precision = self.matmul_precision
        params = enc.flat_params()
        if not xops.mlp_heads_fusable(context, params, enc.num_layers, enc.norm, enc.precision):
            return base._losses(self, batch, want_nll, acc, coeffs)
        heads = (self.alpha_head.weight, self.alpha_head.bias, self.beta_head.weight, self.beta_head.bias)
        ab = xops.mlp_encode_heads(context, params, enc.seeds, enc.num_layers, enc.norm, enc.dropout, enc.training,
                                   enc.precision, heads)
        c_nll, c_mse = coeffs if coeffs is not None else self.loss_coefficients
        return decoder_losses(ab, target, factor, inv_psi, batch_windows=B, want_nll=want_nll,
                              nll_mode=self.nll_mode, c_nll=c_nll, c_mse=c_mse, acc=acc.acc, with_total=True)

    def fused_step_supported(self, batch) -> bool:
        """The training step as [encoder forward (HIP autograd Function), the one-launch decoder (losses, metrics,
        dh, head grads: ops.losses.heads_losses_train), encoder backward from dh]: two decoder launches (the
        heads/losses forward and its backward) become one.  HIP path, decoder small enough for one workgroup."""
        x, y = batch[0], batch[1]
        if self.backend == "torch" or not use_hip(x) or not self.training:
            return False
        if any(p.grad is None for p in self.parameters()):
            return False
        return train_decoder_fits(int(x.shape[0]) * int(x.shape[1]), int(y.shape[2]),
                                  int(self.alpha_head.weight.shape[1]))

    def fused_training_step(self, batch, batch_idx):
        """``training_step`` + ``loss.backward()`` with the decoder in one launch (same math and metric bookkeeping
        as the autograd path: tests/test_gpu_extras.py)."""
        if getattr(batch, "pending", False):
            batch.materialize()
        context, target, factor, inv_psi, B = self._unpack(batch)
        h = self.encode(context)
        c_nll, c_mse = self.loss_coefficients
        grads = (self.alpha_head.weight.grad, self.alpha_head.bias.grad, self.beta_head.weight.grad,
                 self.beta_head.bias.grad)
        N, H = h.shape
        dh_buf = None
        if arch == "mlp" and N % 16:
            # the MLP encoder runs 16-row padded: the decoder writes dh into that padded shape with zero pad rows,
            # so the encoder backward reads it in place (no zero-fill + copy launches)
            dh_buf = torch.empty(((N + 15) // 16 * 16, H), device=h.device, dtype=torch.float32)
            dh_buf._mta_zero_pad = True
        out, dh = heads_losses_train(h.detach(), self.alpha_head.weight, self.alpha_head.bias,
                                     self.beta_head.weight, self.beta_head.bias, target, factor, inv_psi,
                                     batch_windows=B, want_nll=self.want_nll, nll_mode=self.nll_mode, c_nll=c_nll,
                                     c_mse=c_mse, acc=self.train_acc.acc, grads=grads, dh=dh_buf)
        h.backward(dh if dh_buf is None else dh_buf[:N])
        self._log_stage("train", self.train_acc, self.train_log_names)
        return out[3]

    cls = type(name, (base,), {"__init__": __init__, "encode": encode, "_losses": _losses,
                               "fused_step_supported": fused_step_supported,
                               "fused_training_step": fused_training_step,
                               "__doc__": f"{base.__name__} with the {arch} encoder (north-star extra)."})
    return cls


FinancialMlpMse = _make(FinancialLstmMse, "mlp")
FinancialMlpNll = _make(FinancialLstmNll, "mlp")
FinancialMlpCombined = _make(FinancialLstmCombined, "mlp")
FinancialTransformerMse = _make(FinancialLstmMse, "transformer")
FinancialTransformerNll = _make(FinancialLstmNll, "transformer")
FinancialTransformerCombined = _make(FinancialLstmCombined, "transformer")

for _c in (FinancialMlpMse, FinancialMlpNll, FinancialMlpCombined, FinancialTransformerMse, FinancialTransformerNll,
           FinancialTransformerCombined):
    register_model_class(_c.__name__, _c)

__all__ = ["ARCH_PREFIX", "MLPEncoder", "TransformerEncoder", "FinancialMlpMse", "FinancialMlpNll",
           "FinancialMlpCombined", "FinancialTransformerMse", "FinancialTransformerNll",
           "FinancialTransformerCombined"]
