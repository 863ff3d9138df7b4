"""MMIMDb late-fusion path (BASELINE configs[3]) on the HIP kernels.

Drop-in classes for the reference's YAML tags / resolver (config/yaml_constructors.py:126-142,
config/resolvers.py:44-47) with the reference's constructor arguments, attribute names and
``state_dict`` keys (MML_Suite/models/mmimdb.py, models/gates/gated_bimodal.py, models/maxout.py):

    image_model / text_model : MMIMDbModalityEncoder  = BatchNorm1d(in) → Linear(in, out)
    fusion_module            : GatedBiModalNetwork    = tanh(fc_one), tanh(fc_two), gate, mix
    mm_mlp                   : MLPGenreClassifier     = BN → MaxOut → Dropout → BN → MaxOut → Dropout → BN → Linear

The submodules hold parameters only; every computation runs in ``MMIMDbEngine`` as gfx950 HIP
kernels behind the C ABI (include/tspm.h): BatchNorm1d = ``tspm_bn1d_fwd/bwd`` (one launch each way)
and ``tspm_bn_apply_eval`` over [n, C] rows, Linear / MaxOut products = ``tspm_linear_*`` (MFMA small GEMM; the two MaxOut units' weights
are adjacent in FusedAdam's flat buffer and run as ONE [2d, in] product), GMU / MaxOut+Dropout /
BCEWithLogits = ``tspm_gmu_*``, ``tspm_maxout_*``, ``tspm_bce_logits``, Adam = ``tspm_adam_step``.
``FusedMMIMDbStep`` captures forward + loss + backward + Adam in one HIP graph.  No CPU or ATen
fallback: a CPU tensor raises ``TspmError``.

Supported configuration = the reference's MMIMDb configs: GMU fusion or ``multimodal_pooling``
(``MultimodalPooling``, models/pooling.py: max / avg / sum / attention / gated; ``tspm_pool_*``),
MaxOut with 2 units and no bias, Dropout 0.5, biasless GMU.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional

import torch
from torch import nn

from . import _lib as L
from ._lib import linear_bwd
from .optim import FusedAdam
from .step import shared_batches_tracked

_BN_MOMENTUM_DEFAULT = 0.1
# the independent image / text launches (input BatchNorm1d forward and backward, the GMU projections) as
# merged pairs (bitwise the separate launches; 665-670k -> 756k samples/s)
_PAIRS = True
# dropout masks drawn inside the MaxOut forwards (tspm_maxout_fwd_rng; the bits of tspm_dropout_mask)
_RNG_INLAUNCH = True


# ------------------------------------------------------------------------------------------------
# parameter containers (reference attribute names / state_dict keys)
# ------------------------------------------------------------------------------------------------
class MaxOut(nn.Module):
    """models/maxout.py: ``layers`` = num_units × Linear(input_dim, output_dim)."""

    def __init__(self, input_dim: int, output_dim: int, num_units: int = 2, use_bias: bool = True) -> None:
        super().__init__()
        self.input_dim, self.output_dim, self.num_units, self.use_bias = input_dim, output_dim, num_units, use_bias
        self.layers = nn.ModuleList([nn.Linear(input_dim, output_dim, bias=use_bias) for _ in range(num_units)])

    def forward(self, x):  # pragma: no cover - the engine runs the layer
        raise L.TspmError("MaxOut runs inside MMIMDb's HIP engine (call the MMIMDb model)")


class MMIMDbModalityEncoder(nn.Module):
    """models/mmimdb.py:63-93."""

    def __init__(self, input_dim: int, output_dim: int) -> None:
        super().__init__()
        self.net = nn.Sequential(nn.BatchNorm1d(input_dim), nn.Linear(input_dim, output_dim))

    def forward(self, x):  # pragma: no cover
        raise L.TspmError("MMIMDbModalityEncoder runs inside MMIMDb's HIP engine (call the MMIMDb model)")


class GatedBiModalNetwork(nn.Module):
    """models/gates/gated_bimodal.py."""

    def __init__(self, input_one_dim: int, input_two_dim: int, output_one_dim: int, output_two_dim: int, *,
                 use_bias: bool = False) -> None:
        super().__init__()
        self.fc_one = nn.Linear(input_one_dim, output_one_dim, bias=use_bias)
        self.fc_two = nn.Linear(input_two_dim, output_two_dim, bias=use_bias)
        self.hidden_sigmoid = nn.Linear(output_one_dim + output_two_dim, 1, bias=use_bias)
        self.activation = nn.Tanh()
        self.gate_activation = nn.Sigmoid()
        self.use_bias = use_bias

    def forward(self, a, b):  # pragma: no cover
        raise L.TspmError("GatedBiModalNetwork runs inside MMIMDb's HIP engine (call the MMIMDb model)")


POOLING_KINDS = {"max": 0, "avg": 1, "average": 1, "sum": 2, "attention": 3, "gated": 4}


class MultimodalPooling(nn.Module):
    """models/pooling.py:6-127 parameter container (same construction order and state_dict keys):
    proj_a / proj_b, Dropout, Tanh, and the attention (Linear → Tanh → Linear(·, 2) → Softmax) or gate
    (Linear → Tanh → Linear(·, 1) → Sigmoid) scoring MLP; the engine runs it (tspm_pool_*)."""

    def __init__(self, input_dim_a: int, input_dim_b: int, output_dim: int, pooling_type: str = "gated",
                 hidden_dim: Optional[int] = None, dropout: float = 0.0):
        super().__init__()
        self.pooling_type = pooling_type.lower()
        if self.pooling_type not in POOLING_KINDS:
            raise ValueError(f"Unknown pooling type: {self.pooling_type}")
        self.input_dim_a, self.input_dim_b, self.output_dim = input_dim_a, input_dim_b, output_dim
        self.hidden_dim = hidden_dim or max(input_dim_a, input_dim_b)
        self.dropout = dropout
        self.proj_a = nn.Linear(input_dim_a, output_dim)
        self.proj_b = nn.Linear(input_dim_b, output_dim)
        self.dropout_layer = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.activation = nn.Tanh()
        if self.pooling_type == "attention":
            self.attention_layer = nn.Sequential(nn.Linear(output_dim * 2, self.hidden_dim), nn.Tanh(),
                                                 nn.Linear(self.hidden_dim, 2), nn.Softmax(dim=1))
        elif self.pooling_type == "gated":
            self.gate_layer = nn.Sequential(nn.Linear(output_dim * 2, self.hidden_dim), nn.Tanh(),
                                            nn.Linear(self.hidden_dim, 1), nn.Sigmoid())

    @property
    def kind(self) -> int:
        return POOLING_KINDS[self.pooling_type]

    def scorer(self) -> Optional[nn.Sequential]:
        return getattr(self, "attention_layer", None) or getattr(self, "gate_layer", None)

    def forward(self, a, b):  # pragma: no cover - the engine runs the fusion
        raise L.TspmError("MultimodalPooling runs inside the MMIMDb HIP engine")


class MLPGenreClassifier(nn.Module):
    """models/mmimdb.py:20-60."""

    def __init__(self, input_size: int, output_size: int, hidden_size: int) -> None:
        super().__init__()
        self.input_size, self.output_size, self.hidden_size = input_size, output_size, hidden_size
        self.net = nn.Sequential(
            nn.BatchNorm1d(input_size), MaxOut(input_size, hidden_size, use_bias=False), nn.Dropout(p=0.5),
            nn.BatchNorm1d(hidden_size), MaxOut(hidden_size, hidden_size, use_bias=False), nn.Dropout(p=0.5),
            nn.BatchNorm1d(hidden_size), nn.Linear(hidden_size, output_size))

    def forward(self, x):  # pragma: no cover
        raise L.TspmError("MLPGenreClassifier runs inside MMIMDb's HIP engine (call the MMIMDb model)")


def _bce_weight(loss_functions) -> float:
    """Weight of the single bce_with_logits term of a LossFunctionGroup (experiment_utils/loss.py:52,
    98-148); anything else is not the MMIMDb configuration and raises."""
    if loss_functions is None:
        return 1.0
    items = list(loss_functions.items())
    if len(items) != 1:
        raise L.TspmError("MMIMDb HIP step: expected one loss term (bce_with_logits)")
    term = items[0][1]
    fn = getattr(term, "loss_fn", None)
    if not isinstance(fn, nn.BCEWithLogitsLoss) or fn.reduction != "mean" or fn.weight is not None \
            or fn.pos_weight is not None:
        raise L.TspmError("MMIMDb HIP step: the loss must be BCEWithLogitsLoss(reduction='mean')")
    return float(getattr(term, "weight", 1.0))


def _bn(m: nn.BatchNorm1d):
    return m.weight, m.bias, m.running_mean, m.running_var, float(m.eps), float(
        m.momentum if m.momentum is not None else _BN_MOMENTUM_DEFAULT)


# ------------------------------------------------------------------------------------------------
# the kernel schedule
# ------------------------------------------------------------------------------------------------
class MMIMDbEngine:
    """Pre-allocated buffers for one batch size and the launch sequence of forward / backward."""

    def __init__(self, model: "MMIMDb", n: int, device: torch.device):
        if n < 2:
            raise L.TspmError("BatchNorm1d in training mode needs more than one sample per batch")
        self.model, self.n, self.dev = model, n, device
        ie, te, gmu, clf = model.image_model, model.text_model, model.fusion_module, model.mm_mlp
        self.di, self.dt = ie.net[0].num_features, te.net[0].num_features
        self.e = ie.net[1].out_features
        self.pool = gmu if model.fusion_type == "pooling" else None
        if self.pool is not None:
            if te.net[1].out_features != self.e or self.pool.proj_a.in_features != self.e:
                raise L.TspmError("MMIMDb HIP engine: both encoders must share one width")
            self.d = self.pool.output_dim
            self.hd = self.pool.hidden_dim
            self.pool_p = float(self.pool.dropout)
        else:
            if te.net[1].out_features != self.e or gmu.fc_one.in_features != self.e or gmu.fc_two.in_features != self.e:
                raise L.TspmError("MMIMDb HIP engine: both encoders and the GMU inputs must share one width")
            self.d = gmu.fc_one.out_features
            if gmu.fc_two.out_features != self.d or gmu.use_bias:
                raise L.TspmError("MMIMDb HIP engine: GMU outputs must match and carry no bias")
        if clf.input_size != self.d:
            raise L.TspmError("MMIMDb HIP engine: classifier input_size must equal the GMU output width")
        self.h, self.c = clf.hidden_size, clf.output_size
        for mo in (clf.net[1], clf.net[4]):
            if mo.num_units != 2 or mo.use_bias:
                raise L.TspmError("MMIMDb HIP engine: MaxOut with 2 units and no bias (models/mmimdb.py:40-44)")
        self.p = float(clf.net[2].p)
        if abs(self.p - float(clf.net[5].p)) > 0 or not 0.0 <= self.p < 1.0:
            raise L.TspmError("MMIMDb HIP engine: both dropouts must share p < 1")
        for c in (self.di, self.dt, self.d, self.h):
            if c % 4:
                raise L.TspmError("MMIMDb HIP engine: feature widths must be multiples of 4")
        f = dict(device=device, dtype=torch.float32)
        e, d, h, c = self.e, self.d, self.h, self.c
        z = lambda *s: torch.zeros(*s, **f)
        self.I, self.T, self.labels = z(n, self.di), z(n, self.dt), z(n, c)
        self.XnI, self.XnT, self.EI, self.ET = z(n, self.di), z(n, self.dt), z(n, e), z(n, e)
        self.U, self.H, self.gate, self.Z, self.Zn = z(n, 2 * d), z(n, 2 * d), z(n), z(n, d), z(n, d)
        self.A1, self.Y1, self.Y1n = z(n, 2 * h), z(n, h), z(n, h)
        self.A2, self.Y2, self.Y2n = z(n, 2 * h), z(n, h), z(n, h)
        self.logits, self.loss, self.dlogits = z(n, c), z(1), z(n, c)
        self.dY2n, self.dY2, self.dA2, self.dY1n, self.dY1, self.dA1 = z(n, h), z(n, h), z(n, 2 * h), z(n, h), \
            z(n, h), z(n, 2 * h)
        self.dZn, self.dZ, self.dU, self.ds = z(n, d), z(n, d), z(n, 2 * d), z(n)
        self.dEI, self.dET = z(n, e), z(n, e)
        if self.pool is not None:  # U = [proj_a | proj_b], TU = tanh(U), H = dropout(TU) = [a | b]
            hd = self.hd
            self.TU, self.Hpre, self.Hh, self.wts = z(n, 2 * d), z(n, hd), z(n, hd), z(n, 2)
            self.dAB2, self.dS, self.dHpre = z(n, 2 * d), z(n, 2), z(n, hd)
            self.keep_pool = torch.ones(n, 2 * d, dtype=torch.uint8, device=device)
            self.pool_keep_override: Optional[torch.Tensor] = None
        self.dXn, self.dXnT = z(n, self.di), z(n, self.dt)
        # one stream: the text branch on a side stream measured 0.4385 vs 0.4278 ms at batch 256, 0.373 vs
        # 0.365 at 128, 0.859 vs 0.876 at 1024 — the two stream edges cost about what the overlap saves
        self.side = None
        self.keep = torch.ones(2, n, h, dtype=torch.uint8, device=device)
        widths = (self.di, self.dt, d, h)
        self.stat = {k: (z(w), z(w)) for k, w in zip(("i", "t", "b0", "b1", "b2"), widths + (h,))}
        self.stats = z(3 + 3 * c)
        # split-K for the long encoder Linear when its output tiles cannot fill the chip
        self.enc_splits = 4
        tiles = -(-n // 32) * -(-e // 32)
        if self.di < 2048 or tiles >= 256:
            self.enc_splits = 1
        wsb = L.lib().tspm_linear_fwd_splitk_workspace(n, self.di, e, self.enc_splits) if self.enc_splits > 1 else 0
        self.ws = torch.zeros(max(int(wsb) // 4, 4), **f)
        self.ws_bytes = self.ws.numel() * 4
        self.keep_override: Optional[torch.Tensor] = None
        self.rng_ctr_ptr: Optional[int] = None

    @staticmethod
    def _adjacent(mo: MaxOut) -> bool:
        w0, w1 = mo.layers[0].weight, mo.layers[1].weight
        return w0.is_contiguous() and w1.is_contiguous() and w1.data_ptr() == w0.data_ptr() + w0.numel() * 4

    def check_maxout_weights(self) -> None:
        """The backward writes both MaxOut units' weight gradients with ONE product: weights and
        gradients must be adjacent (FusedAdam's flat buffers)."""
        for mo in (self.model.mm_mlp.net[1], self.model.mm_mlp.net[4]):
            if not self._adjacent(mo):
                raise L.TspmError("MaxOut units' weights must be adjacent (create FusedAdam over the model's "
                                  "parameters before the first step)")
            w0, w1 = mo.layers[0].weight, mo.layers[1].weight
            g0, g1 = w0.grad, w1.grad
            if g0 is not None and (g1 is None or g1.data_ptr() != g0.data_ptr() + g0.numel() * 4):
                raise L.TspmError("MaxOut units' gradients must be adjacent (FusedAdam's flat gradient buffer)")

    # -- helpers ------------------------------------------------------------------------------------
    def _fork(self) -> int:
        if self.side is None:
            return L.stream_handle()
        self.side.wait_stream(torch.cuda.current_stream())
        return self.side.cuda_stream

    def _join(self) -> None:
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)

    def _bn_train(self, key, bn, x, width, out, sh):
        g, b, rm, rv, eps, mom = _bn(bn)
        mean, inv = self.stat[key]
        L.check(L.lib().tspm_bn1d_fwd(self.n, width, x.data_ptr(), g.data_ptr(), b.data_ptr(), rm.data_ptr(),
                                      rv.data_ptr(), mom, eps, mean.data_ptr(), inv.data_ptr(), out.data_ptr(), sh),
                "bn1d_fwd")

    @staticmethod
    def _linear_bwd_multi(items, sh) -> None:
        """items: (n, in, out, x, ldx, dy_ptr, ldy, weight, bias, dx, lddx) per Linear — one
        tspm_linear_bwd_multi launch (bitwise the separate tspm_linear_bwd launches)."""
        descs = (L.LinearBwdDesc * len(items))()
        for dsc, (n, fin, fout, x, ldx, dy, ldy, w, b, dx, lddx) in zip(descs, items):
            dsc.n, dsc.in_, dsc.out, dsc.ldx, dsc.ldy, dsc.lddx = n, fin, fout, ldx, ldy, lddx
            dsc.x, dsc.dy, dsc.w = x.data_ptr(), dy, w.data_ptr()
            dsc.dw, dsc.db = w.grad.data_ptr(), (b.grad.data_ptr() if b is not None else None)
            dsc.dx = dx.data_ptr() if dx is not None else None
        L.check(L.lib().tspm_linear_bwd_multi(len(items), descs, sh), "linear_bwd_multi")

    def _bn_train_pair(self, a, b, sh):
        args = []
        for key, bn, x, width, out in (a, b):
            g, bb, rm, rv, eps, mom = _bn(bn)
            mean, inv = self.stat[key]
            args += [width, x.data_ptr(), g.data_ptr(), bb.data_ptr(), rm.data_ptr(), rv.data_ptr(), mom, eps,
                     mean.data_ptr(), inv.data_ptr(), out.data_ptr()]
        L.check(L.lib().tspm_bn1d_fwd_pair(self.n, *args, sh), "bn1d_fwd_pair")

    def _bn_eval(self, bn, x, width, out, sh):
        g, b, rm, rv, eps, _ = _bn(bn)
        L.check(L.lib().tspm_bn_apply_eval(self.n, width, x.data_ptr(), rm.data_ptr(), rv.data_ptr(), eps, g.data_ptr(),
                                           b.data_ptr(), 0, None, None, None, None, None, 0, out.data_ptr(), sh),
                "bn_apply_eval")

    def _bn_bwd(self, key, bn, g_in, x, width, dx, sh):
        mean, inv = self.stat[key]
        L.check(L.lib().tspm_bn1d_bwd(self.n, width, g_in.data_ptr(), x.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                      bn.weight.data_ptr(), bn.weight.grad.data_ptr(), bn.bias.grad.data_ptr(),
                                      L.ptr(dx), sh), "bn1d_bwd")

    def _bn_bwd_maxout(self, key, bn, g_in, x, width, A, keep, scale, dA, sh):
        """BatchNorm1d backward, then the backward of the MaxOut(2) + Dropout that produced its input (two
        launches: one fused launch was measured slower, 618k vs 653k samples/s at batch 256 — its 8 workgroups
        took on routing the wide element-wise kernel spreads over the chip; removed in round 5)."""
        dx = self.dY1 if key == "b1" else self.dY2
        self._bn_bwd(key, bn, g_in, x, width, dx, sh)
        L.check(L.lib().tspm_maxout_bwd(self.n, width, dx.data_ptr(), width, A.data_ptr(), 2 * width, keep, scale,
                                        dA.data_ptr(), 2 * width, sh), "maxout bwd")

    # -- forward ------------------------------------------------------------------------------------
    def forward(self, sh: int, train: bool) -> None:
        lib = L.lib()
        m = self.model
        n, e, d, h, c = self.n, self.e, self.d, self.h, self.c
        ie, te, gmu, net = m.image_model.net, m.text_model.net, m.fusion_module, m.mm_mlp.net
        bn_s = (lambda k, mod, x, w, o, st: self._bn_train(k, mod, x, w, o, st)) if train else \
            (lambda k, mod, x, w, o, st: self._bn_eval(mod, x, w, o, st))
        bn = lambda k, mod, x, w, o: bn_s(k, mod, x, w, o, sh)
        # encoders: BatchNorm1d → Linear (models/mmimdb.py:78-93), then the GMU projections into
        # U = [fc_one | fc_two]; the text branch runs on the side stream (joined before the gate)
        pairs = _PAIRS and self.side is None
        if pairs:  # one stream, independent pairs of launches merged (bitwise the separate launches)
            if train:
                self._bn_train_pair(("t", te[0], self.T, self.dt, self.XnT), ("i", ie[0], self.I, self.di, self.XnI),
                                    sh)
            else:
                bn("t", te[0], self.T, self.dt, self.XnT)
                bn("i", ie[0], self.I, self.di, self.XnI)
            L.check(lib.tspm_linear_fwd(n, self.dt, e, self.XnT.data_ptr(), self.dt, te[1].weight.data_ptr(),
                                        te[1].bias.data_ptr(), 0, None, 1.0, self.ET.data_ptr(), e, sh), "text fc")
            L.check(lib.tspm_linear_fwd_splitk(n, self.di, e, self.XnI.data_ptr(), self.di, ie[1].weight.data_ptr(),
                                               ie[1].bias.data_ptr(), 0, None, 1.0, self.EI.data_ptr(), e,
                                               self.enc_splits, self.ws.data_ptr(), self.ws_bytes, sh), "image fc")
            if self.pool is None:
                L.check(lib.tspm_linear_fwd_pair(n, e, d, self.EI.data_ptr(), e, gmu.fc_one.weight.data_ptr(),
                                                 self.U.data_ptr(), 2 * d, self.ET.data_ptr(), e,
                                                 gmu.fc_two.weight.data_ptr(), self.U.data_ptr() + d * 4, 2 * d, sh),
                        "gmu fc_one/fc_two")
        else:
            st = self._fork()
            bn_s("t", te[0], self.T, self.dt, self.XnT, st)
            L.check(lib.tspm_linear_fwd(n, self.dt, e, self.XnT.data_ptr(), self.dt, te[1].weight.data_ptr(),
                                        te[1].bias.data_ptr(), 0, None, 1.0, self.ET.data_ptr(), e, st), "text fc")
            if self.pool is None:
                L.check(lib.tspm_linear_fwd(n, e, d, self.ET.data_ptr(), e, gmu.fc_two.weight.data_ptr(), None, 0,
                                            None, 1.0, self.U.data_ptr() + d * 4, 2 * d, st), "gmu fc_two")
            bn("i", ie[0], self.I, self.di, self.XnI)
            L.check(lib.tspm_linear_fwd_splitk(n, self.di, e, self.XnI.data_ptr(), self.di, ie[1].weight.data_ptr(),
                                               ie[1].bias.data_ptr(), 0, None, 1.0, self.EI.data_ptr(), e,
                                               self.enc_splits, self.ws.data_ptr(), self.ws_bytes, sh), "image fc")
            if self.pool is None:
                L.check(lib.tspm_linear_fwd(n, e, d, self.EI.data_ptr(), e, gmu.fc_one.weight.data_ptr(), None, 0,
                                            None, 1.0, self.U.data_ptr(), 2 * d, sh), "gmu fc_one")
            self._join()
        if self.pool is None:
            L.check(lib.tspm_gmu_fwd(n, d, self.U.data_ptr(), 2 * d, gmu.hidden_sigmoid.weight.data_ptr(),
                                     self.H.data_ptr(), 2 * d, self.gate.data_ptr(), self.Z.data_ptr(), d, sh), "gmu")
        else:
            self._pool_fwd(sh, train)
        # classifier (models/mmimdb.py:38-47)
        keep, k1, k2, scale = None, None, None, 1.0
        # in-launch masks: each MaxOut forward draws its half of the mask tspm_dropout_mask would write
        rng = train and self.p > 0 and self.keep_override is None and _RNG_INLAUNCH
        if train and self.p > 0:
            scale = 1.0 / (1.0 - self.p)
            if self.keep_override is None and not rng:
                L.check(lib.tspm_dropout_mask(2 * n * h, self.p, self.model._rng_seed, self.rng_ctr_ptr,
                                              self.keep.data_ptr(), sh), "dropout_mask")
            k1, k2 = self.keep[0].data_ptr(), self.keep[1].data_ptr()

        def maxout(A, k, Y, unit):
            if rng:
                L.check(lib.tspm_maxout_fwd_rng(n, h, A.data_ptr(), 2 * h, self.p, self.model._rng_seed,
                                                self.rng_ctr_ptr, unit * n * h, k, scale, Y.data_ptr(), h, sh),
                        "maxout+dropout")
            else:
                L.check(lib.tspm_maxout_fwd(n, h, A.data_ptr(), 2 * h, k, scale, Y.data_ptr(), h, sh), "maxout")
        bn("b0", net[0], self.Z, d, self.Zn)
        self._maxout_product(net[1], self.Zn, d, self.A1, sh)
        maxout(self.A1, k1, self.Y1, 0)
        bn("b1", net[3], self.Y1, h, self.Y1n)
        self._maxout_product(net[4], self.Y1n, h, self.A2, sh)
        maxout(self.A2, k2, self.Y2, 1)
        bn("b2", net[6], self.Y2, h, self.Y2n)
        L.check(lib.tspm_linear_fwd(n, h, c, self.Y2n.data_ptr(), h, net[7].weight.data_ptr(), net[7].bias.data_ptr(),
                                    0, None, 1.0, self.logits.data_ptr(), c, sh), "output fc")

    _POOL_SEED_MIX = 0x5DEECE66D  # the pooling dropout's stream, distinct from the classifier's

    def _pool_fwd(self, sh: int, train: bool) -> None:
        """MultimodalPooling (models/pooling.py:81-127): [proj_a | proj_b] (+ biases) → tanh → dropout →
        max / avg / sum, or the attention / gate scoring MLP → softmax / sigmoid mix."""
        lib, pl = L.lib(), self.pool
        n, e, d, hd = self.n, self.e, self.d, self.hd
        L.check(lib.tspm_linear_fwd(n, e, d, self.EI.data_ptr(), e, pl.proj_a.weight.data_ptr(),
                                    pl.proj_a.bias.data_ptr(), 0, None, 1.0, self.U.data_ptr(), 2 * d, sh), "proj_a")
        L.check(lib.tspm_linear_fwd(n, e, d, self.ET.data_ptr(), e, pl.proj_b.weight.data_ptr(),
                                    pl.proj_b.bias.data_ptr(), 0, None, 1.0, self.U.data_ptr() + d * 4, 2 * d, sh),
                "proj_b")
        keep, scale = None, 1.0
        if train and self.pool_p > 0:
            scale = 1.0 / (1.0 - self.pool_p)
            if self.pool_keep_override is None:
                L.check(lib.tspm_dropout_mask(n * 2 * d, self.pool_p,
                                              (self.model._rng_seed ^ self._POOL_SEED_MIX) & ((1 << 63) - 1),
                                              self.rng_ctr_ptr, self.keep_pool.data_ptr(), sh), "pool dropout_mask")
            keep = self.keep_pool.data_ptr()
        L.check(lib.tspm_pool_act_fwd(n, d, self.U.data_ptr(), 2 * d, keep, scale, self.TU.data_ptr(),
                                      self.H.data_ptr(), sh), "pool tanh+dropout")
        kind, sc = pl.kind, pl.scorer()
        if kind >= 3:
            L.check(lib.tspm_linear_fwd(n, 2 * d, hd, self.H.data_ptr(), 2 * d, sc[0].weight.data_ptr(),
                                        sc[0].bias.data_ptr(), 0, None, 1.0, self.Hpre.data_ptr(), hd, sh), "pool score fc")
        L.check(lib.tspm_pool_mix_fwd(n, d, hd, kind, self.H.data_ptr(), self.Hpre.data_ptr(), self.Hh.data_ptr(),
                                      sc[2].weight.data_ptr() if kind >= 3 else None,
                                      sc[2].bias.data_ptr() if kind >= 3 else None, self.wts.data_ptr(),
                                      self.Z.data_ptr(), d, sh), "pool mix")

    def _pool_bwd(self, sh: int) -> None:
        """Backward of _pool_fwd: dZ → d[a | b] (+ the scoring MLP's gradients) → dU."""
        lib, pl = L.lib(), self.pool
        n, d, hd = self.n, self.d, self.hd
        kind, sc = pl.kind, pl.scorer()
        g = lambda p: p.grad.data_ptr()  # noqa: E731
        L.check(lib.tspm_pool_mix_bwd(n, d, hd, kind, self.dZ.data_ptr(), d, self.H.data_ptr(), self.Hh.data_ptr(),
                                      sc[2].weight.data_ptr() if kind >= 3 else None, self.wts.data_ptr(),
                                      self.dU.data_ptr(), self.dS.data_ptr(), self.dHpre.data_ptr(), sh), "pool mix bwd")
        dab2 = None
        if kind >= 3:
            k = 2 if kind == 3 else 1
            L.check(lib.tspm_linear_bwd_weight(n, hd, k, self.Hh.data_ptr(), hd, self.dS.data_ptr(), k,
                                               g(sc[2].weight), g(sc[2].bias), sh), "pool score fc2 dW")
            linear_bwd(n, 2 * d, hd, self.H.data_ptr(), 2 * d, self.dHpre.data_ptr(), hd, sc[0].weight.data_ptr(),
                       g(sc[0].weight), g(sc[0].bias), self.dAB2.data_ptr(), 2 * d, sh)
            dab2 = self.dAB2.data_ptr()
        keep = self.keep_pool.data_ptr() if self.pool_p > 0 else None
        scale = 1.0 / (1.0 - self.pool_p) if self.pool_p > 0 else 1.0
        # dU overwrites the mix gradient in place (same element, read before written)
        L.check(lib.tspm_pool_act_bwd(n, d, self.dU.data_ptr(), dab2, self.TU.data_ptr(), keep, scale,
                                      self.dU.data_ptr(), sh), "pool tanh+dropout bwd")

    def _maxout_product(self, mo: MaxOut, x, width, A, sh) -> None:
        """A[:, :h] = x @ W0^T, A[:, h:] = x @ W1^T — one [2h, in] product when the units' weights are
        adjacent (FusedAdam's flat buffer), else one product per unit into the strided halves."""
        lib, n, h = L.lib(), self.n, self.h
        if self._adjacent(mo):
            L.check(lib.tspm_linear_fwd(n, width, 2 * h, x.data_ptr(), width, mo.layers[0].weight.data_ptr(), None,
                                        0, None, 1.0, A.data_ptr(), 2 * h, sh), "maxout product")
            return
        for u in range(2):
            L.check(lib.tspm_linear_fwd(n, width, h, x.data_ptr(), width, mo.layers[u].weight.data_ptr(), None, 0,
                                        None, 1.0, A.data_ptr() + u * h * 4, 2 * h, sh), "maxout product")

    def loss_fn(self, sh: int, weight: float, with_grad: bool, stats: bool) -> None:
        L.check(L.lib().tspm_bce_logits(self.n, self.c, self.logits.data_ptr(), self.labels.data_ptr(),
                                        self.loss.data_ptr(), self.dlogits.data_ptr() if with_grad else None, weight,
                                        float(self.model.binary_threshold), self.stats.data_ptr() if stats else None,
                                        sh), "bce_with_logits")

    # -- backward -----------------------------------------------------------------------------------
    def backward(self, sh: int) -> None:
        lib = L.lib()
        m = self.model
        n, e, d, h, c = self.n, self.e, self.d, self.h, self.c
        ie, te, gmu, net = m.image_model.net, m.text_model.net, m.fusion_module, m.mm_mlp.net
        scale = 1.0 / (1.0 - self.p) if self.p > 0 else 1.0
        k1 = self.keep[0].data_ptr() if self.p > 0 else None
        k2 = self.keep[1].data_ptr() if self.p > 0 else None
        g = lambda p: p.grad.data_ptr()
        # output Linear
        linear_bwd(n, h, c, self.Y2n.data_ptr(), h, self.dlogits.data_ptr(), c, net[7].weight.data_ptr(),
                   g(net[7].weight), g(net[7].bias), self.dY2n.data_ptr(), h, sh)
        # BatchNorm1d + MaxOut 2 (+ dropout) backward
        self._bn_bwd_maxout("b2", net[6], self.dY2n, self.Y2, h, self.A2, k2, scale, self.dA2, sh)
        linear_bwd(n, h, 2 * h, self.Y1n.data_ptr(), h, self.dA2.data_ptr(), 2 * h, net[4].layers[0].weight.data_ptr(),
                   g(net[4].layers[0].weight), None, self.dY1n.data_ptr(), h, sh)
        # BatchNorm1d + MaxOut 1 (+ dropout) backward
        self._bn_bwd_maxout("b1", net[3], self.dY1n, self.Y1, h, self.A1, k1, scale, self.dA1, sh)
        linear_bwd(n, d, 2 * h, self.Zn.data_ptr(), d, self.dA1.data_ptr(), 2 * h, net[1].layers[0].weight.data_ptr(),
                   g(net[1].layers[0].weight), None, self.dZn.data_ptr(), d, sh)
        self._bn_bwd("b0", net[0], self.dZn, self.Z, d, self.dZ, sh)
        if self.pool is None:  # GMU
            L.check(lib.tspm_gmu_bwd(n, d, self.dZ.data_ptr(), d, self.H.data_ptr(), 2 * d, self.gate.data_ptr(),
                                     gmu.hidden_sigmoid.weight.data_ptr(), self.dU.data_ptr(), 2 * d,
                                     self.ds.data_ptr(), sh), "gmu bwd")
            L.check(lib.tspm_linear_bwd_weight(n, 2 * d, 1, self.H.data_ptr(), 2 * d, self.ds.data_ptr(), 1,
                                               g(gmu.hidden_sigmoid.weight), None, sh), "gmu gate dW")
            fa, fb = gmu.fc_one, gmu.fc_two
        else:
            self._pool_bwd(sh)
            fa, fb = self.pool.proj_a, self.pool.proj_b
        dU1, dU2 = self.dU.data_ptr(), self.dU.data_ptr() + d * 4
        if _PAIRS and self.side is None:
            # fc_two + fc_one (proj_b + proj_a) backward in one launch, then both encoder Linears, then
            # both input BNs
            self._linear_bwd_multi([(n, e, d, self.ET, e, dU2, 2 * d, fb.weight, fb.bias, self.dET, e),
                                    (n, e, d, self.EI, e, dU1, 2 * d, fa.weight, fa.bias, self.dEI, e)], sh)
            self._linear_bwd_multi([(n, self.dt, e, self.XnT, self.dt, self.dET.data_ptr(), e, te[1].weight,
                                     te[1].bias, self.dXnT, self.dt),
                                    (n, self.di, e, self.XnI, self.di, self.dEI.data_ptr(), e, ie[1].weight,
                                     ie[1].bias, self.dXn, self.di)], sh)
            bt, bi = te[0], ie[0]
            (mt, it), (mi, ii) = self.stat["t"], self.stat["i"]
            L.check(lib.tspm_bn1d_bwd_pair(n, self.dt, self.dXnT.data_ptr(), self.T.data_ptr(), mt.data_ptr(),
                                           it.data_ptr(), bt.weight.data_ptr(), g(bt.weight), g(bt.bias), None,
                                           self.di, self.dXn.data_ptr(), self.I.data_ptr(), mi.data_ptr(),
                                           ii.data_ptr(), bi.weight.data_ptr(), g(bi.weight), g(bi.bias), None, sh),
                    "bn1d_bwd_pair")
            return
        st = self._fork()  # text branch (fc_two, text encoder) on the side stream
        for (dUp, fc, E, dE, key, enc, Xn, X, w, dXn, q) in (
                (dU2, fb, self.ET, self.dET, "t", te, self.XnT, self.T, self.dt, self.dXnT, st),
                (dU1, fa, self.EI, self.dEI, "i", ie, self.XnI, self.I, self.di, self.dXn, sh)):
            linear_bwd(n, e, d, E.data_ptr(), e, dUp, 2 * d, fc.weight.data_ptr(), g(fc.weight),
                       g(fc.bias) if fc.bias is not None else None, dE.data_ptr(), e, q)
            # encoder (the BatchNorm1d input-feature gradient is skipped: nothing consumes it)
            linear_bwd(n, w, e, Xn.data_ptr(), w, dE.data_ptr(), e, enc[1].weight.data_ptr(), g(enc[1].weight),
                       g(enc[1].bias), dXn.data_ptr(), w, q)
            self._bn_bwd(key, enc[0], dXn, X, w, None, q)
        self._join()


# ------------------------------------------------------------------------------------------------
# the model
# ------------------------------------------------------------------------------------------------
class MMIMDb(nn.Module):
    """Drop-in for MML_Suite/models/mmimdb.py:96-338 (GMU or multimodal-pooling fusion)."""

    def __init__(self, image_encoder: MMIMDbModalityEncoder, text_encoder: MMIMDbModalityEncoder,
                 gated_bimodal_network: Optional[GatedBiModalNetwork] = None,
                 multimodal_pooling: Optional[Dict[str, Any]] = None, classifier: MLPGenreClassifier = None,
                 binary_threshold: float = 0.5) -> None:
        super().__init__()
        self.image_model = image_encoder
        self.text_model = text_encoder
        if multimodal_pooling is not None:  # built here, after the YAML's modules (models/mmimdb.py:128-141)
            self.fusion_module = MultimodalPooling(
                input_dim_a=image_encoder.net[-1].out_features, input_dim_b=text_encoder.net[-1].out_features,
                output_dim=classifier.input_size, pooling_type=multimodal_pooling.get("pooling_type", "gated"),
                hidden_dim=multimodal_pooling.get("hidden_dim", None), dropout=multimodal_pooling.get("dropout", 0.0))
            self.fusion_type = "pooling"
        elif gated_bimodal_network is not None:
            self.fusion_module = gated_bimodal_network
            self.fusion_type = "gated"
        else:
            raise ValueError("Either gated_bimodal_network or multimodal_pooling must be provided")
        self.mm_mlp = classifier
        self.binary_threshold = binary_threshold
        self.monitor = None
        self._rng_seed = int(torch.initial_seed()) & ((1 << 63) - 1)
        self._steps: Dict[Any, Any] = {}

    def get_encoder(self, modality):
        name = str(getattr(modality, "value", modality)).lower()
        if "image" in name:
            return self.image_model
        if "text" in name:
            return self.text_model
        raise ValueError(f"Invalid modality: {modality}. Must be image or text")

    def logits_transform(self, logits: torch.Tensor):
        return (torch.sigmoid(logits).detach().cpu().numpy() > self.binary_threshold).astype(int)

    def _engine(self, n: int, device) -> MMIMDbEngine:
        key = ("eng", n)
        eng = self._steps.get(key)
        if eng is None:
            eng = MMIMDbEngine(self, n, device)
            self._steps[key] = eng
        return eng

    @torch.no_grad()
    def forward(self, I: torch.Tensor, T: torch.Tensor, *, is_embd_I: bool = False,
                is_embd_T: bool = False) -> torch.Tensor:
        """HIP forward (models/mmimdb.py:164-200).  Training mode uses batch statistics, updates the
        running statistics and draws fresh dropout masks, as the reference's forward does."""
        if is_embd_I or is_embd_T:
            raise NotImplementedError("MMIMDb HIP path: pre-embedded inputs are not on the configs[3] path")
        for t, nm in ((I, "I"), (T, "T")):
            L.require_cuda_f32(t, nm)
        eng = self._engine(I.shape[0], I.device)
        eng.I.copy_(I)
        eng.T.copy_(T)
        sh = L.stream_handle()
        if self.training and eng.rng_ctr_ptr is None:
            eng._host_ctr = torch.zeros(1, dtype=torch.int64, device=I.device)
            eng.rng_ctr_ptr = eng._host_ctr.data_ptr()
        eng.forward(sh, self.training)
        if self.training:
            eng._host_ctr.add_(1)
            nbt = shared_batches_tracked(self, I.device, (nn.BatchNorm1d,))
            L.counters_add(nbt)
        return eng.logits.clone()

    def train_step(self, batch: Dict[str, Any], optimizer, loss_functions, device, metric_recorder=None,
                   epoch: int = 0) -> Dict[str, Any]:
        """models/mmimdb.py:203-245 on the fused HIP step."""
        I, T, labels = _batch_tensors(batch, device)
        key = ("train", id(optimizer), id(loss_functions), I.shape[0])
        st = self._steps.get(key)
        if st is None:
            st = FusedMMIMDbStep(self, optimizer, loss_functions, I.shape[0])
            self._steps[key] = st
        out = st.step(I, T, labels)
        _record(metric_recorder, out["logits"], labels, batch.get("pattern_name"), self.binary_threshold)
        return {"loss": out["loss"].item()}

    @torch.no_grad()
    def validation_step(self, batch: Dict[str, Any], loss_functions, device, metric_recorder=None,
                        return_test_info: bool = False, epoch: int = None) -> Dict[str, Any]:
        """models/mmimdb.py:247-290: eval-mode forward + BCE on the HIP kernels."""
        self.eval()
        I, T, labels = _batch_tensors(batch, device)
        eng = self._engine(I.shape[0], I.device)
        eng.I.copy_(I)
        eng.T.copy_(T)
        eng.labels.copy_(labels)
        sh = L.stream_handle()
        eng.forward(sh, False)
        eng.loss_fn(sh, _bce_weight(loss_functions), False, False)
        _record(metric_recorder, eng.logits, labels, batch.get("pattern_name"), self.binary_threshold)
        return {"loss": eng.loss.item()}


def _batch_tensors(batch, device):
    def get(name):
        for k, v in batch.items():
            if str(getattr(k, "value", k)).lower() == name:
                return v
        raise KeyError(name)
    I = get("image").to(device, non_blocking=True).float()
    T = get("text").to(device, non_blocking=True).float()
    labels = get("label").to(device, non_blocking=True).float()
    return I, T, labels


def _record(rec, logits, labels, patterns, threshold):
    if rec is None or not hasattr(rec, "update_group_all"):
        return
    import numpy as np
    preds = (torch.sigmoid(logits).detach().cpu().numpy() > threshold).astype(int)
    rec.update_group_all("classification", predictions=preds, targets=labels.detach().cpu().numpy(),
                         m_types=np.array(patterns if patterns is not None else ["it"] * len(preds)))


class FusedMMIMDbStep:
    """One MMIMDb train step (zero_grad-free: the backward overwrites every gradient) — forward, BCE,
    backward and Adam — as one HIP graph replayed per batch (captured on the second call)."""

    def __init__(self, model: MMIMDb, optimizer: FusedAdam, loss_functions, batch: int, use_graph: bool = True,
                 allreduce=None):
        if not isinstance(optimizer, FusedAdam):
            raise L.TspmError("FusedMMIMDbStep needs FusedAdam (the flat gradient buffer the kernels write)")
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise L.TspmError("FusedMMIMDbStep runs on the MI355X: move the model to cuda first")
        self.model, self.opt, self.N = model, optimizer, batch
        self.weight = _bce_weight(loss_functions)
        self.eng = MMIMDbEngine(model, batch, dev)
        self.eng.check_maxout_weights()
        fgs = optimizer.flat_groups()
        self.eng.rng_ctr_ptr = fgs[0].hyper.data_ptr() + L.HYPER_STEP_OFFSET
        self.nbt = shared_batches_tracked(model, dev, (nn.BatchNorm1d,))
        self.use_graph, self.allreduce = use_graph, allreduce
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.calls = 0
        self.log_stats = False

    @property
    def keep_override(self):
        return self.eng.keep_override

    @keep_override.setter
    def keep_override(self, v):
        self.eng.keep_override = v

    def _fwd_bwd(self) -> None:
        sh = L.stream_handle()
        self.eng.forward(sh, True)
        self.eng.loss_fn(sh, self.weight, True, self.log_stats)
        self.eng.backward(sh)
        L.counters_add(self.nbt)

    def _all(self) -> None:
        self._fwd_bwd()
        if self.allreduce is None:
            self.opt.launch(L.stream_handle())

    def step(self, I: torch.Tensor, T: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
        e = self.eng
        e.I.copy_(I, non_blocking=True)
        e.T.copy_(T, non_blocking=True)
        e.labels.copy_(labels, non_blocking=True)
        self.run()
        return {"loss": e.loss, "logits": e.logits}

    def run(self) -> None:
        self.model.train()
        self.opt.sync_hyper()
        if self.eng.keep_override is not None:
            self.eng.keep.copy_(self.eng.keep_override.reshape(self.eng.keep.shape).to(torch.uint8), non_blocking=True)
        if self.eng.pool is not None and self.eng.pool_keep_override is not None:
            self.eng.keep_pool.copy_(self.eng.pool_keep_override.reshape(self.eng.keep_pool.shape).to(torch.uint8),
                                     non_blocking=True)
        if not self.use_graph or self.calls == 0:
            self._all()
        else:
            if self.graph is None:
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with L.graph_capture(g):
                    self._all()
                self.graph = g
            self.graph.replay()
        if self.allreduce is not None:
            self.allreduce()
            self.opt.launch(L.stream_handle())
        self.opt.note_steps(1)
        self.calls += 1


def f1_metrics(stats: torch.Tensor, classes: int) -> Dict[str, float]:
    """f1_samples / f1_macro / f1_weighted / f1_micro (sklearn.metrics.f1_score, zero_division=0, as
    configured in mmimdb_baseline.yaml) from the counts tspm_bce_logits accumulates."""
    s = stats.detach().double().cpu()
    n = max(float(s[1]), 1.0)
    tp, fp, fn = s[3::3][:classes], s[4::3][:classes], s[5::3][:classes]
    den = 2 * tp + fp + fn
    f1k = torch.where(den > 0, 2 * tp / den.clamp(min=1e-300), torch.zeros_like(den))
    sup = tp + fn
    micro_den = float(2 * tp.sum() + fp.sum() + fn.sum())
    return {"loss": float(s[0]) / n, "f1_samples": float(s[2]) / n, "f1_macro": float(f1k.mean()),
            "f1_weighted": float((f1k * sup).sum() / sup.sum()) if float(sup.sum()) > 0 else 0.0,
            "f1_micro": float(2 * tp.sum()) / micro_den if micro_den > 0 else 0.0}


# ------------------------------------------------------------------------------------------------
# input stage + epoch harness
# ------------------------------------------------------------------------------------------------
PATTERNS = {"it": (1.0, 1.0), "i": (1.0, 0.0), "t": (0.0, 1.0)}  # (image, text) presence


def synthetic_features(n: int, seed: int = 1234, image_dim: int = 4096, text_dim: int = 300, genres: int = 23):
    """MM-IMDb-shaped synthetic features for benches (no dataset in the image): VGG16 fc7-like image
    features (ReLU output, non-negative), mean-word2vec-like text features, and multi-hot genre labels with
    at least one genre per movie (MML_Suite/data/mmimdb.py:122-200 shapes).  CPU tensors, seeded."""
    g = torch.Generator().manual_seed(seed)
    image = torch.relu(torch.randn(n, image_dim, generator=g))
    text = 0.1 * torch.randn(n, text_dim, generator=g)
    labels = (torch.rand(n, genres, generator=g) < 0.15).float()
    labels[torch.arange(n), torch.randint(0, genres, (n,), generator=g)] = 1.0
    return image, text, labels


class MMIMDbCorpus:
    """HBM-resident MM-IMDb features (replaces the per-sample HDF5 reads + collate of
    MML_Suite/data/mmimdb.py:122-200 and the step's ``.to(device)``; the HDF5 file itself needs h5py,
    which this image lacks — construct from arrays, e.g. exported once with the reference's reader).
    ``gather`` assembles a batch on device with the input-stage kernel (``tspm_avmnist_gather`` used
    as a generic row gather: one launch per tensor, the missing-modality pattern as a row mask)."""

    def __init__(self, image, text, labels, device):
        t = lambda a: torch.as_tensor(a, dtype=torch.float32).contiguous().to(device)
        self.image, self.text, self.labels = t(image), t(text), t(labels)
        self.n = self.image.shape[0]
        if self.text.shape[0] != self.n or self.labels.shape[0] != self.n:
            raise L.TspmError("MMIMDbCorpus: image / text / labels row counts differ")
        self.device = device
        self._masks: Dict[int, Dict[str, torch.Tensor]] = {}

    def _mask(self, n: int, pattern: str):
        if pattern == "it":
            return None, None
        m = self._masks.setdefault(n, {})
        if pattern not in m:
            ip, tp = PATTERNS[pattern]
            m[pattern] = (torch.full((n,), ip, device=self.device), torch.full((n,), tp, device=self.device))
        return m[pattern]

    def gather(self, index: torch.Tensor, I_out, T_out, Y_out, pattern: str = "it", row_masks=None) -> None:
        """Rows ``index`` into the step's buffers; the absent modality of ``pattern`` zeroed, or per row
        with ``row_masks`` = (image presence [n], text presence [n]) float tensors."""
        lib, sh, n = L.lib(), L.stream_handle(), index.numel()
        im, tm = self._mask(n, pattern) if row_masks is None else row_masks
        for src, w, mask, out in ((self.image, self.image.shape[1], im, I_out), (self.text, self.text.shape[1], tm, T_out),
                                  (self.labels, self.labels.shape[1], None, Y_out)):
            L.check(lib.tspm_avmnist_gather(n, index.data_ptr(), self.n, src.data_ptr(), w, None, 0, None, None,
                                            L.ptr(mask), None, out.data_ptr(), None, None, sh), "mmimdb gather")


def _evaluate(model: MMIMDb, corpus: MMIMDbCorpus, batch: int, weight: float, pattern: str) -> Dict[str, float]:
    """Metrics of one missing-data pattern over the whole validation corpus (eval mode: BatchNorm
    running statistics, so a one-row last batch is valid, as in the reference)."""
    model.eval()
    sh = L.stream_handle()
    stats = None
    for s in range(0, corpus.n, batch):
        idx = torch.arange(s, min(s + batch, corpus.n), device=corpus.device)
        eng = model._engine(idx.numel(), corpus.device)
        if stats is None:
            stats = torch.zeros_like(eng.stats)
        eng.stats.zero_()
        corpus.gather(idx, eng.I, eng.T, eng.labels, pattern)
        eng.forward(sh, False)
        eng.loss_fn(sh, weight, False, True)
        stats += eng.stats
    return f1_metrics(stats, model.mm_mlp.output_size)


def validation_loss(model: MMIMDb, corpus: MMIMDbCorpus, batch: int, weight: float, patterns=("it", "i", "t"),
                    generator: Optional[torch.Generator] = None) -> float:
    """The loss train_multimodal.py monitors (save_metric "loss", :494-541,750-758): the mean of the
    per-batch losses over the validation loader, whose dataset holds every sample once per selected
    pattern (len = N x #patterns, item k -> pattern k // N: data/base_dataset.py:89-92) and which
    shuffles (mmimdb_baseline.yaml: shuffle true — the permutation here is seeded, not the reference's
    RNG draws).  Batches mix patterns; the absent modality is zeroed per row."""
    model.eval()
    sh = L.stream_handle()
    n, P = corpus.n, len(patterns)
    order = torch.randperm(n * P, generator=generator) if generator is not None else torch.arange(n * P)
    pres = torch.tensor([PATTERNS[p] for p in patterns], dtype=torch.float32)
    losses = []
    for s in range(0, n * P, batch):
        ks = order[s:s + batch]
        idx, pid = (ks % n).to(corpus.device), ks // n
        im, tm = pres[pid, 0].to(corpus.device), pres[pid, 1].to(corpus.device)
        eng = model._engine(ks.numel(), corpus.device)
        corpus.gather(idx, eng.I, eng.T, eng.labels, row_masks=(im, tm))
        eng.forward(sh, False)
        eng.loss_fn(sh, weight, False, False)
        losses.append(eng.loss.clone())
    # one host read for the epoch; np.mean of the per-batch fp32 losses as the reference computes it
    import numpy as np
    return float(np.mean([float(v) for v in torch.cat(losses).cpu()]))


def fit_mmimdb(model: MMIMDb, optimizer: FusedAdam, train: MMIMDbCorpus, val: MMIMDbCorpus, batch: int,
               epochs: int, loss_functions=None, patience: int = 25, seed: int = 0,
               patterns=("it", "i", "t"), min_delta: float = 1e-3, checkpoint_dir=None,
               scheduler=None) -> List[Dict[str, Any]]:
    """The epoch loop of train_multimodal.py for the MMIMDb config, every batch on the HIP path:
    shuffled train batches over every sample (the DataLoader's drop_last=False, config/data_config.py:121;
    a last batch of one row is skipped — BatchNorm1d in training mode rejects it in the reference too),
    the validation loss over all selected patterns together (``validation_loss``), per-pattern
    validation metrics with the absent modality zeroed, early stopping on that loss with the
    reference's check (harness.check_early_stopping: patience 25 from the YAML, min_delta 1e-3 =
    TrainingConfig.early_stopping_min_delta), ``epoch_{n}.pth`` / ``best.pth`` through
    harness.CheckpointManager on improvement, and ReduceLROnPlateau on the validation loss.
    Returns one dict per epoch: train loss / f1s, ``val_loss`` and ``val_{pattern}`` metrics."""
    from .harness import CheckpointManager, check_early_stopping
    weight = _bce_weight(loss_functions)
    steps: Dict[int, FusedMMIMDbStep] = {}

    def step_for(n):
        st = steps.get(n)
        if st is None:
            st = FusedMMIMDbStep(model, optimizer, loss_functions, n)
            st.log_stats = True
            steps[n] = st
        return st
    main = step_for(batch)
    gen = torch.Generator(device="cpu").manual_seed(seed)
    vgen = torch.Generator(device="cpu").manual_seed(seed + 1)
    ckpt = CheckpointManager(checkpoint_dir) if checkpoint_dir is not None else None
    history, best, wait = [], None, 0
    for ep in range(1, epochs + 1):
        model.train()
        for st in steps.values():
            st.eng.stats.zero_()
        perm = torch.randperm(train.n, generator=gen).to(train.device)
        for s in range(0, train.n, batch):
            rows = perm[s:s + batch]
            if rows.numel() < 2:
                break
            st = step_for(rows.numel())
            train.gather(rows, st.eng.I, st.eng.T, st.eng.labels)
            st.run()
        tot = main.eng.stats.clone()
        for n, st in steps.items():
            if n != batch:
                tot += st.eng.stats
        rec = {"epoch": ep, "train": f1_metrics(tot, model.mm_mlp.output_size),
               "val_loss": validation_loss(model, val, batch, weight, patterns, vgen)}
        for p in patterns:
            rec[f"val_{p}"] = _evaluate(model, val, batch, weight, p)
        history.append(rec)
        vm = {"loss": rec["val_loss"]}
        is_best, cont, wait = check_early_stopping(vm, best, patience, min_delta, wait)
        if is_best:
            best = dict(vm)
            if ckpt is not None:
                ckpt.save_checkpoint(model, optimizer, scheduler, ep, vm, is_best=True)
        if not cont:
            break
        if scheduler is not None:
            scheduler.step(rec["val_loss"])
    return history
