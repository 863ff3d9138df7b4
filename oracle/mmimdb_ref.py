"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's MMIMDb late-fusion train step
(BASELINE configs[3]).  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path never does.

Restates, with plain ``torch.nn`` / ``torch.nn.functional`` on the CPU:
  * ``MMIMDbModalityEncoder``  = BatchNorm1d(in) → Linear(in, out)          (MML_Suite/models/mmimdb.py:63-93)
  * ``GatedBiModalNetwork``    = tanh(fc_one), tanh(fc_two), sigmoid(hidden_sigmoid(cat)),
                                 g*h1 + (1-g)*h2, no biases                    (models/gates/gated_bimodal.py)
  * ``MLPGenreClassifier``     = BN → MaxOut(2, no bias) → Dropout(.5) → BN → MaxOut → Dropout → BN → Linear
                                                                               (models/mmimdb.py:20-60, models/maxout.py)
  * ``MultimodalPooling``     = proj_a/proj_b → tanh → dropout, max/avg/sum/attention/gated pooling
                                                                               (models/pooling.py:6-127)
  * ``MMIMDb.forward`` / ``train_step``: BCEWithLogits(mean) × weight 1.0, Adam (lr 1e-5, wd 1e-3)
                                                                               (models/mmimdb.py:164-245,
                                                                                configs/mmimdb/centralised/mmimdb_baseline.yaml)
Module attribute names follow the reference so ``state_dict`` keys are identical; construction order
(image encoder, text encoder, GMU, classifier) follows the YAML, so ``torch.manual_seed(s)`` before
construction reproduces the reference's initial weights.  Dropout takes explicit keep masks.

Pinned: ``tests/golden/mmimdb_step_b4.npz`` was produced by the REAL reference modules imported in the
build container (``tests/golden/make_mmimdb_golden.py``); ``tests/test_oracle_golden.py`` checks this
restatement against it.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn.functional as F
from torch import nn

IMAGE_DIM, TEXT_DIM, EMBED, HIDDEN, GENRES = 4096, 300, 512, 512, 23


class OracleMaxOut(nn.Module):
    def __init__(self, i: int, o: int, units: int = 2, bias: bool = False):
        super().__init__()
        self.layers = nn.ModuleList([nn.Linear(i, o, bias=bias) for _ in range(units)])

    def forward(self, x, trace: Optional["MaxOutTrace"] = None, site: str = ""):
        if trace is not None:
            return trace.maxout(site, self.layers[0](x), self.layers[1](x))
        y = self.layers[0](x)
        for l in self.layers[1:]:
            y = torch.max(y, l(x))
        return y


class MaxOutTrace:
    """Parity instrument (test infrastructure): records both MaxOut units' outputs per site
    (``mo1``, ``mo2``) and, in force mode, replaces the element-wise choice by a given one
    (0 = unit 0, 1 = unit 1, 2 = tie: value and gradient split half/half, as torch.max's derivative
    does for equal inputs) — the fp64 oracle then follows the fp32 implementation's decisions."""

    def __init__(self, force: Optional[Dict[str, torch.Tensor]] = None):
        self.force = force
        self.units: Dict[str, tuple] = {}

    def maxout(self, site: str, a0: torch.Tensor, a1: torch.Tensor) -> torch.Tensor:
        self.units[site] = (a0.detach(), a1.detach())
        if self.force is None or site not in self.force:
            return torch.max(a0, a1)
        c = self.force[site].to(a0.device)
        return torch.where(c == 1, a1, torch.where(c == 0, a0, 0.5 * (a0 + a1)))


class OracleEncoder(nn.Module):
    def __init__(self, i: int, o: int):
        super().__init__()
        self.net = nn.Sequential(nn.BatchNorm1d(i), nn.Linear(i, o))

    def forward(self, x):
        return self.net(x)


class OracleGMU(nn.Module):
    def __init__(self, d1: int, d2: int, o1: int, o2: int):
        super().__init__()
        self.fc_one = nn.Linear(d1, o1, bias=False)
        self.fc_two = nn.Linear(d2, o2, bias=False)
        self.hidden_sigmoid = nn.Linear(o1 + o2, 1, bias=False)

    def forward(self, a, b):
        h1 = torch.tanh(self.fc_one(a))
        h2 = torch.tanh(self.fc_two(b))
        g = torch.sigmoid(self.hidden_sigmoid(torch.cat([h1, h2], dim=1)))
        return g.view(g.size(0), 1) * h1 + (1 - g).view(g.size(0), 1) * h2


class OracleMultimodalPooling(nn.Module):
    """models/pooling.py:6-127 (MultimodalPooling): proj_a / proj_b → tanh → dropout (one module, two
    independent draws), then max / avg / sum / attention (Linear → tanh → Linear(·, 2) → softmax) /
    gated (Linear → tanh → Linear(·, 1) → sigmoid) pooling.  Module names, construction order and
    state_dict keys as the reference's."""

    def __init__(self, da: int, db: int, out: int, pooling_type: str = "gated", hidden_dim: Optional[int] = None,
                 dropout: float = 0.0):
        super().__init__()
        self.pooling_type = pooling_type.lower()
        self.hidden_dim = hidden_dim or max(da, db)
        self.dropout = dropout
        self.proj_a = nn.Linear(da, out)
        self.proj_b = nn.Linear(db, out)
        self.dropout_layer = nn.Dropout(dropout) if dropout > 0 else nn.Identity()
        self.activation = nn.Tanh()
        if self.pooling_type == "attention":
            self.attention_layer = nn.Sequential(nn.Linear(out * 2, self.hidden_dim), nn.Tanh(),
                                                 nn.Linear(self.hidden_dim, 2), nn.Softmax(dim=1))
        elif self.pooling_type == "gated":
            self.gate_layer = nn.Sequential(nn.Linear(out * 2, self.hidden_dim), nn.Tanh(),
                                            nn.Linear(self.hidden_dim, 1), nn.Sigmoid())

    def forward(self, x_a, x_b, keep_a=None, keep_b=None, trace=None):
        a = self.activation(self.proj_a(x_a))
        b = self.activation(self.proj_b(x_b))
        if self.training and self.dropout > 0:
            if keep_a is None:
                a, b = self.dropout_layer(a), self.dropout_layer(b)
            else:
                s = 1.0 / (1.0 - self.dropout)
                a = a * (keep_a.to(a.dtype) * s)
                b = b * (keep_b.to(b.dtype) * s)
        t = self.pooling_type
        if t == "max":
            return trace.maxout("pool", a, b) if trace is not None else torch.max(a, b)
        if t in ("avg", "average"):
            return (a + b) / 2
        if t == "sum":
            return a + b
        combined = torch.cat([a, b], dim=1)
        if t == "attention":
            s = self.attention_layer(combined)
            return s[:, 0].unsqueeze(1).expand_as(a) * a + s[:, 1].unsqueeze(1).expand_as(b) * b
        if t == "gated":
            g = self.gate_layer(combined)
            return g * a + (1 - g) * b
        raise ValueError(f"Unknown pooling type: {t}")


class OracleClassifier(nn.Module):
    def __init__(self, i: int, o: int, h: int):
        super().__init__()
        self.net = nn.Sequential(nn.BatchNorm1d(i), OracleMaxOut(i, h), nn.Dropout(0.5), nn.BatchNorm1d(h),
                                 OracleMaxOut(h, h), nn.Dropout(0.5), nn.BatchNorm1d(h), nn.Linear(h, o))

    def forward(self, x, keep1=None, keep2=None, trace=None):
        n = self.net
        x = n[1](n[0](x), trace, "mo1")
        x = _dropout(x, keep1, self.training)
        x = n[4](n[3](x), trace, "mo2")
        x = _dropout(x, keep2, self.training)
        return n[7](n[6](x))


def _dropout(x, keep, training):
    if not training:
        return x
    if keep is None:
        return F.dropout(x, 0.5, True)
    return x * (keep.to(x.dtype) * 2.0)  # ATen: input * (bernoulli(1-p) / (1-p))


class OracleMMIMDb(nn.Module):
    """``pooling`` (the YAML's ``multimodal_pooling`` dict) replaces the GMU: the reference builds the
    encoders and the classifier from the YAML first and MultimodalPooling inside MMIMDb.__init__
    (models/mmimdb.py:128-141), which is the seeded construction order reproduced here."""

    def __init__(self, image_dim=IMAGE_DIM, text_dim=TEXT_DIM, embed=EMBED, hidden=HIDDEN, genres=GENRES,
                 pooling: Optional[Dict] = None):
        super().__init__()
        self.image_model = OracleEncoder(image_dim, embed)
        self.text_model = OracleEncoder(text_dim, embed)
        if pooling is None:
            self.fusion_module = OracleGMU(embed, embed, embed, embed)
            self.mm_mlp = OracleClassifier(embed, genres, hidden)
            self.fusion_type = "gated"
        else:
            clf = OracleClassifier(embed, genres, hidden)
            self.fusion_module = OracleMultimodalPooling(embed, embed, embed, pooling.get("pooling_type", "gated"),
                                                         pooling.get("hidden_dim"), pooling.get("dropout", 0.0))
            self.mm_mlp = clf
            self.fusion_type = "pooling"

    def forward(self, I, T, keep1=None, keep2=None, trace=None, keep_pool=None):
        a, b = self.image_model(I), self.text_model(T)
        if self.fusion_type == "pooling":
            ka, kb = (None, None) if keep_pool is None else keep_pool
            z = self.fusion_module(a, b, ka, kb, trace)
        else:
            z = self.fusion_module(a, b)
        return self.mm_mlp(z, keep1, keep2, trace)


def build_oracle_mmimdb(seed: int = 0, **dims) -> OracleMMIMDb:
    torch.manual_seed(seed)
    return OracleMMIMDb(**dims)


def synthetic_batch(n: int, seed: int = 1234, image_dim=IMAGE_DIM, text_dim=TEXT_DIM, genres=GENRES):
    """MM-IMDb-shaped features: VGG16 fc7 image features (non-negative, ReLU output) and
    mean word2vec text features; multi-hot genre labels with at least one genre per movie."""
    g = torch.Generator().manual_seed(seed)
    image = torch.relu(torch.randn(n, image_dim, generator=g))
    text = 0.1 * torch.randn(n, text_dim, generator=g)
    labels = (torch.rand(n, genres, generator=g) < 0.15).float()
    first = torch.randint(0, genres, (n,), generator=g)
    labels[torch.arange(n), first] = 1.0
    return image, text, labels


def bce_loss(logits, labels):
    return F.binary_cross_entropy_with_logits(logits, labels)


def train_step(model: OracleMMIMDb, opt, image, text, labels, keep1=None, keep2=None,
               trace: Optional[MaxOutTrace] = None, keep_pool=None) -> Dict[str, torch.Tensor]:
    """models/mmimdb.py:203-245 (minus the host metric recorder): zero_grad, forward, BCE, backward, Adam
    (``opt=None``: gradients only)."""
    model.train()
    for p in model.parameters():
        p.grad = None
    logits = model(image, text, keep1, keep2, trace, keep_pool)
    loss = bce_loss(logits, labels)
    loss.backward()
    if opt is not None:
        opt.step()
    return {"loss": loss.detach(), "logits": logits.detach()}


def f1_counts(logits: torch.Tensor, labels: torch.Tensor, threshold: float = 0.5) -> List[float]:
    """The device metric counts of tspm_bce_logits (without the loss slots) restated on the CPU."""
    p = torch.sigmoid(logits) > threshold
    y = labels > 0.5
    tp, fp, fn = (p & y).sum(1), (p & ~y).sum(1), (~p & y).sum(1)
    den = 2 * tp + fp + fn
    f1 = torch.where(den > 0, 2 * tp.double() / den.clamp(min=1), torch.zeros_like(den, dtype=torch.double))
    out = [float(f1.sum())]
    for k in range(logits.shape[1]):
        pk, yk = p[:, k], y[:, k]
        out += [float((pk & yk).sum()), float((pk & ~yk).sum()), float((~pk & yk).sum())]
    return out


def eval_forward(model: OracleMMIMDb, image, text) -> torch.Tensor:
    model.eval()
    with torch.no_grad():
        return model(image, text)
