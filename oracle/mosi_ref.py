"""ORACLE — CPU restatement of the MOSI UTT-Fusion train step (BASELINE configs[4]).  TEST
INFRASTRUCTURE ONLY: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it; the product package never does.

Restates (reference = TArsenii/task-specific-pretraining-multimodal, paths under ``MML_Suite/``):

* ``LSTMEncoder``   models/msa/networks/lstm.py:8-67 — nn.LSTM(input, hidden, batch_first=True), zero
                    initial state, the padded length run in full (no packing), embd "last" = h_n or
                    "maxpool" = F.max_pool1d over the time axis of r_out (lstm.py:47-52)
* ``TextCNN``       models/msa/networks/textcnn.py:10-69 — three nn.Conv2d(1, C, (k, input)), ReLU,
                    max over time, cat, Dropout, Linear + ReLU
* ``FcClassifier``  models/msa/networks/classifier.py:83-117 — (Linear, ReLU, [BatchNorm1d if use_bn,]
                    Dropout) per layer, fc_out
* ``UttFusionModel`` forward / train_step — models/msa/utt_fusion.py:105-200: cat(A, V, T) embeddings →
                    classifier → CE(logits.squeeze(), labels.squeeze()) → backward →
                    clip_grad_norm_(parameters, clip) → Adam
                    (configs/mosi/centralised/utt_fusion_base_training.yaml: hidden 64, 3x128 filters of
                    heights 3/4/5 over 768-d text, classifier 192 → 192/64/32 → 3, dropout 0.5, clip 1.0,
                    Adam lr 1e-3 / wd 1e-3); the MOSEI config (configs/mosei/centralised/
                    utt_fusion_train_mosei.yaml) is ``MOSEI``: 74/35-d inputs, "maxpool" embeddings,
                    TextCNN dropout 0.7, classifier 192 → 96/48 → 3 with use_bn and dropout 0.66, clip 0.5

Module attribute names follow the reference (identical state_dict keys); construction order is the
YAML's (netA, netV, netT, netC), so ``torch.manual_seed(s)`` before construction reproduces the
reference's initial weights.  Dropout takes explicit keep masks; ``MosiTrace`` records or forces the
ReLU and time-max decisions (parity instrument, as avmnist_ref.MaskTrace).

Pinned: ``tests/golden/mosi_step_b4.npz`` and ``mosei_step_b4.npz`` were produced by the REAL reference
modules (``tests/golden/make_mosi_golden.py [mosei]``); ``tests/test_mosi_cpu.py`` checks this restatement
against both.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .avmnist_ref import OracleAdam  # noqa: F401  (torch.optim.Adam's single-tensor update)

AUDIO_DIM, VIDEO_DIM, TEXT_DIM, HIDDEN, FILTERS, HEIGHTS = 5, 20, 768, 64, 128, (3, 4, 5)
CLS_LAYERS, CLASSES = (192, 64, 32), 3


@dataclass(frozen=True)
class UttConfig:
    """The YAML's model block (netA / netV / netT / netC / clip) and its optimizer."""
    audio_dim: int = AUDIO_DIM
    video_dim: int = VIDEO_DIM
    text_dim: int = TEXT_DIM
    embd_method: str = "last"
    text_dropout: float = 0.5
    cls_layers: Tuple[int, ...] = CLS_LAYERS
    cls_dropout: float = 0.5
    use_bn: bool = False
    clip: float = 1.0
    lr: float = 1e-3
    weight_decay: float = 1e-3


# configs/mosi/centralised/utt_fusion_base_training.yaml
MOSI = UttConfig()
# configs/mosei/centralised/utt_fusion_train_mosei.yaml
MOSEI = UttConfig(audio_dim=74, video_dim=35, embd_method="maxpool", text_dropout=0.7, cls_layers=(96, 48),
                  cls_dropout=0.66, use_bn=True, clip=0.5, lr=2e-4, weight_decay=1e-5)


class OracleLSTMEncoder(nn.Module):
    def __init__(self, input_size: int, hidden_size: int, embd_method: str = "last"):
        super().__init__()
        self.input_size, self.hidden_size = input_size, hidden_size
        self.rnn = nn.LSTM(input_size, hidden_size, batch_first=True)
        assert embd_method in ("last", "maxpool")
        self.embd_method = embd_method


class OracleTextCNN(nn.Module):
    def __init__(self, input_size: int, embd_size: int = 128, in_channels: int = 1, out_channels: int = 128,
                 kernel_heights=(3, 4, 5), dropout: float = 0.5):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels, out_channels, (kernel_heights[0], input_size), stride=1, padding=0)
        self.conv2 = nn.Conv2d(in_channels, out_channels, (kernel_heights[1], input_size), stride=1, padding=0)
        self.conv3 = nn.Conv2d(in_channels, out_channels, (kernel_heights[2], input_size), stride=1, padding=0)
        self.dropout = nn.Dropout(dropout)
        self.embd = nn.Sequential(nn.Linear(len(kernel_heights) * out_channels, embd_size), nn.ReLU(inplace=True))
        self.hidden_size = embd_size
        self.p = float(dropout)


class OracleFcClassifier(nn.Module):
    def __init__(self, input_dim: int, layers: List[int], output_dim: int, dropout: float = 0.3,
                 use_bn: bool = False):
        super().__init__()
        mods = []
        for width in layers:
            mods += [nn.Linear(input_dim, width), nn.ReLU()]
            if use_bn:
                mods.append(nn.BatchNorm1d(width))
            if dropout > 0:
                mods.append(nn.Dropout(dropout))
            input_dim = width
        self.module = nn.Sequential(*mods)
        self.fc_out = nn.Linear(layers[-1], output_dim)
        self.p = float(dropout)
        self.widths = list(layers)


class OracleUttFusion(nn.Module):
    def __init__(self, netA, netV, netT, netC, clip: Optional[float] = None):
        super().__init__()
        self.netA, self.netV, self.netT, self.netC = netA, netV, netT, netC
        self.clip = clip


def build_oracle_utt(seed: int = 0, audio_dim=None, video_dim=None, text_dim=None,
                     cfg: UttConfig = MOSI) -> OracleUttFusion:
    torch.manual_seed(seed)
    a = OracleLSTMEncoder(audio_dim or cfg.audio_dim, HIDDEN, cfg.embd_method)
    v = OracleLSTMEncoder(video_dim or cfg.video_dim, HIDDEN, cfg.embd_method)
    t = OracleTextCNN(text_dim or cfg.text_dim, embd_size=HIDDEN, dropout=cfg.text_dropout, in_channels=1,
                      out_channels=FILTERS, kernel_heights=list(HEIGHTS))
    c = OracleFcClassifier(3 * HIDDEN, list(cfg.cls_layers), CLASSES, dropout=cfg.cls_dropout, use_bn=cfg.use_bn)
    return OracleUttFusion(a, v, t, c, clip=cfg.clip)


class MosiTrace:
    """Parity instrument (test infrastructure): records — or, with ``force``, replaces — the ReLU masks
    and time-max argmax decisions of the forward.  Sites: ``text.pool{i}`` (time argmax of conv i, int64
    [B, C]), ``text.relu{i}`` (ReLU of the pooled conv i value, bool [B, C]), ``text.embd`` and
    ``cls.relu{j}`` (bool masks), ``lstm.{a,v}.pool`` (time argmax of the "maxpool" embedding, int64
    [B, H])."""

    def __init__(self, force: Optional[Dict[str, torch.Tensor]] = None):
        self.force = force
        self.pre: Dict[str, torch.Tensor] = {}
        self.idx: Dict[str, torch.Tensor] = {}

    def relu(self, site, x):
        self.pre[site] = x.detach()
        if self.force is None or site not in self.force:
            return F.relu(x)
        return x * self.force[site].to(device=x.device, dtype=x.dtype)

    def time_max(self, i, conv):  # conv [B, C, Tout] before the ReLU
        site_p, site_r = f"text.pool{i}", f"text.relu{i}"
        act = F.relu(conv)
        _, idx = F.max_pool1d(act, act.size(2), return_indices=True)
        self.pre[site_p] = conv.detach()
        self.idx[site_p] = idx.squeeze(2)
        if self.force is None or site_p not in self.force:
            return F.max_pool1d(act, act.size(2)).squeeze(2)
        at = conv.gather(2, self.force[site_p].to(conv.device).unsqueeze(2)).squeeze(2)
        self.pre[site_r] = at.detach()
        return at * self.force[site_r].to(device=at.device, dtype=at.dtype)


    def lstm_max(self, site, r_out):  # r_out [B, T, H]
        in_feat = r_out.transpose(1, 2)
        _, idx = F.max_pool1d(in_feat, in_feat.size(2), in_feat.size(2), return_indices=True)
        self.pre[site] = r_out.detach()
        self.idx[site] = idx.squeeze(2)
        if self.force is None or site not in self.force:
            return F.max_pool1d(in_feat, in_feat.size(2), in_feat.size(2)).squeeze(-1)
        return in_feat.gather(2, self.force[site].to(r_out.device).unsqueeze(2)).squeeze(2)


def lstm_forward(enc: OracleLSTMEncoder, x: torch.Tensor, trace: Optional[MosiTrace] = None,
                 site: str = "lstm") -> torch.Tensor:
    r_out, (h_n, _) = enc.rnn(x)
    if enc.embd_method == "last":
        return h_n.squeeze(0)
    if trace is not None:
        return trace.lstm_max(site, r_out)
    in_feat = r_out.transpose(1, 2)  # lstm.py:47-52
    return F.max_pool1d(in_feat, in_feat.size(2), in_feat.size(2)).squeeze(-1)


def textcnn_forward(net: OracleTextCNN, x: torch.Tensor, training: bool, keep: Optional[torch.Tensor],
                    trace: Optional[MosiTrace] = None) -> torch.Tensor:
    b, t, f = x.shape
    x4 = x.view(b, 1, t, f)
    outs = []
    for i, conv in enumerate((net.conv1, net.conv2, net.conv3)):
        y = F.conv2d(x4, conv.weight, conv.bias).squeeze(3)  # [B, C, Tout]
        if trace is None:
            act = F.relu(y)
            outs.append(F.max_pool1d(act, act.size(2)).squeeze(2))
        else:
            outs.append(trace.time_max(i, y))
    h = torch.cat(outs, 1)
    if training and net.p > 0:
        h = h * (keep.to(h.dtype) / (1.0 - net.p)) if keep is not None else F.dropout(h, net.p, True)
    z = F.linear(h, net.embd[0].weight, net.embd[0].bias)
    return F.relu(z) if trace is None else trace.relu("text.embd", z)


def classifier_forward(net: OracleFcClassifier, x: torch.Tensor, training: bool,
                       keeps: Optional[List[torch.Tensor]], trace: Optional[MosiTrace] = None) -> torch.Tensor:
    lin = [m for m in net.module if isinstance(m, nn.Linear)]
    bns = [m for m in net.module if isinstance(m, nn.BatchNorm1d)]
    for j, l in enumerate(lin):
        z = F.linear(x, l.weight, l.bias)
        x = F.relu(z) if trace is None else trace.relu(f"cls.relu{j}", z)
        if bns:
            x = bns[j](x)  # the module: batch statistics + running-stat update in train mode
        if training and net.p > 0:
            x = x * (keeps[j].to(x.dtype) / (1.0 - net.p)) if keeps is not None else F.dropout(x, net.p, True)
    return F.linear(x, net.fc_out.weight, net.fc_out.bias)


def forward(model: OracleUttFusion, A, V, T, training: bool, keeps: Optional[Dict[str, torch.Tensor]] = None,
            trace: Optional[MosiTrace] = None) -> torch.Tensor:
    """models/msa/utt_fusion.py:105-140 (all three modalities present)."""
    keeps = keeps or {}
    a = lstm_forward(model.netA, A, trace, "lstm.a.pool")
    v = lstm_forward(model.netV, V, trace, "lstm.v.pool")
    t = textcnn_forward(model.netT, T, training, keeps.get("text"), trace)
    ck = [keeps[f"cls{j}"] for j in range(len(model.netC.widths))] if "cls0" in keeps else None
    return classifier_forward(model.netC, torch.cat([a, v, t], dim=-1), training, ck, trace)


def train_step(model: OracleUttFusion, opt: Optional[OracleAdam], A, V, T, labels,
               keeps: Optional[Dict[str, torch.Tensor]] = None, trace: Optional[MosiTrace] = None) -> Dict:
    """utt_fusion.py:151-200: forward, zero_grad, CE(logits.squeeze(), labels.squeeze()) * 1.0, backward,
    clip_grad_norm_(parameters, clip), Adam (``opt=None``: stop after the clip)."""
    model.train()
    logits = forward(model, A, V, T, True, keeps, trace)
    for p in model.parameters():
        p.grad = None
    loss = 0.0 + 1.0 * F.cross_entropy(logits.squeeze(), labels.squeeze())
    loss.backward()
    norm = None
    if model.clip is not None:
        norm = torch.nn.utils.clip_grad_norm_(model.parameters(), model.clip)
    if opt is not None:
        opt.step()
    preds = F.softmax(logits.detach(), dim=-1).argmax(dim=-1)
    return {"loss": loss.detach(), "logits": logits.detach(), "preds": preds, "total_norm": norm}


@torch.no_grad()
def validation_step(model: OracleUttFusion, A, V, T, labels) -> Dict:
    model.eval()
    logits = forward(model, A, V, T, False)
    loss = 0.0 + 1.0 * F.cross_entropy(logits.squeeze(), labels)
    return {"loss": loss, "logits": logits, "preds": F.softmax(logits, dim=-1).argmax(dim=-1)}


def synthetic_batch(n: int, steps: int = 50, seed: int = 1234, lengths: Optional[List[int]] = None,
                    cfg: UttConfig = MOSI):
    """MOSI-shaped batch (aligned_50: 5-d COVAREP audio, 20-d Facet video, 768-d BERT text, 3 classes; the
    MOSEI config's 74-d / 35-d with ``cfg=MOSEI``).  ``lengths``: per-sample valid steps; the rest is zero
    padding (pad_sequence)."""
    g = torch.Generator().manual_seed(seed)
    A = torch.randn(n, steps, cfg.audio_dim, generator=g)
    V = 0.5 * torch.randn(n, steps, cfg.video_dim, generator=g)
    T = 0.3 * torch.randn(n, steps, cfg.text_dim, generator=g)
    if lengths is not None:
        for i, ln in enumerate(lengths):
            A[i, ln:] = 0
            V[i, ln:] = 0
            T[i, ln:] = 0
    y = torch.randint(0, CLASSES, (n,), generator=g)
    return A, V, T, y


def keep_masks(n: int, seed: int, p: Optional[float] = None, cfg: UttConfig = MOSI) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    pt, pc = (cfg.text_dropout, cfg.cls_dropout) if p is None else (p, p)
    out = {"text": (torch.rand(n, 3 * FILTERS, generator=g) >= pt).to(torch.uint8)}
    for j, w in enumerate(cfg.cls_layers):
        out[f"cls{j}"] = (torch.rand(n, w, generator=g) >= pc).to(torch.uint8)
    return out
