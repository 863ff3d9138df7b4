"""MOSI UTT-Fusion on the HIP path (BASELINE.json configs[4]).

Drop-ins for the reference's classes, same constructor arguments, attribute names and ``state_dict``
keys (MML_Suite paths):

* ``LSTMEncoder``     models/msa/networks/lstm.py:8-67   (``rnn`` = nn.LSTM parameter container, "last" /
                      "maxpool")
* ``TextCNN``         models/msa/networks/textcnn.py:10-69
* ``FcClassifier``    models/msa/networks/classifier.py:83-117
* ``UttFusionModel``  models/msa/utt_fusion.py:25-294 (forward, train_step with clip_grad_norm_,
                      validation_step, get_embeddings, get_encoder)

configs/mosi/centralised/utt_fusion_base_training.yaml: LSTM 5→64 (audio) and 20→64 (video), TextCNN
over 768-d text (3 x 128 filters of heights 3/4/5, dropout 0.5, Linear 384→64 + ReLU), FcClassifier
192 → 192/64/32 → 3 (ReLU + dropout 0.5 per layer), cross-entropy, clip 1.0, Adam lr 1e-3 / wd 1e-3.
configs/mosei/centralised/utt_fusion_train_mosei.yaml (the same model on CMU-MOSEI): LSTM 74→64 and 35→64
with the "maxpool" embedding, TextCNN dropout 0.7, FcClassifier 192 → 96/48 → 3 with ``use_bn`` (Linear →
ReLU → BatchNorm1d → Dropout 0.66), clip 0.5, Adam lr 2e-4 / wd 1e-5, batch 256.

``MosiEngine`` is the step's kernel schedule for a fixed (batch, steps): inputs time-major on the device
([T][B][F], rows (t, b)); LSTM input projections and weight gradients on the MFMA GEMM
(``tspm_linear_*``), the recurrences in ``tspm_lstm_fwd/bwd`` (both encoders in one launch each), the
TextCNN convolutions on the LDS-staged implicit-GEMM conv kernel (a (h, 768) kernel over [B,1,T,768]
is a 1-D convolution with 768 input channels; the reference's [C,1,h,768] weight is already its OHWI
layout), pooling + dropout in ``tspm_textcnn_pool_fwd``, the sparse TextCNN weight gradient in
``tspm_textcnn_bwd``, the classifier on the small-GEMM kernel, cross-entropy, the clip coefficient
(``tspm_grad_clip_coef``) and Adam (``tspm_adam_step_clip``).  ``FusedMosiStep`` captures all of it as
one HIP graph.
"""
from __future__ import annotations

import ctypes
import os
from collections import defaultdict
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from ._lib import linear_bwd
from .optim import FusedAdam

NUM_CLASSES = 3  # data/mosi.py:26 (classification_labels)
_CLS_SEED_SALT = 0x6A09E667F3BCC909  # the classifier masks' seed = model seed ^ salt (independent of the text masks)
PATTERNS = {"atv": (1.0, 1.0, 1.0), "at": (1.0, 1.0, 0.0), "av": (1.0, 0.0, 1.0), "tv": (0.0, 1.0, 1.0),
            "a": (1.0, 0.0, 0.0), "t": (0.0, 1.0, 0.0), "v": (0.0, 0.0, 1.0)}  # (audio, text, video) data/mosi.py:60-68


# The model / optimizer blocks of the two UTT-Fusion YAMLs (configs/mosi/centralised/utt_fusion_base_training.yaml,
# configs/mosei/centralised/utt_fusion_train_mosei.yaml): what build_utt_fusion constructs, in YAML order.
YAML_CONFIGS = {
    "mosi": dict(audio_dim=5, video_dim=20, text_dim=768, embd_method="last", text_dropout=0.5, cls_layers=(192, 64, 32),
                 cls_dropout=0.5, use_bn=False, clip=1.0, lr=1e-3, weight_decay=1e-3, batch=128),
    "mosei": dict(audio_dim=74, video_dim=35, text_dim=768, embd_method="maxpool", text_dropout=0.7, cls_layers=(96, 48),
                  cls_dropout=0.66, use_bn=True, clip=0.5, lr=2e-4, weight_decay=1e-5, batch=256),
}


def build_utt_fusion(name: str = "mosi") -> "UttFusionModel":
    """UttFusionModel of the named YAML (netA, netV, netT, netC constructed in the YAML's order, so a
    ``torch.manual_seed`` before the call gives the reference's initial weights)."""
    c = YAML_CONFIGS[name]
    netA = LSTMEncoder(input_size=c["audio_dim"], hidden_size=64, embd_method=c["embd_method"])
    netV = LSTMEncoder(input_size=c["video_dim"], hidden_size=64, embd_method=c["embd_method"])
    netT = TextCNN(input_size=c["text_dim"], embd_size=64, dropout=c["text_dropout"], in_channels=1, out_channels=128,
                   kernel_heights=[3, 4, 5])
    netC = FcClassifier(input_dim=192, layers=list(c["cls_layers"]), output_dim=3, dropout=c["cls_dropout"],
                        use_bn=c["use_bn"])
    return UttFusionModel(netA, netV, netT, netC, clip=c["clip"])


# ------------------------------------------------------------------------------------------------
# parameter containers (reference attribute names / state_dict keys / construction order)
# ------------------------------------------------------------------------------------------------
class LSTMEncoder(nn.Module):
    """lstm.py:8-67: one-directional nn.LSTM(batch_first=True); embd "last" = h_n, "maxpool" = max over
    time of r_out (lstm.py:47-52, F.max_pool1d: first maximum)."""

    def __init__(self, input_size: int, hidden_size: int, embd_method: str = "last"):
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.rnn = nn.LSTM(self.input_size, self.hidden_size, batch_first=True)
        assert embd_method in ["maxpool", "attention", "last"]
        if embd_method == "attention":
            raise NotImplementedError("LSTMEncoder HIP path: embd_method 'last' or 'maxpool' (the MOSI / MOSEI "
                                      "UTT-Fusion configs)")
        self.embd_method = embd_method

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """Inference embedding h_T of x [B, T, input] (gradients flow through UttFusionModel only)."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()) and x.requires_grad:
            raise L.TspmError("LSTMEncoder: train it inside UttFusionModel (the fused HIP step / its autograd node)")
        return _encode_lstm(self, x)


class TextCNN(nn.Module):
    """textcnn.py:10-69: Conv2d(in, C, (h_i, input)) x3 → ReLU → time-max → cat → Dropout → Linear + ReLU."""

    def __init__(self, input_size: int, embd_size: int = 128, in_channels: int = 1, out_channels: int = 128,
                 kernel_heights: Sequence[int] = (3, 4, 5), dropout: float = 0.5) -> None:
        super().__init__()
        if in_channels != 1 or len(kernel_heights) != 3:
            raise NotImplementedError("TextCNN HIP path: in_channels 1 and three kernel heights (textcnn.py:24-44)")
        self.conv1 = nn.Conv2d(in_channels, out_channels, (kernel_heights[0], input_size), stride=1, padding=0)
        self.conv2 = nn.Conv2d(in_channels, out_channels, (kernel_heights[1], input_size), stride=1, padding=0)
        self.conv3 = nn.Conv2d(in_channels, out_channels, (kernel_heights[2], input_size), stride=1, padding=0)
        self.dropout = nn.Dropout(dropout)
        self.embd = nn.Sequential(nn.Linear(len(kernel_heights) * out_channels, embd_size), nn.ReLU(inplace=True))
        self.hidden_size = embd_size
        self.heights = [int(k) for k in kernel_heights]
        self.out_channels = out_channels
        self.input_size = input_size

    def convs(self):
        return [self.conv1, self.conv2, self.conv3]


class FcClassifier(nn.Module):
    """classifier.py:83-117: per layer Linear → ReLU (→ BatchNorm1d) (→ Dropout); fc_out."""

    def __init__(self, input_dim: int, layers: List[int], output_dim: int, *, dropout: float = 0.3,
                 use_bn: bool = False) -> None:
        super().__init__()
        if len(layers) == 0:
            raise NotImplementedError("FcClassifier HIP path: at least one hidden layer")
        self.all_layers = []
        for i in range(0, len(layers)):
            self.all_layers.append(nn.Linear(input_dim, layers[i]))
            self.all_layers.append(nn.ReLU())
            if use_bn:
                self.all_layers.append(nn.BatchNorm1d(layers[i]))
            if dropout > 0:
                self.all_layers.append(nn.Dropout(dropout))
            input_dim = layers[i]
        self.module = nn.Sequential(*self.all_layers)
        self.fc_out = nn.Linear(layers[-1], output_dim)
        self.widths = [int(w) for w in layers]
        self.use_bn = bool(use_bn)

    @property
    def dropout_p(self) -> float:
        """The rate the kernels use, read from the nn.Dropout modules each time (one rate per classifier,
        classifier.py:104-105; 0 when the classifier was built without dropout)."""
        ps = {float(m.p) for m in self.module if isinstance(m, nn.Dropout)}
        if len(ps) > 1:
            raise L.TspmError(f"FcClassifier HIP path: one dropout rate for every layer (found {sorted(ps)})")
        return ps.pop() if ps else 0.0

    @dropout_p.setter
    def dropout_p(self, p: float) -> None:
        drops = [m for m in self.module if isinstance(m, nn.Dropout)]
        if not drops and p > 0:
            raise L.TspmError("FcClassifier was built without dropout layers")
        for m in drops:
            m.p = float(p)

    def linears(self):
        return [m for m in self.module if isinstance(m, nn.Linear)]

    def bns(self):
        return [m for m in self.module if isinstance(m, nn.BatchNorm1d)]


# ------------------------------------------------------------------------------------------------
# kernel schedule
# ------------------------------------------------------------------------------------------------
def _conv_algo(n: int) -> L.ConvAlgo:
    """TextCNN conv tile: the LDS-staged kernel (64-row x 128-channel tiles) when the batch allows,
    else the register-direct kernel's heuristic."""
    if n % 64 == 0:
        return L.ConvAlgo(1, 2, 2, 1, 1, 1)
    return L.ConvAlgo()


class MosiEngine:
    """Execution plan of UttFusionModel for a fixed (batch, steps): pre-allocated time-major buffers, one
    fixed sequence of libtspm launches on the caller's stream (graph-capturable)."""

    def __init__(self, model: "UttFusionModel", batch: int, steps: int, device: torch.device):
        self.m, self.B, self.T, self.device = model, batch, steps, device
        a, v, t, c = model.netA, model.netV, model.netT, model.netC
        if a.hidden_size != 64 or v.hidden_size != 64:
            raise NotImplementedError("MOSI HIP path: LSTM hidden size 64 (tspm_lstm_fwd)")
        if steps > 255 or min(t.heights) > steps or max(t.heights) > 5:
            raise L.TspmError("MOSI HIP path: 1 <= kernel heights <= min(5, steps) and steps <= 255")
        f = dict(device=device, dtype=torch.float32)
        B, T, H = batch, steps, 64
        self.fa, self.fv, self.ft = a.input_size, v.input_size, t.input_size
        self.A = torch.zeros(T, B, self.fa, **f)          # time-major inputs
        self.V = torch.zeros(T, B, self.fv, **f)
        self.X = torch.zeros(T, B, self.ft, **f)
        self.labels = torch.zeros(B, dtype=torch.int64, device=device)
        self.groups = torch.zeros(B, dtype=torch.int32, device=device)
        self.E = a.hidden_size + v.hidden_size + t.hidden_size
        if c.linears()[0].in_features != self.E:
            raise L.TspmError("FcClassifier input_dim must equal the sum of the three embedding sizes")
        self.fused = torch.zeros(B, self.E, **f)
        self.lstm = {}
        for name, enc in (("a", a), ("v", v)):
            self.lstm[name] = dict(xg=torch.empty(T * B, 4 * H, **f), gates=torch.empty(T * B, 4 * H, **f),
                                   cs=torch.empty(T * B, H, **f), hs=torch.empty((T + 1) * B, H, **f),
                                   dg=torch.empty(T * B, 4 * H, **f))
            # "maxpool" embedding: the time index of each unit's maximum (uint8 [B][H])
            self.lstm[name]["arg"] = (torch.zeros(B, H, dtype=torch.uint8, device=device)
                                      if enc.embd_method == "maxpool" else None)
        C, nc = t.out_channels, 3 * t.out_channels
        self.C, self.nc = C, nc
        self.conv_shapes = [L.ConvShape(B, T, 1, self.ft, C, k, 1, 1, 0, T - k + 1, 1) for k in t.heights]
        self.conv_algo = _conv_algo(B)
        from .engine import tuned_table
        tab = tuned_table()
        self.conv_algos = []
        for s in self.conv_shapes:
            e = tab.get(("fwd", s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride))
            self.conv_algos.append(L.ConvAlgo(*e) if e is not None else self.conv_algo)
        self.conv_out = [torch.empty((T - k + 1) * B, C, **f) for k in t.heights]
        lib = L.lib()
        ws = max(lib.tspm_conv_fwd_workspace(ctypes.byref(s), ctypes.byref(al))
                 for s, al in zip(self.conv_shapes, self.conv_algos))
        self.conv_ws = torch.zeros(max(int(ws), 256), dtype=torch.uint8, device=device)
        self.pooled = torch.empty(B, nc, **f)
        self.argmax = torch.empty(B, nc, dtype=torch.uint8, device=device)
        self.fc_in = torch.empty(B, nc, **f)
        self.widths = c.widths
        self.h = [torch.empty(B, w, **f) for w in self.widths]
        self.logits = torch.empty(B, c.fc_out.out_features, **f)
        self.dlogits = torch.empty_like(self.logits)
        self.dh = [torch.empty(B, w, **f) for w in self.widths]
        # FcClassifier(use_bn): per layer the ReLU output r (the BatchNorm input), its batch statistics and the
        # gradient of r's Linear (the BN backward writes it with the ReLU mask applied)
        self.use_bn = c.use_bn
        if self.use_bn:
            self.r = [torch.empty(B, w, **f) for w in self.widths]
            self.bn_mean = [torch.empty(w, **f) for w in self.widths]
            self.bn_inv = [torch.empty(w, **f) for w in self.widths]
            self.dr = [torch.empty(B, w, **f) for w in self.widths]
        self.dfused = torch.empty(B, self.E, **f)
        self.dfc_in = torch.empty(B, nc, **f)
        self.g_work = torch.empty(B, nc, **f)
        self.loss = torch.zeros(1, **f)
        self.stats = torch.zeros(4, **f)
        # dropout keep masks: TextCNN (before the embedding Linear) + one per classifier layer
        sizes = [nc] + self.widths
        self.keep_all = torch.ones(B * sum(sizes), dtype=torch.uint8, device=device)
        self.keeps, off = [], 0
        for w in sizes:
            self.keeps.append(self.keep_all[off:off + B * w].view(B, w))
            off += B * w
        self.keep_override: Optional[Dict[str, torch.Tensor]] = None
        self.rng_ctr_ptr: Optional[int] = None
        self._host_ctr: Optional[torch.Tensor] = None
        # LSTM weight gradients reduce over T*B rows into 256 x {in, 64} outputs (8-16 output tiles): split
        # the reduction so the launch fills the chip (tspm_linear_bwd_weight_splitk)
        # — one split for all four (db_ih and db_hh come from two calls and must stay bitwise equal)
        sp = max(1, min(32, (T * B) // 128))
        self.wg_splits = {fin: sp for fin in (self.fa, self.fv, H)}
        wsb = max(int(lib.tspm_linear_bwd_weight_splitk_workspace(T * B, fin, 4 * H, sp)) for fin in (self.fa, self.fv, H))
        self.wg_ws = torch.empty(max(wsb // 4, 1), **f)
        self.concurrent = os.environ.get("TSPM_MOSI_SERIAL", "0") != "1"
        self.side: Optional[torch.cuda.Stream] = None
        self.clip_coef = torch.ones(1, **f)
        self.total_norm = torch.zeros(1, **f)
        self.clip_ws = torch.zeros(int(lib.tspm_grad_clip_workspace()) // 4 + 1, **f)
        self.grad_of = lambda p: p.grad  # noqa: E731  (FusedAdam's flat gradient views)
        self._index = torch.arange(B, dtype=torch.int64, device=device)
        self._lens = torch.full((B,), T, dtype=torch.int32, device=device)
        self._offs = torch.arange(B, dtype=torch.int64, device=device) * T

    # -- inputs -------------------------------------------------------------------------------------
    def load(self, A: torch.Tensor, V: torch.Tensor, T: torch.Tensor, labels: Optional[torch.Tensor] = None) -> None:
        """Batch-first [B, T, F] reference tensors → the time-major buffers (tspm_seq_gather: one launch per
        modality, the dense batch seen as B sequences of length T)."""
        lib, sh = L.lib(), L.stream_handle()
        for src, dst, nm in ((A, self.A, "audio"), (V, self.V, "video"), (T, self.X, "text")):
            L.require_cuda_f32(src, nm)
            if tuple(src.shape) != (self.B, self.T, dst.shape[2]):
                raise L.TspmError(f"{nm} batch shape {tuple(src.shape)} != planned {(self.B, self.T, dst.shape[2])}")
            src = src.contiguous()
            L.check(lib.tspm_seq_gather(self.B, self._index.data_ptr(), self.B, src.data_ptr(), self._offs.data_ptr(),
                                        self._lens.data_ptr(), dst.shape[2], self.T, dst.data_ptr(),
                                        self.B * dst.shape[2], dst.shape[2], None, None, None, sh), "seq_gather")
        if labels is not None:
            self.labels.copy_(labels.reshape(-1).to(self.labels.dtype), non_blocking=True)

    # -- forward ------------------------------------------------------------------------------------
    def apply_keep_override(self) -> None:
        """Copy injected dropout masks (parity hook: {"text", "cls0", ...} -> uint8) into the keep buffers;
        called before the step runs, outside any captured graph."""
        if self.keep_override is None:
            return
        names = ["text"] + [f"cls{j}" for j in range(len(self.widths))]
        for k, dst in zip(names, self.keeps):
            dst.copy_(self.keep_override[k].reshape(dst.shape).to(torch.uint8), non_blocking=True)

    def _keep_masks(self, train: bool, sh: int) -> None:
        """Fresh keep masks for one training forward: the TextCNN slice (keeps[0]) at the TextCNN's own rate
        (textcnn.py:45, netT.dropout.p), the classifier slices at the classifier's (classifier.py:104-105);
        two independent draws (the classifier's under a derived seed) on the same step counter."""
        pt, pc = float(self.m.netT.dropout.p), float(self.m.netC.dropout_p)
        if not train or (pt <= 0 and pc <= 0) or self.keep_override is not None:
            return
        if self.rng_ctr_ptr is None:
            self._host_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
            self.rng_ctr_ptr = self._host_ctr.data_ptr()
        lib, seed = L.lib(), self.m._rng_seed
        nt = self.keeps[0].numel()
        if pt > 0:
            L.check(lib.tspm_dropout_mask(nt, pt, seed, self.rng_ctr_ptr, self.keep_all.data_ptr(), sh),
                    "dropout_mask (text)")
        if pc > 0:
            L.check(lib.tspm_dropout_mask(self.keep_all.numel() - nt, pc, seed ^ _CLS_SEED_SALT, self.rng_ctr_ptr,
                                          self.keep_all.data_ptr() + nt, sh), "dropout_mask (classifier)")
        if self._host_ctr is not None and self.rng_ctr_ptr == self._host_ctr.data_ptr():
            self._host_ctr.add_(1)  # outside FusedMosiStep nothing else advances the counter: fresh masks per step

    def _fork(self):
        """Side stream for the LSTM half of the step (it shares no buffer with the TextCNN half until the
        classifier): returns (side torch stream, its handle) after making it wait for the main stream."""
        if self.side is None:
            self.side = L.shared_streams(self.device, 1)[0]
            self._ev = [torch.cuda.Event() for _ in range(4)]
        main = torch.cuda.current_stream(self.device)
        self._ev[0].record(main)
        self.side.wait_event(self._ev[0])
        return self.side, self.side.cuda_stream

    def _join(self) -> None:
        self._ev[1].record(self.side)
        torch.cuda.current_stream(self.device).wait_event(self._ev[1])

    def forward(self, sh: int, train: bool) -> None:
        """Dropout masks, then the LSTM half (side stream) concurrently with the TextCNN half (caller's
        stream), joined before the classifier; everything graph-capturable."""
        self._keep_masks(train, sh)
        if self.concurrent:
            side, sh_side = self._fork()
            with torch.cuda.stream(side):
                self._forward_lstm(sh_side)
            self._forward_text(sh, train)
            self._join()
        else:
            self._forward_lstm(sh)
            self._forward_text(sh, train)
        self._forward_classifier(sh, train)

    def _forward_lstm(self, sh: int) -> None:
        lib, m = L.lib(), self.m
        B, T = self.B, self.T
        # LSTM input projections over all T*B rows, then both recurrences in one launch
        descs = (L.LstmFwdDesc * 2)()
        for i, (name, enc, x, fin, col) in enumerate((("a", m.netA, self.A, self.fa, 0),
                                                      ("v", m.netV, self.V, self.fv, m.netA.hidden_size))):
            bufs, rnn = self.lstm[name], enc.rnn
            L.check(lib.tspm_linear_fwd(T * B, fin, 4 * enc.hidden_size, x.data_ptr(), fin, rnn.weight_ih_l0.data_ptr(),
                                        rnn.bias_ih_l0.data_ptr(), 0, None, 1.0, bufs["xg"].data_ptr(),
                                        4 * enc.hidden_size, sh), "lstm input projection")
            d = descs[i]
            d.batch, d.steps, d.hidden, d.ld_out = B, T, enc.hidden_size, self.E
            d.xg, d.w_hh, d.b_hh = bufs["xg"].data_ptr(), rnn.weight_hh_l0.data_ptr(), rnn.bias_hh_l0.data_ptr()
            d.gates, d.cs, d.hs = bufs["gates"].data_ptr(), bufs["cs"].data_ptr(), bufs["hs"].data_ptr()
            d.h_out = self.fused.data_ptr() + col * 4
            d.argmax = L.ptr(bufs["arg"])
        L.check(lib.tspm_lstm_fwd(2, descs, sh), "lstm_fwd")

    def _forward_text(self, sh: int, train: bool) -> None:
        lib, m = L.lib(), self.m
        B, T = self.B, self.T
        # TextCNN: three convolutions (implicit GEMM), pooling + dropout, embedding Linear + ReLU
        t = m.netT
        for conv, s, al, y in zip(t.convs(), self.conv_shapes, self.conv_algos, self.conv_out):
            L.check(lib.tspm_conv_fwd(ctypes.byref(s), ctypes.byref(al), self.X.data_ptr(), None,
                                      conv.weight.data_ptr(), y.data_ptr(), None, self.conv_ws.data_ptr(),
                                      self.conv_ws.numel(), sh), "textcnn conv")
        heights = (ctypes.c_int32 * 3)(*t.heights)
        outs = (ctypes.c_void_p * 3)(*[y.data_ptr() for y in self.conv_out])
        biases = (ctypes.c_void_p * 3)(*[cv.bias.data_ptr() for cv in t.convs()])
        tp = t.dropout.p
        keep_t = self.keeps[0].data_ptr() if (train and tp > 0) else None
        L.check(lib.tspm_textcnn_pool_fwd(B, T, 3, heights, self.C, outs, biases, keep_t,
                                          1.0 / (1.0 - tp) if tp < 1 else 0.0, self.pooled.data_ptr(),
                                          self.argmax.data_ptr(), self.fc_in.data_ptr(), self.nc, sh), "textcnn pool")
        col_t = m.netA.hidden_size + m.netV.hidden_size
        emb = t.embd[0]
        L.check(lib.tspm_linear_fwd(B, self.nc, emb.out_features, self.fc_in.data_ptr(), self.nc, emb.weight.data_ptr(),
                                    emb.bias.data_ptr(), 1, None, 1.0, self.fused.data_ptr() + col_t * 4, self.E, sh),
                "textcnn embd")

    def _forward_classifier(self, sh: int, train: bool) -> None:
        lib, m, B = L.lib(), self.m, self.B
        # FcClassifier: (Linear, ReLU, [BatchNorm1d,] Dropout) per layer, fc_out
        c = m.netC
        cp = c.dropout_p
        x, fin = self.fused, self.E
        if self.use_bn:
            for j, (lin, bn, hbuf) in enumerate(zip(c.linears(), c.bns(), self.h)):
                w = lin.out_features
                L.check(lib.tspm_linear_fwd(B, fin, w, x.data_ptr(), fin, lin.weight.data_ptr(), lin.bias.data_ptr(),
                                            1, None, 1.0, self.r[j].data_ptr(), w, sh), f"classifier {j}")
                if train:
                    keep = self.keeps[1 + j].data_ptr() if cp > 0 else None
                    L.check(lib.tspm_bn1d_fwd_drop(B, w, self.r[j].data_ptr(), bn.weight.data_ptr(), bn.bias.data_ptr(),
                                                   bn.running_mean.data_ptr(), bn.running_var.data_ptr(),
                                                   float(bn.momentum), float(bn.eps), self.bn_mean[j].data_ptr(),
                                                   self.bn_inv[j].data_ptr(), keep,
                                                   1.0 / (1.0 - cp) if 0 < cp < 1 else 1.0, hbuf.data_ptr(), sh),
                            f"classifier bn {j}")
                else:
                    L.check(lib.tspm_bn_apply_eval(B, w, self.r[j].data_ptr(), bn.running_mean.data_ptr(),
                                                   bn.running_var.data_ptr(), float(bn.eps), bn.weight.data_ptr(),
                                                   bn.bias.data_ptr(), 0, None, None, None, None, None, 0,
                                                   hbuf.data_ptr(), sh), f"classifier bn {j} (eval)")
                x, fin = hbuf, w
            if train:  # num_batches_tracked += 1 of every classifier BatchNorm1d: one launch
                from .step import shared_batches_tracked
                L.counters_add(shared_batches_tracked(m, self.device, (nn.BatchNorm1d,)), 1, sh)
        else:  # Linear + ReLU + Dropout in one launch per layer
            for j, (lin, hbuf) in enumerate(zip(c.linears(), self.h)):
                keep = self.keeps[1 + j].data_ptr() if (train and cp > 0) else None
                L.check(lib.tspm_linear_fwd(B, fin, lin.out_features, x.data_ptr(), fin, lin.weight.data_ptr(),
                                            lin.bias.data_ptr(), 1, keep, 1.0 / (1.0 - cp) if cp < 1 else 0.0,
                                            hbuf.data_ptr(), lin.out_features, sh), f"classifier {j}")
                x, fin = hbuf, lin.out_features
        fo = c.fc_out
        L.check(lib.tspm_linear_fwd(B, fin, fo.out_features, x.data_ptr(), fin, fo.weight.data_ptr(),
                                    fo.bias.data_ptr(), 0, None, 1.0, self.logits.data_ptr(), fo.out_features, sh),
                "classifier out")

    def loss_fn(self, sh: int, weight: float, with_grad: bool, stats: bool = False) -> None:
        L.check(L.lib().tspm_cross_entropy(self.B, self.logits.shape[1], self.logits.data_ptr(), self.labels.data_ptr(),
                                           self.loss.data_ptr(), self.dlogits.data_ptr() if with_grad else None, weight,
                                           self.stats.data_ptr() if stats else None, sh), "cross_entropy")

    # -- backward -----------------------------------------------------------------------------------
    def backward(self, sh: int) -> None:
        lib, m, g = L.lib(), self.m, self.grad_of
        B, T = self.B, self.T
        c = m.netC
        cscale = 1.0 / (1.0 - c.dropout_p) if c.dropout_p > 0 else 1.0
        lins = c.linears()
        fo = c.fc_out
        linear_bwd(B, self.widths[-1], fo.out_features, self.h[-1].data_ptr(), self.widths[-1], self.dlogits.data_ptr(),
                   fo.out_features, fo.weight.data_ptr(), g(fo.weight).data_ptr(), g(fo.bias).data_ptr(),
                   self.dh[-1].data_ptr(), self.widths[-1], sh)
        bns = c.bns()
        for j in range(len(lins) - 1, -1, -1):
            w = self.widths[j]
            if self.use_bn:  # Dropout → BatchNorm1d → ReLU backward in one launch: dy of the Linear in dr[j]
                keep = self.keeps[1 + j].data_ptr() if c.dropout_p > 0 else None
                L.check(lib.tspm_bn1d_bwd_drop_relu(B, w, self.dh[j].data_ptr(), keep, cscale, self.r[j].data_ptr(),
                                                    self.bn_mean[j].data_ptr(), self.bn_inv[j].data_ptr(),
                                                    bns[j].weight.data_ptr(), g(bns[j].weight).data_ptr(),
                                                    g(bns[j].bias).data_ptr(), self.dr[j].data_ptr(), sh),
                        "cls bn bwd")
                dy = self.dr[j]
            else:
                L.check(lib.tspm_act_bwd(B, w, self.dh[j].data_ptr(), w, self.h[j].data_ptr(), w, cscale, sh),
                        "cls relu")
                dy = self.dh[j]
            xin, fin = (self.h[j - 1], self.widths[j - 1]) if j > 0 else (self.fused, self.E)
            dx, lddx = (self.dh[j - 1], self.widths[j - 1]) if j > 0 else (self.dfused, self.E)
            linear_bwd(B, fin, w, xin.data_ptr(), fin, dy.data_ptr(), w, lins[j].weight.data_ptr(),
                       g(lins[j].weight).data_ptr(), g(lins[j].bias).data_ptr(), dx.data_ptr(), lddx, sh)
        if self.concurrent:
            side, sh_side = self._fork()
            with torch.cuda.stream(side):
                self._backward_lstm(sh_side)
            self._backward_text(sh)
            self._join()
        else:
            self._backward_text(sh)
            self._backward_lstm(sh)

    def _backward_text(self, sh: int) -> None:
        lib, m, g = L.lib(), self.m, self.grad_of
        B, T = self.B, self.T
        # TextCNN: embedding ReLU, Linear, then pooling/dropout and the sparse conv weight gradients
        t = m.netT
        col_t = m.netA.hidden_size + m.netV.hidden_size
        emb = t.embd[0]
        dcol = self.dfused.data_ptr() + col_t * 4
        L.check(lib.tspm_act_bwd(B, emb.out_features, dcol, self.E, self.fused.data_ptr() + col_t * 4, self.E, 1.0, sh),
                "textcnn embd relu")
        linear_bwd(B, self.nc, emb.out_features, self.fc_in.data_ptr(), self.nc, dcol, self.E, emb.weight.data_ptr(),
                   g(emb.weight).data_ptr(), g(emb.bias).data_ptr(), self.dfc_in.data_ptr(), self.nc, sh)
        heights = (ctypes.c_int32 * 3)(*t.heights)
        dws = (ctypes.c_void_p * 3)(*[g(cv.weight).data_ptr() for cv in t.convs()])
        dbs = (ctypes.c_void_p * 3)(*[g(cv.bias).data_ptr() for cv in t.convs()])
        tp = t.dropout.p
        L.check(lib.tspm_textcnn_bwd(B, T, self.ft, 3, heights, self.C, self.X.data_ptr(), self.dfc_in.data_ptr(),
                                     self.nc, self.keeps[0].data_ptr() if tp > 0 else None,
                                     1.0 / (1.0 - tp) if 0 < tp < 1 else 1.0, self.pooled.data_ptr(),
                                     self.argmax.data_ptr(), dws, dbs, self.g_work.data_ptr(), sh), "textcnn bwd")

    def _backward_lstm(self, sh: int) -> None:
        lib, m, g = L.lib(), self.m, self.grad_of
        B, T = self.B, self.T
        # LSTMs: backward through time (one launch for both), then the weight gradients as GEMMs over T*B rows
        descs = (L.LstmBwdDesc * 2)()
        for i, (name, enc, col) in enumerate((("a", m.netA, 0), ("v", m.netV, m.netA.hidden_size))):
            bufs, rnn = self.lstm[name], enc.rnn
            d = descs[i]
            d.batch, d.steps, d.hidden, d.ld_dh = B, T, enc.hidden_size, self.E
            d.w_hh, d.gates, d.cs = rnn.weight_hh_l0.data_ptr(), bufs["gates"].data_ptr(), bufs["cs"].data_ptr()
            d.dh, d.dgates = self.dfused.data_ptr() + col * 4, bufs["dg"].data_ptr()
            d.argmax = L.ptr(bufs["arg"])
        L.check(lib.tspm_lstm_bwd(2, descs, sh), "lstm_bwd")
        for name, enc, x, fin in (("a", m.netA, self.A, self.fa), ("v", m.netV, self.V, self.fv)):
            bufs, rnn, H = self.lstm[name], enc.rnn, enc.hidden_size
            # dW_hh = dgates^T h_{t-1} (rows (t, b) of hs[0:T]); db_hh = column sums of dgates
            ws, wsb = self.wg_ws.data_ptr(), self.wg_ws.numel() * 4
            L.check(lib.tspm_linear_bwd_weight_splitk(T * B, H, 4 * H, bufs["hs"].data_ptr(), H, bufs["dg"].data_ptr(),
                                                      4 * H, g(rnn.weight_hh_l0).data_ptr(),
                                                      g(rnn.bias_hh_l0).data_ptr(), self.wg_splits[H], ws, wsb, sh),
                    "lstm dW_hh")
            # dW_ih = dgates^T x; db_ih = the same column sums (same split and order: bitwise db_hh)
            L.check(lib.tspm_linear_bwd_weight_splitk(T * B, fin, 4 * H, x.data_ptr(), fin, bufs["dg"].data_ptr(),
                                                      4 * H, g(rnn.weight_ih_l0).data_ptr(),
                                                      g(rnn.bias_ih_l0).data_ptr(), self.wg_splits[fin], ws, wsb, sh),
                    "lstm dW_ih")

    def clip(self, sh: int, flat_grad: torch.Tensor, grad_scale: float) -> None:
        """clip_grad_norm_(model.parameters(), clip) coefficient into ``clip_coef`` (utt_fusion.py:188-189)."""
        L.check(L.lib().tspm_grad_clip_coef(flat_grad.numel(), flat_grad.data_ptr(), grad_scale, float(self.m.clip),
                                            self.clip_coef.data_ptr(), self.total_norm.data_ptr(),
                                            self.clip_ws.data_ptr(), self.clip_ws.numel() * 4, sh), "grad_clip")


def _ce_weight(loss_functions) -> Optional[float]:
    from .step import _ce_weight as ce
    return ce(loss_functions)


class FusedMosiStep:
    """One UTT-Fusion train step — forward, cross-entropy, backward, gradient clip, Adam — as one HIP
    graph (captured on the second call; the backward overwrites every gradient, no zero_grad pass)."""

    def __init__(self, model: "UttFusionModel", optimizer: FusedAdam, loss_functions, batch: int, steps: int,
                 use_graph: bool = True, allreduce=None):
        if not isinstance(optimizer, FusedAdam):
            raise L.TspmError("FusedMosiStep needs FusedAdam (the flat gradient buffer the kernels write)")
        dev = next(model.parameters()).device
        if dev.type != "cuda":
            raise L.TspmError("FusedMosiStep runs on the MI355X: move the model to cuda first")
        fgs = optimizer.flat_groups()
        if len(fgs) != 1:
            raise L.TspmError("FusedMosiStep: one FusedAdam parameter group (the clip norm spans all parameters)")
        self.model, self.opt, self.N, self.T = model, optimizer, batch, steps
        self.weight = _ce_weight(loss_functions)
        if self.weight is None:
            raise L.TspmError("FusedMosiStep: the loss group must be a single cross-entropy term")
        self.eng = MosiEngine(model, batch, steps, dev)
        self.eng.rng_ctr_ptr = fgs[0].hyper.data_ptr() + L.HYPER_STEP_OFFSET
        if model.clip is not None:
            optimizer.clip_coef = self.eng.clip_coef
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        self.allreduce = allreduce
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.calls = 0
        self.log = None  # metrics.ClassificationLog (train predictions on the device)

    @property
    def keep_override(self):
        return self.eng.keep_override

    @keep_override.setter
    def keep_override(self, v):
        self.eng.keep_override = v

    def _fwd_bwd(self) -> None:
        sh = L.stream_handle()
        e = self.eng
        e.forward(sh, True)
        e.loss_fn(sh, self.weight, True, True)
        if self.log is not None:
            lg = self.log
            L.check(L.lib().tspm_classify_update(self.N, e.logits.shape[1], e.logits.data_ptr(), e.labels.data_ptr(),
                                                 e.groups.data_ptr(), len(lg.groups), lg.conf.data_ptr(), None,
                                                 e.loss.data_ptr(), lg.loss_log.data_ptr(), lg.counters.data_ptr(),
                                                 lg.capacity, sh), "classify_update")
        e.backward(sh)

    def _opt(self) -> None:
        sh = L.stream_handle()
        if self.model.clip is not None:
            fg = self.opt.flat_groups()[0]
            self.eng.clip(sh, fg.grad, self.opt.grad_scale)
        self.opt.launch(sh)

    def _all(self) -> None:
        self._fwd_bwd()
        if self.allreduce is None:
            self._opt()

    def step(self, A, V, T, labels) -> Dict[str, torch.Tensor]:
        self.eng.load(A, V, T, labels)
        self.run()
        return {"loss": self.eng.loss, "logits": self.eng.logits}

    def run(self) -> None:
        self.model.train()
        self.opt.sync_hyper()
        self.eng.apply_keep_override()
        if self.model.clip is not None:
            self.opt.clip_coef = self.eng.clip_coef
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
            self._opt()
        self.opt.note_steps(1)
        self.calls += 1


class FusedMosiEvalStep:
    """``validation_step``'s device work (utt_fusion.py:202-244) for one (batch, steps) shape as one HIP graph:
    eval-mode forward (no dropout; running statistics in the MOSEI classifier BatchNorm1d), the loss group's
    cross-entropy, and ``tspm_classify_update`` (softmax argmax, per-pattern confusion counts, the batch loss
    appended to the epoch's log) — no host synchronisation.  Inputs are the engine's time-major buffers
    (``mosi_data.MOSI.device_loader(step_for=...)`` gathers into them) or a batch-first batch via ``step``."""

    def __init__(self, model: "UttFusionModel", loss_functions, batch: int, steps: int, log, use_graph: bool = True):
        dev = next(model.parameters()).device
        self.model, self.N, self.T, self.log = model, batch, steps, log
        self.weight = _ce_weight(loss_functions)
        if self.weight is None:
            raise L.TspmError("FusedMosiEvalStep: the loss group must be a single cross-entropy term")
        self.eng = model._engine(batch, steps, dev)
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.calls = 0

    def _all(self) -> None:
        sh, e, lg = L.stream_handle(), self.eng, self.log
        e.forward(sh, False)
        e.loss_fn(sh, self.weight, False)
        L.check(L.lib().tspm_classify_update(self.N, e.logits.shape[1], e.logits.data_ptr(), e.labels.data_ptr(),
                                             e.groups.data_ptr(), len(lg.groups), lg.conf.data_ptr(), None,
                                             e.loss.data_ptr(), lg.loss_log.data_ptr(), lg.counters.data_ptr(),
                                             lg.capacity, sh), "classify_update")

    def step(self, A, V, T, labels) -> None:
        self.eng.load(A, V, T, labels)
        self.run()

    def run(self) -> None:
        self.model.eval()
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
        self.calls += 1


# ------------------------------------------------------------------------------------------------
# the model
# ------------------------------------------------------------------------------------------------
def _modality(batch: Dict[Any, Any], name: str):
    for k, v in batch.items():
        kk = str(getattr(k, "value", k)).lower().split(".")[-1]
        if kk == name:
            return v
    raise KeyError(f"batch has no {name!r} modality key (keys: {list(batch.keys())})")


class _UttFn(torch.autograd.Function):
    """The whole UTT-Fusion forward as one autograd node (HIP schedule forward and backward), for the
    reference's own train_step sequence with a non-fused optimizer."""

    @staticmethod
    def forward(ctx, A, V, T, model: "UttFusionModel", *params):
        eng = model._engine(A.shape[0], A.shape[1], A.device)
        eng.load(A, V, T)
        eng.apply_keep_override()
        eng.forward(L.stream_handle(), True)
        model._fwd_generation += 1
        ctx.model, ctx.eng, ctx.gen = model, eng, model._fwd_generation
        return eng.logits.clone()

    @staticmethod
    def backward(ctx, g):
        model, eng = ctx.model, ctx.eng
        if model._fwd_generation != ctx.gen:
            raise L.TspmError("UttFusionModel: another training forward ran before this backward")
        eng.dlogits.copy_(g.reshape(eng.dlogits.shape))
        grads: Dict[int, torch.Tensor] = {}

        def grad_of(p):
            t = grads.get(id(p))
            if t is None:
                t = torch.empty_like(p)
                grads[id(p)] = t
            return t
        for p in model.parameters():  # allocate on this stream before the backward forks its side stream
            grad_of(p)
        eng.grad_of = grad_of
        try:
            eng.backward(L.stream_handle())
        finally:
            eng.grad_of = lambda p: p.grad  # noqa: E731
        return (None, None, None, None, *[grads.get(id(p)) for p in model.parameters()])


class UttFusionModel(nn.Module):
    """models/msa/utt_fusion.py:25-294 drop-in (MultimodalMonitoringMixin hooks are not on the hot path)."""

    def __init__(self, netA: LSTMEncoder, netV: LSTMEncoder, netT: TextCNN, netC: FcClassifier, *,
                 clip: Optional[float] = None, pretrained_path: Optional[str] = None) -> None:
        super().__init__()
        self.netA = netA
        self.netV = netV
        self.netT = netT
        self.netC = netC
        self.clip = clip
        self.pretrained_path = pretrained_path
        self._rng_seed = int(torch.initial_seed()) & ((1 << 63) - 1)
        self._engines: Dict[Any, MosiEngine] = {}
        self._steps: Dict[Any, FusedMosiStep] = {}
        self._fwd_generation = 0

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._engines, self._steps = {}, {}
        return out

    def _engine(self, b: int, t: int, device) -> MosiEngine:
        if torch.device(device).type != "cuda":
            raise L.TspmError("UttFusionModel (tspm_amd) runs on the MI355X only (no CPU fallback)")
        key = (b, t, device)
        eng = self._engines.get(key)
        if eng is None:
            eng = MosiEngine(self, b, t, device)
            self._engines[key] = eng
        return eng

    def fused_step(self, optimizer: FusedAdam, loss_functions, batch: int, steps: int) -> FusedMosiStep:
        """The cached FusedMosiStep for (optimizer, loss group, batch, padded steps) — one captured graph per
        padded length (mosi_data.MOSI.device_loader(step_for=...) gathers straight into its inputs)."""
        key = (id(optimizer), id(loss_functions), int(batch), int(steps))
        st = self._steps.get(key)
        if st is None:
            st = FusedMosiStep(self, optimizer, loss_functions, int(batch), int(steps))
            self._steps[key] = st
        return st

    def load_pretrained(self) -> None:
        """utt_fusion.py:63-78 (weights-only checkpoint load)."""
        if self.pretrained_path is None:
            raise ValueError("No pretrained weights loaded.")
        sd = torch.load(self.pretrained_path, map_location="cpu", weights_only=True)
        self.load_state_dict(sd["model_state_dict"])

    def get_encoder(self, modality):
        name = str(getattr(modality, "value", modality)).lower().split(".")[-1]
        enc = {"audio": self.netA, "video": self.netV, "text": self.netT}.get(name)
        if enc is None:
            raise ValueError(f"Unknown modality: {modality}")
        return enc

    def flatten_parameters(self) -> None:
        """utt_fusion.py:142-147 (cuDNN RNN weight flattening; nothing to do on this path)."""

    def forward(self, A: Optional[torch.Tensor] = None, V: Optional[torch.Tensor] = None,
                T: Optional[torch.Tensor] = None, *, is_embd_A: bool = False, is_embd_V: bool = False,
                is_embd_T: bool = False) -> torch.Tensor:
        """utt_fusion.py:105-140 with all three modalities given as [B, T, F] sequences (a missing modality
        is the zeroed tensor the dataset delivers, data/base_dataset.py:61-74)."""
        assert not all((A is None, V is None, T is None)), "At least one of A, V, T must be provided"
        assert not all([is_embd_A, is_embd_V, is_embd_T]), "Cannot have all embeddings as True"
        if A is None or V is None or T is None or is_embd_A or is_embd_V or is_embd_T:
            raise NotImplementedError("UttFusionModel HIP path: A, V and T sequences (no pre-embedded inputs)")
        A, V, T = A.float(), V.float(), T.float()
        if not (A.is_cuda and V.is_cuda and T.is_cuda):
            raise L.TspmError("UttFusionModel (tspm_amd) runs on the MI355X only; move the model and inputs to the "
                              "ROCm device (there is no CPU fallback)")
        if self.training and torch.is_grad_enabled():
            params = list(self.parameters())
            return _UttFn.apply(A, V, T, self, *params)
        eng = self._engine(A.shape[0], A.shape[1], A.device)
        eng.load(A, V, T)
        eng.forward(L.stream_handle(), self.training)
        return eng.logits.clone()

    def train_step(self, batch: Dict[str, Any], optimizer, loss_functions, device, metric_recorder,
                   **kwargs: Any) -> Dict[str, Any]:
        """utt_fusion.py:151-200.  With FusedAdam and the single cross-entropy loss group: one FusedMosiStep
        graph (forward, loss, backward, clip_grad_norm_, Adam); otherwise the reference's own sequence
        on the HIP forward/backward (one autograd node)."""
        A = _modality(batch, "audio").to(device).float()
        V = _modality(batch, "video").to(device).float()
        T = _modality(batch, "text").to(device).float()
        labels = batch["label"].to(device)
        miss = batch.get("pattern_name")
        if isinstance(optimizer, FusedAdam) and _ce_weight(loss_functions) is not None and A.is_cuda:
            out = self.fused_step(optimizer, loss_functions, A.shape[0], A.shape[1]).step(A, V, T, labels)
            logits, loss = out["logits"], out["loss"]
        else:
            self.train()
            logits = self.forward(A, V, T)
            optimizer.zero_grad()
            loss = loss_functions(logits.squeeze(), labels.squeeze())["total_loss"]
            loss.backward()
            if self.clip is not None:
                torch.nn.utils.clip_grad_norm_(self.parameters(), self.clip)
            optimizer.step()
        if metric_recorder is not None:
            preds = torch.softmax(logits.detach(), dim=-1).argmax(dim=-1).squeeze()
            metric_recorder.update_group_all("classification", predictions=preds.cpu().numpy(),
                                             targets=labels.squeeze().detach().cpu().numpy(),
                                             m_types=np.array(miss if miss is not None else []))
        return {"loss": float(loss.item())}

    @torch.no_grad()
    def validation_step(self, batch: Dict[str, Any], loss_functions, device, metric_recorder,
                        return_test_info: bool = False, **kwargs: Any) -> Dict[str, Any]:
        """utt_fusion.py:202-256: eval-mode forward (no dropout) + the loss group on the HIP kernels."""
        self.eval()
        A = _modality(batch, "audio").to(device).float()
        V = _modality(batch, "video").to(device).float()
        T = _modality(batch, "text").to(device).float()
        labels = batch["label"].to(device)
        miss = np.array(batch.get("pattern_name", []))
        eng = self._engine(A.shape[0], A.shape[1], A.device)
        eng.load(A, V, T, labels)
        sh = L.stream_handle()
        eng.forward(sh, False)
        w = _ce_weight(loss_functions)
        if w is not None:
            eng.loss_fn(sh, w, False)
            loss = eng.loss.clone()
        else:
            loss = loss_functions(eng.logits.squeeze(), labels)["total_loss"]
        preds = torch.softmax(eng.logits, dim=-1).argmax(dim=-1).squeeze()
        if metric_recorder is not None:
            metric_recorder.update_group_all("classification", predictions=preds.cpu().numpy(),
                                             targets=labels.squeeze().cpu().numpy(), m_types=miss)
        self.train()
        if return_test_info:
            return {"loss": loss.item(), "predictions": [preds.cpu().numpy()], "labels": [labels.cpu().numpy()],
                    "miss_types": [list(miss)]}
        return {"loss": loss.item()}

    @torch.no_grad()
    def get_embeddings(self, dataloader, device) -> Dict[Any, List[np.ndarray]]:
        """utt_fusion.py:258-294."""
        self.eval()
        emb: Dict[Any, List[np.ndarray]] = defaultdict(list)
        for batch in dataloader:
            A = _modality(batch, "audio").to(device).float()
            V = _modality(batch, "video").to(device).float()
            T = _modality(batch, "text").to(device).float()
            eng = self._engine(A.shape[0], A.shape[1], A.device)
            eng.load(A, V, T)
            eng.forward(L.stream_handle(), False)
            ha, hv = self.netA.hidden_size, self.netV.hidden_size
            keys = [k for k in batch.keys() if str(getattr(k, "value", k)).lower().split(".")[-1] in
                    ("audio", "video", "text")]
            cols = {"audio": slice(0, ha), "video": slice(ha, ha + hv), "text": slice(ha + hv, eng.E)}
            for k in keys:
                name = str(getattr(k, "value", k)).lower().split(".")[-1]
                emb[k].append(eng.fused[:, cols[name]].cpu().numpy())
            emb["label"] += list(batch["label"])
        return emb


def _encode_lstm(enc: LSTMEncoder, x: torch.Tensor) -> torch.Tensor:
    """Standalone LSTMEncoder embedding (inference): projection GEMM + one-problem tspm_lstm_fwd."""
    L.require_cuda_f32(x, "LSTMEncoder input")
    B, T, F = x.shape
    dev, H = x.device, enc.hidden_size
    f = dict(device=dev, dtype=torch.float32)
    xt = x.transpose(0, 1).contiguous() if T > 1 else x.reshape(1, B, F).contiguous()
    xg, gates = torch.empty(T * B, 4 * H, **f), torch.empty(T * B, 4 * H, **f)
    cs, hs, out = torch.empty(T * B, H, **f), torch.empty((T + 1) * B, H, **f), torch.empty(B, H, **f)
    arg = torch.empty(B, H, dtype=torch.uint8, device=dev) if enc.embd_method == "maxpool" else None
    lib, sh, rnn = L.lib(), L.stream_handle(), enc.rnn
    L.check(lib.tspm_linear_fwd(T * B, F, 4 * H, xt.data_ptr(), F, rnn.weight_ih_l0.data_ptr(),
                                rnn.bias_ih_l0.data_ptr(), 0, None, 1.0, xg.data_ptr(), 4 * H, sh), "lstm proj")
    d = (L.LstmFwdDesc * 1)()
    d[0].batch, d[0].steps, d[0].hidden, d[0].ld_out = B, T, H, H
    d[0].xg, d[0].w_hh, d[0].b_hh = xg.data_ptr(), rnn.weight_hh_l0.data_ptr(), rnn.bias_hh_l0.data_ptr()
    d[0].gates, d[0].cs, d[0].hs, d[0].h_out = gates.data_ptr(), cs.data_ptr(), hs.data_ptr(), out.data_ptr()
    d[0].argmax = L.ptr(arg)
    L.check(lib.tspm_lstm_fwd(1, d, sh), "lstm_fwd")
    return out
