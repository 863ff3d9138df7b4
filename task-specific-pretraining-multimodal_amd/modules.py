"""Drop-in replacements for the reference's encoder and fusion classes.

* ``BasicBlock`` / ``ResNetEncoder`` / ``ResNet18`` / ``ResNet34`` — same constructor signatures,
  submodule names, creation + initialisation order (so ``torch.manual_seed`` gives bit-identical
  weights) and ``state_dict`` keys as MML_Suite/models/msa/networks/resnet.py:8-54,113-239.  The
  submodules are parameter containers only: ``forward`` runs the libtspm HIP schedule
  (``engine.EncoderEngine``) and plugs into autograd as one ``torch.autograd.Function`` per encoder.
* ``AVMNIST`` — MML_Suite/models/avmnist.py:188-410 (late fusion by concat → Linear/ReLU/Dropout/
  Linear/ReLU/Linear), with ``train_step`` running the fused native step (``step.FusedTrainStep``:
  forward, cross-entropy, backward, Adam as one captured HIP graph) when the optimizer is this
  package's ``FusedAdam`` and the loss group is the reference's single cross-entropy term; otherwise
  it follows the reference's own autograd sequence with the HIP encoders/head.

Conv weights are kept OHWI (``channels_last`` view of the OIHW parameter); values, shapes and keys
are unchanged, so ``best.pth`` / ``encoder_{mod}_best.pth`` checkpoints interoperate.
"""
from __future__ import annotations

from collections import defaultdict
from functools import partial
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from .engine import EncoderEngine, prepare_encoder_layout

NUM_CLASSES = 10  # MML_Suite/data/avmnist.py:29


# ------------------------------------------------------------------------------------------------
# ResNet encoder (parameter containers in the reference's creation order)
# ------------------------------------------------------------------------------------------------
class BasicBlock(nn.Module):
    """Parameter container of resnet.py:8-54 (conv1, bn1, relu, conv2, bn2, downsample)."""
    expansion: int = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None,
                 norm_layer=None) -> None:
        super().__init__()
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d
        self.conv1 = nn.Conv2d(inplanes, planes, kernel_size=3, stride=stride, padding=1, bias=False)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=1, padding=1, bias=False)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):  # pragma: no cover - blocks run inside the encoder schedule
        raise RuntimeError("BasicBlock is executed by ResNetEncoder's HIP schedule, not standalone")


class ResNetEncoder(nn.Module):
    """resnet.py:113-219 — ResNet encoder for 1-channel AVMNIST inputs, HIP-executed."""

    def __init__(self, block=BasicBlock, layers: Sequence[int] = (2, 2, 2, 2), in_channels: int = 1,
                 hidden_dim: int = 128, zero_init_residual: bool = False, norm_layer=None) -> None:
        super().__init__()
        if isinstance(block, str):
            if block.lower() not in ("basicblock", "basic"):
                raise NotImplementedError(f"block {block!r}: only BasicBlock (ResNet18/34) is on the HIP path")
            block = BasicBlock
        if getattr(block, "expansion", 1) != 1:
            raise NotImplementedError("Bottleneck (ResNet50) is outside the AVMNIST hot path (SURVEY §8)")
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d
        if norm_layer is not nn.BatchNorm2d:
            raise NotImplementedError("only nn.BatchNorm2d is supported on the HIP path")
        self._norm_layer = norm_layer
        self.hidden_dim = hidden_dim
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2d(in_channels, self.inplanes, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = norm_layer(self.inplanes)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(BasicBlock, 64, layers[0])
        self.layer2 = self._make_layer(BasicBlock, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(BasicBlock, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(BasicBlock, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * BasicBlock.expansion, hidden_dim)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)
        self._engines: Dict[Tuple, EncoderEngine] = {}
        self._fwd_generation = 0

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2d(self.inplanes, planes * block.expansion, kernel_size=1, stride=stride, bias=False),
                norm_layer(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample, norm_layer)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, norm_layer=norm_layer))
        return nn.Sequential(*layers)

    def get_embedding_size(self) -> int:
        return self.hidden_dim

    # -- HIP execution ---------------------------------------------------------------------------
    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._engines = {}  # parameters moved: drop plans bound to old storage
        return out

    def engine_for(self, x: torch.Tensor) -> EncoderEngine:
        if x.dim() == 3:
            n, h, w = x.shape
        else:
            n, _, h, w = x.shape
        key = (n, h, w, x.device)
        eng = self._engines.get(key)
        if eng is None:
            prepare_encoder_layout(self)
            eng = EncoderEngine(self, n, h, w, x.device)
            self._engines[key] = eng
        return eng

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise L.TspmError("ResNetEncoder (tspm_amd) runs on the MI355X only; move the model and inputs to the "
                              "ROCm device (there is no CPU fallback)")
        x = x.float()
        if x.dim() == 4 and not x.is_contiguous():
            x = x.contiguous()
        eng = self.engine_for(x)
        params = [p for p in self.parameters()]
        if self.training and torch.is_grad_enabled():
            return _EncoderFn.apply(x, self, eng, *params)
        emb = torch.empty(eng.N, self.hidden_dim, device=x.device, dtype=torch.float32)
        eng.forward(x, emb, self.hidden_dim, train=self.training)
        if self.training:
            self._fwd_generation += 1
        return emb


class _EncoderFn(torch.autograd.Function):
    """One autograd node for the whole encoder: forward = HIP schedule, backward = HIP schedule."""

    @staticmethod
    def forward(ctx, x, enc: ResNetEncoder, eng: EncoderEngine, *params):
        emb = torch.empty(eng.N, enc.hidden_dim, device=x.device, dtype=torch.float32)
        eng.forward(x, emb, enc.hidden_dim, train=True)
        enc._fwd_generation += 1
        ctx.enc, ctx.eng, ctx.gen = enc, eng, enc._fwd_generation
        ctx.n_params = len(params)
        return emb

    @staticmethod
    def backward(ctx, g):
        enc, eng = ctx.enc, ctx.eng
        if enc._fwd_generation != ctx.gen:
            raise L.TspmError("ResNetEncoder: another training forward ran before this backward; the HIP plan "
                              "keeps one set of saved activations per (batch, H, W)")
        g = g.contiguous().float()
        grads: Dict[int, torch.Tensor] = {}

        def grad_of(p):
            t = grads.get(id(p))
            if t is None:
                t = torch.empty_like(p, memory_format=torch.channels_last if p.dim() == 4 else torch.contiguous_format)
                grads[id(p)] = t
            return t

        eng.grad_of = grad_of
        try:
            eng.backward(g, enc.hidden_dim)
        finally:
            eng.grad_of = _engine_default_grad_of
        out = [grads.get(id(p)) for p in enc.parameters()]
        return (None, None, None, *out)


def _engine_default_grad_of(p):
    from .engine import _default_grad_of
    return _default_grad_of(p)


def ResNet18(in_channels: int = 1, hidden_dim: int = 128) -> ResNetEncoder:
    """resnet.py:222-229."""
    return ResNetEncoder(block=BasicBlock, layers=[2, 2, 2, 2], in_channels=in_channels, hidden_dim=hidden_dim)


def ResNet34(in_channels: int = 1, hidden_dim: int = 128) -> ResNetEncoder:
    """resnet.py:232-239."""
    return ResNetEncoder(block=BasicBlock, layers=[3, 4, 6, 3], in_channels=in_channels, hidden_dim=hidden_dim)


# ------------------------------------------------------------------------------------------------
# Fusion model
# ------------------------------------------------------------------------------------------------
def _ce_weight_of(loss_functions):
    from .step import _ce_weight
    return _ce_weight(loss_functions)


def modality_key(batch: Dict[Any, Any], name: str):
    """Find the batch key for modality ``name`` ('audio' / 'image').  The reference keys batches by
    ``modalities.Modality`` members (un-vendored package); accept those, plain strings, or any enum
    whose name/value is the modality name."""
    for k in batch.keys():
        if isinstance(k, str):
            if k.lower() == name:
                return k
            continue
        for attr in ("value", "name"):
            v = getattr(k, attr, None)
            if isinstance(v, str) and v.lower() == name:
                return k
        if str(k).lower().split(".")[-1] == name:
            return k
    raise KeyError(f"batch has no {name!r} modality key (keys: {list(batch.keys())})")


class _HeadFn(torch.autograd.Function):
    """Fusion head  Linear(192,128) → ReLU → Dropout → Linear(128,64) → ReLU → Linear(64,10)
    (models/avmnist.py:219-230) on libtspm kernels; dropout keep-mask drawn on device."""

    @staticmethod
    def forward(ctx, fused, model: "AVMNIST", w0, b0, w3, b3, w5, b5):
        n = fused.shape[0]
        dev = fused.device
        sh = L.stream_handle()
        lib = L.lib()
        hd, h2 = model.hidden_dim, model.hidden_dim // 2
        fused = fused.contiguous()
        h1 = torch.empty(n, hd, device=dev)
        hh = torch.empty(n, h2, device=dev)
        logits = torch.empty(n, NUM_CLASSES, device=dev)
        keep = None
        scale = 1.0
        if model.training and model.dropout_p > 0:
            keep = model._draw_keep(n * hd, dev).view(n, hd)
            scale = 1.0 / (1.0 - model.dropout_p)
        L.check(lib.tspm_linear_fwd(n, fused.shape[1], hd, fused.data_ptr(), fused.shape[1], w0.data_ptr(), b0.data_ptr(),
                                    1, L.ptr(keep), scale, h1.data_ptr(), hd, sh), "head fc0")
        L.check(lib.tspm_linear_fwd(n, hd, h2, h1.data_ptr(), hd, w3.data_ptr(), b3.data_ptr(), 1, None, 1.0,
                                    hh.data_ptr(), h2, sh), "head fc3")
        L.check(lib.tspm_linear_fwd(n, h2, NUM_CLASSES, hh.data_ptr(), h2, w5.data_ptr(), b5.data_ptr(), 0, None, 1.0,
                                    logits.data_ptr(), NUM_CLASSES, sh), "head fc5")
        ctx.save_for_backward(fused, h1, hh, w0, w3, w5)
        ctx.scale = scale
        return logits

    @staticmethod
    def backward(ctx, g):
        fused, h1, hh, w0, w3, w5 = ctx.saved_tensors
        g = g.contiguous().float()
        n = g.shape[0]
        sh = L.stream_handle()
        lib = L.lib()
        hd, h2 = h1.shape[1], hh.shape[1]
        dev = g.device
        gw5, gb5 = torch.empty_like(w5), torch.empty(w5.shape[0], device=dev)
        gw3, gb3 = torch.empty_like(w3), torch.empty(w3.shape[0], device=dev)
        gw0, gb0 = torch.empty_like(w0), torch.empty(w0.shape[0], device=dev)
        dh = torch.empty(n, h2, device=dev)
        dh1 = torch.empty(n, hd, device=dev)
        dfused = torch.empty_like(fused)
        L.check(lib.tspm_linear_bwd_weight(n, h2, NUM_CLASSES, hh.data_ptr(), h2, g.data_ptr(), NUM_CLASSES,
                                           gw5.data_ptr(), gb5.data_ptr(), sh), "head fc5 wgrad")
        L.check(lib.tspm_linear_bwd_data(n, h2, NUM_CLASSES, g.data_ptr(), NUM_CLASSES, w5.data_ptr(), dh.data_ptr(), h2,
                                         sh), "head fc5 dgrad")
        L.check(lib.tspm_act_bwd(n, h2, dh.data_ptr(), h2, hh.data_ptr(), h2, 1.0, sh), "head relu")
        L.check(lib.tspm_linear_bwd_weight(n, hd, h2, h1.data_ptr(), hd, dh.data_ptr(), h2, gw3.data_ptr(),
                                           gb3.data_ptr(), sh), "head fc3 wgrad")
        L.check(lib.tspm_linear_bwd_data(n, hd, h2, dh.data_ptr(), h2, w3.data_ptr(), dh1.data_ptr(), hd, sh),
                "head fc3 dgrad")
        L.check(lib.tspm_act_bwd(n, hd, dh1.data_ptr(), hd, h1.data_ptr(), hd, ctx.scale, sh), "head relu+dropout")
        F = fused.shape[1]
        L.check(lib.tspm_linear_bwd_weight(n, F, hd, fused.data_ptr(), F, dh1.data_ptr(), hd, gw0.data_ptr(),
                                           gb0.data_ptr(), sh), "head fc0 wgrad")
        L.check(lib.tspm_linear_bwd_data(n, F, hd, dh1.data_ptr(), hd, w0.data_ptr(), dfused.data_ptr(), F, sh),
                "head fc0 dgrad")
        return dfused, None, gw0, gb0, gw3, gb3, gw5, gb5


class AVMNIST(nn.Module):
    """models/avmnist.py:188-410 drop-in (MultimodalMonitoringMixin hooks are not on the hot path)."""

    def __init__(self, audio_encoder: nn.Module, image_encoder: nn.Module, hidden_dim: int, *, dropout: float = 0.0,
                 fusion_fn: str = "concat") -> None:
        super().__init__()
        self.audio_encoder = audio_encoder
        self.image_encoder = image_encoder
        self.embd_size_A = audio_encoder.get_embedding_size()
        self.embd_size_I = image_encoder.get_embedding_size()
        self.hidden_dim = hidden_dim
        fc_fusion = nn.Linear(self.embd_size_A + self.embd_size_I, hidden_dim)
        fc_intermediate = nn.Linear(hidden_dim, hidden_dim // 2)
        fc_out = nn.Linear(hidden_dim // 2, NUM_CLASSES)
        self.dropout_p = float(dropout)
        self.net = nn.Sequential(fc_fusion, nn.ReLU(), nn.Dropout(dropout) if dropout > 0 else nn.Identity(),
                                 fc_intermediate, nn.ReLU(), fc_out)
        if fusion_fn.lower() != "concat":
            raise ValueError(f"Unknown fusion function: {fusion_fn}")
        self.fusion_fn = partial(torch.cat, dim=1)
        self._fused_step = None
        self._rng_seed = int(torch.initial_seed()) & ((1 << 63) - 1)
        self._rng_ctr = None
        self.keep_override: Optional[torch.Tensor] = None  # parity hook: inject the dropout keep-mask

    # -- dropout mask --------------------------------------------------------------------------------
    def _draw_keep(self, count: int, dev: torch.device) -> torch.Tensor:
        if self.keep_override is not None:
            k = self.keep_override.to(device=dev, dtype=torch.uint8).reshape(-1)
            if k.numel() != count:
                raise L.TspmError("keep_override has the wrong number of elements")
            return k
        if self._rng_ctr is None or self._rng_ctr.device != dev:
            self._rng_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
        keep = torch.empty(count, dtype=torch.uint8, device=dev)
        L.check(L.lib().tspm_dropout_mask(count, self.dropout_p, self._rng_seed, self._rng_ctr.data_ptr(),
                                          keep.data_ptr(), L.stream_handle()), "dropout_mask")
        self._rng_ctr.add_(1)
        return keep

    # -- forward (autograd path) ---------------------------------------------------------------------
    def forward(self, A: Optional[torch.Tensor] = None, I: Optional[torch.Tensor] = None, *, is_embd_A: bool = False,
                is_embd_I: bool = False) -> torch.Tensor:
        assert not all((A is None, I is None)), "At least one of A, I must be provided"
        assert not all([is_embd_A, is_embd_I]), "Cannot have all embeddings as True"
        ref = A if A is not None else I
        A = A if A is not None else torch.zeros(I.size(0), self.embd_size_A, device=ref.device)
        I = I if I is not None else torch.zeros(A.size(0), self.embd_size_I, device=ref.device)
        audio = self.audio_encoder(A) if not is_embd_A else A
        image = self.image_encoder(I) if not is_embd_I else I
        fused = self.fusion_fn((audio, image))
        n0, n3, n5 = self.net[0], self.net[3], self.net[5]
        return _HeadFn.apply(fused, self, n0.weight, n0.bias, n3.weight, n3.bias, n5.weight, n5.bias)

    # -- steps ---------------------------------------------------------------------------------------
    def _unpack(self, batch, device):
        ka, ki = modality_key(batch, "audio"), modality_key(batch, "image")
        A = batch[ka].to(device, non_blocking=True).float()
        I = batch[ki].to(device, non_blocking=True).float()
        labels = batch["labels"].to(device, non_blocking=True)
        return A, I, labels, batch.get("pattern_name")

    @staticmethod
    def _device_log(metric_recorder):
        from .metrics import DeviceMetricRecorder
        return metric_recorder.log if isinstance(metric_recorder, DeviceMetricRecorder) else None

    @staticmethod
    def _group_ids(batch, log, miss_type, device):
        g = batch.get("pattern_ids")
        if g is not None:
            return g.to(device, non_blocking=True)
        return log.group_ids(miss_type) if (log is not None and miss_type is not None) else None

    def train_step(self, batch: Dict[Any, Any], optimizer, loss_functions, device, metric_recorder, **kwargs):
        """models/avmnist.py:269-310.  Fused native step when possible (see module docstring).  With a
        metrics.DeviceMetricRecorder the batch's predictions are recorded on the device inside the step's
        HIP graph; with the reference's MetricRecorder they are copied to the host as the reference does."""
        from .step import FusedTrainStep, fused_step_supported
        A, I, labels, miss_type = self._unpack(batch, device)
        dlog = self._device_log(metric_recorder)
        if fused_step_supported(self, optimizer, loss_functions, A, I):
            if self._fused_step is None or not self._fused_step.matches(A, I, optimizer, loss_functions):
                self._fused_step = FusedTrainStep(self, optimizer, loss_functions, A.shape[0])
            self._fused_step.log = dlog
            out = self._fused_step.step(A, I, labels, self._group_ids(batch, dlog, miss_type, device))
            logits = out["logits"]
            loss_t = out["loss"]
            if dlog is not None:
                return {"loss": float(loss_t.item())}
        else:
            self.train()
            optimizer.zero_grad()
            logits = self.forward(A=A, I=I)
            loss_t = loss_functions(logits, labels)["total_loss"]
            loss_t.backward()
            optimizer.step()
        if metric_recorder is not None:
            predictions = torch.softmax(logits.detach(), dim=1).argmax(dim=1).cpu().numpy()
            metric_recorder.update_group_all("classification", predictions=predictions,
                                             targets=labels.detach().cpu().numpy(),
                                             m_types=np.array(miss_type if miss_type is not None else []))
        return {"loss": float(loss_t.item())}

    def eval_step_for(self, loss_functions, batch: int, log=None):
        """The cached FusedEvalStep for this batch size (one HIP graph per size)."""
        from .step import FusedEvalStep
        cache = self.__dict__.setdefault("_fused_eval", {})
        st = cache.get(batch)
        if st is None or st.ce_weight != _ce_weight_of(loss_functions):
            st = FusedEvalStep(self, loss_functions, batch, log)
            cache[batch] = st
        st.log = log
        return st

    def validation_step(self, batch, loss_functions, device, metric_recorder, return_test_info: bool = False):
        """models/avmnist.py:312-360 (eval-mode BN running stats, dropout off).  With a single
        cross-entropy loss group the batch runs as one FusedEvalStep graph (predictions recorded on the
        device when metric_recorder is a metrics.DeviceMetricRecorder)."""
        self.eval()
        with torch.no_grad():
            A, I, labels, miss_type = self._unpack(batch, device)
            dlog = self._device_log(metric_recorder)
            if (_ce_weight_of(loss_functions) is not None and A.is_cuda and I.is_cuda and A.dim() == 3
                    and tuple(A.shape[1:]) == (32, 94) and tuple(I.shape[-2:]) == (28, 28)):
                st = self.eval_step_for(loss_functions, A.shape[0], dlog)
                out = st.step(A, I, labels, self._group_ids(batch, dlog, miss_type, device))
                if dlog is not None and not return_test_info:
                    return {"loss": out["loss"].item()}
                loss = out["loss"]
                predictions = out["preds"].cpu().numpy()
            else:
                logits = self.forward(A=A, I=I)
                loss = loss_functions(logits, labels)["total_loss"]
                predictions = torch.softmax(logits, dim=1).argmax(dim=1).cpu().numpy()
            labels_np = labels.cpu().numpy()
            miss_type = np.array(miss_type if miss_type is not None else [])
            if metric_recorder is not None and dlog is None:
                metric_recorder.update_group_all(group_name="classification", predictions=predictions,
                                                 targets=labels_np, m_types=miss_type)
            if return_test_info:
                return {"loss": loss.item(), "predictions": predictions, "labels": labels_np, "miss_types": miss_type}
        return {"loss": loss.item()}

    def get_embeddings(self, dataloader, device) -> Dict[Any, Any]:
        """models/avmnist.py:362-401."""
        embeddings = defaultdict(list)
        self.to(device)
        self.eval()
        for batch in dataloader:
            with torch.no_grad():
                ka, ki = modality_key(batch, "audio"), modality_key(batch, "image")
                A, I, miss_type = batch[ka], batch[ki], np.array(batch["pattern_name"])
                A = A[miss_type == "ai"].to(device).float()
                I = I[miss_type == "ai"].to(device).float()
                embeddings[ka].append(self.audio_encoder(A).detach().cpu().numpy())
                embeddings[ki].append(self.image_encoder(I).detach().cpu().numpy())
                embeddings["label"] += list(batch["labels"])
        return embeddings

    def get_encoder(self, modality) -> nn.Module:
        name = str(getattr(modality, "value", modality)).lower().split(".")[-1]
        if name == "audio":
            return self.audio_encoder
        if name == "image":
            return self.image_encoder
        raise ValueError(f"Unknown modality: {modality}")
