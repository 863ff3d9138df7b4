"""ORACLE — CPU fp32 restatement of the AVMNIST late-fusion train step.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker / the timed CPU baseline.  The product package never imports it.

What is restated (reference = TArsenii/task-specific-pretraining-multimodal @ 2025-09-12,
paths relative to ``MML_Suite/``):

* ``BasicBlock``                  models/msa/networks/resnet.py:8-54
* ``ResNetEncoder`` ctor + init   models/msa/networks/resnet.py:113-189 (kaiming_normal fan_out conv
                                  init, BN weight 1 / bias 0, module creation order kept so that the
                                  same ``torch.manual_seed`` yields bit-identical weights)
* ``ResNetEncoder.forward``       models/msa/networks/resnet.py:199-219
* ``ResNet18`` / ``ResNet34``     models/msa/networks/resnet.py:222-239
* ``AVMNIST`` ctor / forward      models/avmnist.py:193-267 (concat fusion, Linear→ReLU→Dropout→
                                  Linear→ReLU→Linear; keys net.0 / net.3 / net.5)
* ``AVMNIST.train_step``          models/avmnist.py:269-310 (zero_grad, fwd, CE, bwd, Adam step)
* ``LossFunctionGroup``           experiment_utils/loss.py:98-148 (0.0 + 1.0 * CrossEntropyLoss(mean))
* Adam (L2 weight decay folded into the gradient), as torch.optim.Adam's single-tensor path that
  the reference instantiates at config/optimizer_config.py:199-226.

The forward is written with ``torch.nn.functional`` on CPU (fp32); dropout takes an explicit keep
mask so that GPU parity runs can inject the same mask.  Pinned against the real reference by
``tests/golden/make_golden.py`` (bit-exact on CPU) and re-checked by ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
NUM_CLASSES = 10  # MML_Suite/data/avmnist.py:29


# --------------------------------------------------------------------------------------------
# Parameter containers in the reference's creation order (RNG-consumption order matters).
# --------------------------------------------------------------------------------------------
class _OracleBlock(nn.Module):
    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


class OracleResNet(nn.Module):
    def __init__(self, layers: List[int], in_channels: int = 1, hidden_dim: int = 128):
        super().__init__()
        self.hidden_dim = hidden_dim
        self.layer_counts = list(layers)
        self._inplanes = 64
        self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0], 1)
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, hidden_dim)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make(self, planes: int, blocks: int, stride: int) -> nn.Sequential:
        ds = None
        if stride != 1 or self._inplanes != planes:
            ds = nn.Sequential(nn.Conv2d(self._inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        mods = [_OracleBlock(self._inplanes, planes, stride, ds)]
        self._inplanes = planes
        for _ in range(1, blocks):
            mods.append(_OracleBlock(self._inplanes, planes))
        return nn.Sequential(*mods)

    def get_embedding_size(self) -> int:
        return self.hidden_dim


def oracle_resnet18(in_channels: int = 1, hidden_dim: int = 128) -> OracleResNet:
    return OracleResNet([2, 2, 2, 2], in_channels, hidden_dim)


def oracle_resnet34(in_channels: int = 1, hidden_dim: int = 128) -> OracleResNet:
    return OracleResNet([3, 4, 6, 3], in_channels, hidden_dim)


class OracleAVMNIST(nn.Module):
    def __init__(self, audio_encoder: OracleResNet, image_encoder: OracleResNet, hidden_dim: int = 128,
                 dropout: float = 0.5):
        super().__init__()
        self.audio_encoder = audio_encoder
        self.image_encoder = image_encoder
        ea, ei = audio_encoder.get_embedding_size(), image_encoder.get_embedding_size()
        fc_fusion = nn.Linear(ea + ei, hidden_dim)
        fc_mid = nn.Linear(hidden_dim, hidden_dim // 2)
        fc_out = nn.Linear(hidden_dim // 2, NUM_CLASSES)
        self.dropout_p = float(dropout)
        self.net = nn.Sequential(fc_fusion, nn.ReLU(), nn.Dropout(dropout) if dropout > 0 else nn.Identity(),
                                 fc_mid, nn.ReLU(), fc_out)


def build_oracle_avmnist(seed: int = 0, audio_hidden: int = 64, image_hidden: int = 128, hidden: int = 128,
                         dropout: float = 0.5) -> OracleAVMNIST:
    """Seeded construction in the order the YAML config builds it (``!ResNet18`` audio encoder, then
    ``!ResNet34`` image encoder, then ``AVMNIST`` itself: configs/avmnist/centralised/
    train_avmnist_resnet.yaml:10-21, train_multimodal.py:143-144)."""
    torch.manual_seed(seed)
    a = oracle_resnet18(1, audio_hidden)
    i = oracle_resnet34(1, image_hidden)
    return OracleAVMNIST(a, i, hidden, dropout)


# --------------------------------------------------------------------------------------------
# Functional forward (fp32, CPU)
# --------------------------------------------------------------------------------------------
def _bn(x: torch.Tensor, bn: nn.BatchNorm2d, training: bool) -> torch.Tensor:
    # F.batch_norm updates running stats in place in training mode (momentum 0.1, unbiased var)
    return F.batch_norm(x, bn.running_mean, bn.running_var, bn.weight, bn.bias, training, BN_MOMENTUM, BN_EPS)


def _bump_tracked(bn: nn.BatchNorm2d, training: bool) -> None:
    if training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)


class MaskTrace:
    """Parity instrument (test infrastructure): every ReLU and max-pool of the forward goes through
    here when a trace is passed.  Record mode keeps each site's input (pre-activation / pooled map)
    and the pool's argmax; force mode additionally REPLACES the decision -- the ReLU becomes
    ``x * mask`` and the pool a gather at the given flat indices -- so an fp64 run can follow the
    exact threshold / argmax decisions an fp32 implementation took (a decision on an element whose
    value is within rounding of the threshold or of a tie is not a property of the algorithm).
    Sites: ``{prefix}stem``, ``{prefix}mp``, ``{prefix}blk{i}.a1``, ``{prefix}blk{i}.out`` (block i in
    forward order), ``head.h1``, ``head.hh``."""

    def __init__(self, force: Optional[Dict[str, torch.Tensor]] = None):
        self.force = force
        self.pre: Dict[str, torch.Tensor] = {}
        self.idx: Dict[str, torch.Tensor] = {}

    def relu(self, site: str, x: torch.Tensor) -> torch.Tensor:
        self.pre[site] = x.detach()
        if self.force is None or site not in self.force:
            return F.relu(x)
        return x * self.force[site].to(device=x.device, dtype=x.dtype)

    def maxpool(self, site: str, x: torch.Tensor) -> torch.Tensor:
        out, idx = F.max_pool2d(x, 3, 2, 1, return_indices=True)
        self.pre[site] = x.detach()
        self.idx[site] = idx
        if self.force is None or site not in self.force:
            return out
        fi = self.force[site].to(x.device)
        n, c, p, q = out.shape
        return x.flatten(2).gather(2, fi.reshape(n, c, p * q)).view(n, c, p, q)


def block_forward(b: _OracleBlock, x: torch.Tensor, training: bool, trace: Optional[MaskTrace] = None,
                  site: str = "") -> torch.Tensor:
    if trace is None:
        relu = lambda t, k: F.relu(t)  # noqa: E731
    else:
        relu = lambda t, k: trace.relu(site + k, t)  # noqa: E731
    out = F.conv2d(x, b.conv1.weight, None, b.stride, 1)
    out = relu(_bn(out, b.bn1, training), ".a1"); _bump_tracked(b.bn1, training)
    out = F.conv2d(out, b.conv2.weight, None, 1, 1)
    out = _bn(out, b.bn2, training); _bump_tracked(b.bn2, training)
    if b.downsample is not None:
        c, bn = b.downsample[0], b.downsample[1]
        identity = _bn(F.conv2d(x, c.weight, None, c.stride, 0), bn, training); _bump_tracked(bn, training)
    else:
        identity = x
    return relu(out + identity, ".out")


def encoder_forward(enc: OracleResNet, x: torch.Tensor, training: bool, trace: Optional[MaskTrace] = None,
                    prefix: str = "") -> torch.Tensor:
    if x.dim() == 3:  # resnet.py:201-203
        x = x.unsqueeze(1)
    x = F.conv2d(x, enc.conv1.weight, None, 2, 3)
    x = _bn(x, enc.bn1, training)
    x = F.relu(x) if trace is None else trace.relu(prefix + "stem", x)
    _bump_tracked(enc.bn1, training)
    x = F.max_pool2d(x, 3, 2, 1) if trace is None else trace.maxpool(prefix + "mp", x)
    i = 0
    for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
        for blk in layer:
            x = block_forward(blk, x, training, trace, f"{prefix}blk{i}")
            i += 1
    x = F.adaptive_avg_pool2d(x, (1, 1)).flatten(1)
    return F.linear(x, enc.fc.weight, enc.fc.bias)


def head_forward(model: OracleAVMNIST, fused: torch.Tensor, training: bool,
                 keep_mask: Optional[torch.Tensor], trace: Optional[MaskTrace] = None) -> torch.Tensor:
    net = model.net
    relu = (lambda t, k: F.relu(t)) if trace is None else (lambda t, k: trace.relu(k, t))  # noqa: E731
    h = relu(F.linear(fused, net[0].weight, net[0].bias), "head.h1")
    if training and model.dropout_p > 0:
        if keep_mask is None:
            keep_mask = torch.bernoulli(torch.full_like(h, 1.0 - model.dropout_p))
        h = h * (keep_mask.to(h.dtype) / (1.0 - model.dropout_p))
    h = relu(F.linear(h, net[3].weight, net[3].bias), "head.hh")
    return F.linear(h, net[5].weight, net[5].bias)


def avmnist_forward(model: OracleAVMNIST, audio: torch.Tensor, image: torch.Tensor, training: bool,
                    keep_mask: Optional[torch.Tensor] = None,
                    trace: Optional[MaskTrace] = None) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    ea = encoder_forward(model.audio_encoder, audio, training, trace, "audio.")
    ei = encoder_forward(model.image_encoder, image, training, trace, "image.")
    logits = head_forward(model, torch.cat((ea, ei), dim=1), training, keep_mask, trace)
    return logits, ea, ei


# --------------------------------------------------------------------------------------------
# Adam exactly as torch.optim.Adam's single-tensor path (L2 weight decay folded into grad)
# --------------------------------------------------------------------------------------------
class OracleAdam:
    def __init__(self, params: List[torch.Tensor], lr: float = 5e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-4):
        self.params = list(params)
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        self.step_count = 0
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]

    @torch.no_grad()
    def step(self) -> None:
        self.step_count += 1
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        step_size = self.lr / bc1
        bc2_sqrt = bc2 ** 0.5
        for p, m, v in zip(self.params, self.m, self.v):
            if p.grad is None:
                continue
            g = p.grad
            if self.wd != 0:
                g = g.add(p, alpha=self.wd)
            m.lerp_(g, 1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / bc2_sqrt).add_(self.eps)
            p.addcdiv_(m, denom, value=-step_size)


def train_step(model: OracleAVMNIST, opt: Optional[OracleAdam], audio: torch.Tensor, image: torch.Tensor,
               labels: torch.Tensor, keep_mask: Optional[torch.Tensor] = None,
               trace: Optional[MaskTrace] = None) -> Dict[str, torch.Tensor]:
    """models/avmnist.py:269-310 restated: zero_grad → fwd → CE(mean)·1.0 → backward → Adam
    (``opt=None``: stop before the optimizer step, gradients left in ``.grad``)."""
    for p in model.parameters():
        p.grad = None
    logits, ea, ei = avmnist_forward(model, audio, image, True, keep_mask, trace)
    loss = 0.0 + 1.0 * F.cross_entropy(logits, labels)  # loss.py:131-148 (defaultdict(float) + w·CE)
    loss.backward()
    if opt is not None:
        opt.step()
    preds = torch.softmax(logits.detach(), 1).argmax(1)
    return {"loss": loss.detach(), "logits": logits.detach(), "emb_audio": ea.detach(), "emb_image": ei.detach(),
            "preds": preds}


# --------------------------------------------------------------------------------------------
# Synthetic AVMNIST-shaped inputs (BASELINE.md "Synthetic inputs")
# --------------------------------------------------------------------------------------------
def synthetic_batch(batch: int, seed: int = 1234, lut: Optional[torch.Tensor] = None):
    """Audio: fp32 [B,32,94] = 10**clip(N(0.108, 5.85), log10 2.2e-9, log10 1.52e7).
    Image: uint8 [B,28,28] with 81 % zeros, rest U{1..255}; float image = LUT[u8] * (1/255) when a LUT
    is given (data/avmnist.py:186-191), else u8 * (1/255).  Labels U{0..9} int64."""
    import numpy as np
    rng = np.random.default_rng(seed)
    la = np.clip(rng.normal(0.108, 5.85, size=(batch, 32, 94)), math.log10(2.2e-9), math.log10(1.52e7))
    audio = torch.from_numpy((10.0 ** la).astype(np.float32))
    u8 = rng.integers(1, 256, size=(batch, 28, 28)).astype(np.uint8)
    u8[rng.random((batch, 28, 28)) < 0.81] = 0
    img_u8 = torch.from_numpy(u8)
    mapped = lut[img_u8.long()] if lut is not None else img_u8
    image = (mapped.to(torch.float32) * (1.0 / 255.0)).unsqueeze(1)
    labels = torch.from_numpy(rng.integers(0, 10, size=(batch,)).astype(np.int64))
    return audio, image, labels, img_u8


def param_names_in_order(model: nn.Module) -> List[str]:
    return [n for n, _ in model.named_parameters()]


def state_dict_fp32(model: nn.Module) -> "OrderedDict[str, torch.Tensor]":
    return OrderedDict((k, v.detach().clone()) for k, v in model.state_dict().items())
