"""ORACLE — CPU fp32 restatement of the monomodal encoder pre-training step.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module.  The product package never imports it.

Restated (reference = TArsenii/task-specific-pretraining-multimodal @ 2025-09-12, paths relative to
``MML_Suite/``):

* ``MonomodalEncoder``             train_monomodal.py:64-95 — ``encoder`` + ``classifier =
                                   nn.Linear(output_dim, num_classes)`` (created after the encoder,
                                   which the YAML tag built first: configs/avmnist/mono/
                                   train_{audio,image}_encoder_resnet.yaml:10-17, train_monomodal.py:525-529)
* ``MonomodalEncoder.train_step``  train_monomodal.py:97-260 — zero_grad → encoder → classifier →
                                   LossFunctionGroup (0.0 + 1.0·CE) → backward → Adam →
                                   ``argmax(logits, 1)`` predictions, accuracy = mean(pred == label)
* ``MonomodalEncoder.validation_step`` train_monomodal.py:262-418 (no_grad, eval-mode BN)

The encoder forward and Adam are the ones of ``avmnist_ref`` (pinned bit-exact against the real
reference by tests/golden/make_golden.py); this module is pinned by tests/golden/make_mono_golden.py
(the real ``train_monomodal.MonomodalEncoder.train_step``, bit-exact on CPU).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .avmnist_ref import (NUM_CLASSES, OracleAdam, OracleResNet, encoder_forward, oracle_resnet18,  # noqa: F401
                          oracle_resnet34)


class OracleMonomodal(nn.Module):
    def __init__(self, encoder: OracleResNet, output_dim: int, num_classes: int = NUM_CLASSES):
        super().__init__()
        self.encoder = encoder
        self.classifier = nn.Linear(output_dim, num_classes)


def build_oracle_monomodal(modality: str = "audio", seed: int = 0) -> OracleMonomodal:
    """Seeded construction in the order train_monomodal.py builds it: the YAML's ``!ResNet18``
    (audio, hidden 64) / ``!ResNet34`` (image, hidden 128) encoder, then the classifier Linear."""
    torch.manual_seed(seed)
    if modality == "audio":
        enc, dim = oracle_resnet18(1, 64), 64
    elif modality == "image":
        enc, dim = oracle_resnet34(1, 128), 128
    else:
        raise ValueError(modality)
    return OracleMonomodal(enc, dim, NUM_CLASSES)


def forward(model: OracleMonomodal, x: torch.Tensor, training: bool, trace=None) -> torch.Tensor:
    """``trace``: an avmnist_ref.MaskTrace (parity instrument; sites prefixed ``enc.``)."""
    e = encoder_forward(model.encoder, x, training, trace, "enc.")
    if e.dim() > 2:  # train_monomodal.py:83-86
        e = e.reshape(e.shape[0], -1)
    return F.linear(e, model.classifier.weight, model.classifier.bias)


def train_step(model: OracleMonomodal, opt: Optional[OracleAdam], x: torch.Tensor, labels: torch.Tensor,
               trace=None) -> Dict[str, torch.Tensor]:
    for p in model.parameters():
        p.grad = None
    logits = forward(model, x, True, trace)
    loss = 0.0 + 1.0 * F.cross_entropy(logits, labels)
    loss.backward()
    if opt is not None:
        opt.step()
    preds = torch.argmax(logits.detach(), dim=1)
    return {"loss": loss.detach(), "logits": logits.detach(), "preds": preds,
            "accuracy": (preds == labels).float().mean()}


@torch.no_grad()
def validation_step(model: OracleMonomodal, x: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
    logits = forward(model, x, False)
    loss = 0.0 + 1.0 * F.cross_entropy(logits, labels)
    preds = torch.argmax(logits, dim=1)
    return {"loss": loss, "logits": logits, "preds": preds, "accuracy": (preds == labels).float().mean()}
