"""ORACLE — CPU restatement of the AVMNIST evaluation bookkeeping.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module.  Restated (paths under ``MML_Suite/``):

* ``validation_step``     models/avmnist.py:312-360 — eval-mode forward (running BN statistics, no
                          dropout), ``LossFunctionGroup`` total = 0.0 + 1.0·CE(mean), predictions =
                          ``softmax(logits, 1).argmax(1)``
* ``update_group_all``    experiment_utils/metric_recorder.py:126-145 — per pattern (m_type) the
                          (prediction, target) pairs; restated as per-pattern confusion counts
* epoch loss              train_multimodal.py:525-541 — ``np.mean`` of the per-batch ``loss.item()``
Metric values from the counts are pinned separately against the reference's MetricRecorder
(tests/golden/avmnist_metrics.json).
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .avmnist_ref import avmnist_forward


def predictions(logits: torch.Tensor) -> torch.Tensor:
    """models/avmnist.py:345 (first maximum of the softmax)."""
    return torch.softmax(logits, dim=1).argmax(dim=1)


def confusion(labels: np.ndarray, preds: np.ndarray, groups: Optional[np.ndarray], n_groups: int,
              classes: int = 10) -> np.ndarray:
    conf = np.zeros((n_groups, classes, classes), dtype=np.int64)
    g = np.zeros(len(labels), np.int64) if groups is None else np.asarray(groups, np.int64)
    ok = (labels >= 0) & (labels < classes) & (g >= 0) & (g < n_groups)
    np.add.at(conf, (g[ok], labels[ok], preds[ok]), 1)
    return conf


@torch.no_grad()
def validation_step(model, audio: torch.Tensor, image: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
    model.eval()
    logits, _, _ = avmnist_forward(model, audio, image, False)
    loss = 0.0 + 1.0 * F.cross_entropy(logits, labels)
    return {"loss": loss, "logits": logits, "preds": predictions(logits)}


def epoch_loss(batch_losses: Sequence[float]) -> float:
    return float(np.mean([float(x) for x in batch_losses]))
