"""The MOSI / MOSEI epoch metric of the UTT-Fusion YAMLs (configs/mosi/centralised/utt_fusion_base_training.yaml
``metrics: MSA: metrics.msa_binary_classification``), restated for the device-count recorder.

Reference: MML_Suite/metrics/msa.py:8-26 (``msa_binarize``) and :44-92 (``msa_binary_classification``).  Classes
are 0 negative / 1 neutral / 2 positive (data/mosi.py classification_labels).  "Has0" scores neutral-vs-rest
over every sample, "Non0" positive-vs-negative over the non-neutral samples.  Reference quirks kept as they are,
because the keys and values must be the reference's: the Recall_* and Precision_* entries are computed with
``f1_score`` (msa.py:54-59,66-71), ``accuracy_score`` takes (preds, truth) — symmetric, so harmless — and every
value is ``round(x, 4)``.

The function is a function of the 3x3 confusion matrix only, so ``metrics.evaluate`` feeds it the expanded
arrays of the device counts (order-independent integer sums: the values are the raw-array call's).
"""
from __future__ import annotations

from typing import Dict

import numpy as np


def msa_binarize(preds: np.ndarray, labels: np.ndarray):
    """msa.py:8-26: (binary_preds, binary_truth, non_zero_indices, non_zero_binary_preds, non_zero_binary_truth)."""
    preds, labels = np.asarray(preds), np.asarray(labels)
    binary_truth = (labels == 1).astype(int)
    binary_preds = (preds == 1).astype(int)
    nz = np.where(labels != 1)[0]
    return binary_preds, binary_truth, nz, (preds[nz] == 2).astype(int), (labels[nz] == 2).astype(int)


def msa_binary_classification(y_true: np.ndarray, y_pred: np.ndarray) -> Dict[str, float]:
    """msa.py:44-92 — the 20 rounded scores, same keys in the same order."""
    from sklearn.metrics import accuracy_score, f1_score

    bp, bt, _, nzp, nzt = msa_binarize(y_pred, y_true)
    out: Dict[str, float] = {}
    for tag, (truth, pred) in (("Non0", (nzt, nzp)), ("Has0", (bt, bp))):
        out[f"{tag}_Accuracy"] = round(accuracy_score(pred, truth), 4)
        for name in ("F1", "Recall", "Precision"):  # all three are f1_score in the reference (msa.py:51-71)
            for avg in ("weighted", "macro", "micro"):
                out[f"{tag}_{name}_{avg}"] = round(f1_score(truth, pred, average=avg), 4)
    return out
