"""Epoch metrics from device-side confusion counts.

The reference turns every batch's logits into host predictions (``softmax → argmax → .cpu()``,
MML_Suite/models/avmnist.py:305-309,345-350) and stores them in a ``MetricRecorder``
(experiment_utils/metric_recorder.py:67-275) that, at epoch end, concatenates them per missing-data
pattern and calls the metric functions the YAML names (configs/avmnist/centralised/
train_avmnist_resnet.yaml:105-163: sklearn accuracy, balanced accuracy, F1 / precision / recall with
macro / micro / weighted averaging, confusion matrix).  Every one of those is a function of the
per-pattern confusion matrix, so here the batch work is one ``tspm_classify_update`` launch (inside
the step's HIP graph) that adds to int64 confusion counts on the device and logs the batch loss; the
host reads the counts ONCE per epoch and evaluates the very same sklearn functions on the compressed
form — one (label, prediction) pair per non-zero cell with its count as ``sample_weight`` — which
gives the values of the uncompressed call (integer weights: every sum is exact; only cells that
occur are passed, so the inferred label set is unchanged; pinned against raw-array sklearn calls in
tests/test_metrics_cpu.py).  Functions not known to be confusion-only get the expanded arrays.
"""
from __future__ import annotations

import importlib
import logging
from collections import OrderedDict
from functools import partial
from typing import Any, Callable, Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L

NUM_CLASSES = 10
# metric functions whose value depends only on the (true, pred) multiset and that take sample_weight
CONFUSION_ONLY = {"accuracy_score", "balanced_accuracy_score", "f1_score", "precision_score", "recall_score",
                  "fbeta_score", "confusion_matrix", "jaccard_score", "cohen_kappa_score", "matthews_corrcoef",
                  "precision_recall_fscore_support", "multilabel_confusion_matrix"}


class ClassificationLog:
    """Device buffers fed by ``tspm_classify_update``: confusion counts [groups, K, K] (int64), the
    per-batch loss log (fp32) and counters {batches, samples}.  ``groups`` names the missing-data
    patterns (``pattern_name`` values) in id order — by default ``data.AVMNIST.get_all_possible_patterns()``,
    the order of the batches' ``pattern_ids``."""

    def __init__(self, device: torch.device, groups: Sequence[str] = ("a", "ai", "i"), classes: int = NUM_CLASSES,
                 capacity: int = 1 << 16):
        if device.type != "cuda":
            raise L.TspmError("ClassificationLog lives on the ROCm device")
        self.device, self.groups, self.classes, self.capacity = device, list(groups), classes, capacity
        self.gid = {g: i for i, g in enumerate(self.groups)}
        self.conf = torch.zeros(len(self.groups), classes, classes, dtype=torch.int64, device=device)
        self.loss_log = torch.zeros(capacity, dtype=torch.float32, device=device)
        self.counters = torch.zeros(2, dtype=torch.int64, device=device)

    def reset(self) -> None:
        self.conf.zero_()
        self.counters.zero_()

    def group_ids(self, names: Sequence[str]) -> torch.Tensor:
        try:
            ids = [self.gid[n] for n in names]
        except KeyError as e:
            raise L.TspmError(f"pattern {e} is not one of this log's groups {self.groups}") from None
        return torch.tensor(ids, dtype=torch.int32).to(self.device, non_blocking=True)

    def update(self, logits: torch.Tensor, labels: torch.Tensor, groups: Optional[torch.Tensor] = None,
               loss: Optional[torch.Tensor] = None, pred_out: Optional[torch.Tensor] = None,
               stream: Optional[torch.cuda.Stream] = None) -> None:
        n = logits.shape[0]
        if logits.shape[-1] != self.classes or labels.numel() != n:
            raise L.TspmError("classify_update: logits / labels shape mismatch")
        if groups is not None and (groups.dtype != torch.int32 or groups.numel() != n):
            raise L.TspmError("classify_update: groups must be int32 [n]")
        L.check(L.lib().tspm_classify_update(
            n, self.classes, logits.data_ptr(), labels.data_ptr(), L.ptr(groups), len(self.groups),
            self.conf.data_ptr(), L.ptr(pred_out), L.ptr(loss), self.loss_log.data_ptr() if loss is not None else None,
            self.counters.data_ptr(), self.capacity, L.stream_handle(stream)), "tspm_classify_update")

    def fetch(self):
        """(confusion [G,K,K] int64, per-batch losses [batches] float32, samples) — one sync."""
        cnt = self.counters.cpu()
        b = int(cnt[0])
        if b > self.capacity:
            raise L.TspmError(f"loss log overflow: {b} batches > capacity {self.capacity}")
        return self.conf.cpu().numpy(), self.loss_log[:b].cpu().numpy(), int(cnt[1])

    @staticmethod
    def mean_loss(losses: np.ndarray) -> float:
        """np.mean over the per-batch Python floats, as train_epoch / validate_epoch do
        (train_multimodal.py:491,541)."""
        return float(np.mean([float(x) for x in losses])) if len(losses) else float("nan")


# metric functions the reference's YAMLs name from its own ``metrics`` package (MML_Suite/metrics/__init__.py),
# restated in this package (the reference is not importable on the GPU box)
REFERENCE_METRICS = {
    "metrics.msa_binary_classification": ("msa_metrics", "msa_binary_classification"),   # metrics/msa.py:44-92
    "metrics.msa.msa_binary_classification": ("msa_metrics", "msa_binary_classification"),
}


def _resolve(path: str) -> Callable:
    if path in REFERENCE_METRICS:
        mod, fn = REFERENCE_METRICS[path]
        return getattr(importlib.import_module(f"{__package__}.{mod}"), fn)
    if path in ("metrics.confusion_matrix_from_logits", "metrics.msa.confusion_matrix_from_logits"):
        path = "sklearn.metrics.confusion_matrix"  # metrics/msa.py:40-41: the same call
    mod, fn = path.rsplit(".", 1)
    return getattr(importlib.import_module(mod), fn)


def compressed(conf: np.ndarray):
    """(y_true, y_pred, weight) with one entry per non-zero confusion cell, row-major."""
    t, p = np.nonzero(conf)
    return t.astype(np.int64), p.astype(np.int64), conf[t, p].astype(np.int64)


def evaluate(fn_path: str, kwargs: Dict[str, Any], conf: np.ndarray):
    """Value of metric ``fn_path(y_true, y_pred, **kwargs)`` over the samples counted in ``conf``."""
    fn = _resolve(fn_path)
    t, p, w = compressed(conf)
    if fn_path in REFERENCE_METRICS:  # not sklearn: the expanded arrays
        return fn(np.repeat(t, w), np.repeat(p, w), **kwargs)
    if fn_path.rsplit(".", 1)[1] in CONFUSION_ONLY and "sample_weight" not in kwargs:
        return fn(t, p, sample_weight=w, **kwargs)
    return fn(np.repeat(t, w), np.repeat(p, w), **kwargs)


class DeviceMetricRecorder:
    """``MetricRecorder.calculate_all_groups`` results (same keys: ``f"{metric}_{PATTERN}"``, e.g.
    ``accuracy_AI``, ``ConfusionMatrix_A``; metric_recorder.py:147-234) from a :class:`ClassificationLog`.

    ``config`` is the reference's ``MetricConfig`` (or anything with ``.metrics`` / ``.groups``), or a
    plain ``{"metrics": …, "groups": …}`` dict as in the YAML."""

    def __init__(self, config, log: ClassificationLog):
        metrics = config["metrics"] if isinstance(config, dict) else config.metrics
        groups = config.get("groups", {}) if isinstance(config, dict) else config.groups
        self.metrics = OrderedDict((k, (v["function"], dict(v.get("kwargs", {})))) for k, v in metrics.items())
        self.groups = {g: list(ms) for g, ms in groups.items()}
        self.log = log
        self.current_results: Dict[str, Dict[str, Any]] = {}

    def reset(self) -> None:
        self.log.reset()
        self.current_results.clear()

    def calculate_metrics_for_group(self, group_name: str, epoch: Optional[int] = None,
                                    loss: Optional[float] = None, conf: Optional[np.ndarray] = None) -> Dict[str, Any]:
        if group_name not in self.groups:
            raise ValueError(f"Unknown metric group: {group_name}")
        if conf is None:
            conf = self.log.fetch()[0]
        results: Dict[str, Any] = {"loss": loss} if loss is not None else {}
        # patterns in sorted name order (the reference keeps first-seen order; values are identical)
        for gi, pattern in sorted(enumerate(self.log.groups), key=lambda x: x[1]):
            c = conf[gi]
            if c.sum() == 0:
                continue
            tag = pattern.replace("z", "").upper()
            for name in self.groups[group_name]:
                if name not in self.metrics:
                    continue
                path, kw = self.metrics[name]
                try:
                    value = evaluate(path, kw, c)
                except (ImportError, AttributeError):
                    raise
                except Exception as e:  # metric_recorder.py:199-203: a failing metric is reported and skipped
                    print(f"Error calculating metric {name}: {e}")
                    logging.getLogger(__name__).error(f"Metric calculation error - {name}: {e}")
                    continue
                if isinstance(value, dict):
                    for k, v in value.items():
                        results[f"{name}_{k}_{tag}"] = v
                else:
                    results[f"{name}_{tag}"] = value
        self.current_results[group_name] = results
        return results

    def calculate_all_groups(self, epoch: Optional[int] = None, loss: Optional[float] = None) -> Dict[str, Dict]:
        conf = self.log.fetch()[0]
        return {g: self.calculate_metrics_for_group(g, epoch, loss, conf) for g in self.groups}

    def get_group_result(self, group_name: str, metric_name: str, default: Any = None) -> Any:
        return self.current_results.get(group_name, {}).get(metric_name, default)
