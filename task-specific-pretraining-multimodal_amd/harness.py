"""Epoch harness: train / validate epochs and the fit loop of MML_Suite/train_multimodal.py on the
fused HIP steps, with the epoch's bookkeeping on the device.

Reference (``MML_Suite/``):
  train_epoch            train_multimodal.py:438-491  per batch model.train_step → loss.item(); mean
  validate_epoch         train_multimodal.py:494-541  per batch model.validation_step → loss.item(); mean
  check_early_stopping   train_multimodal.py:329-377
  _train_loop            train_multimodal.py:554-791  epochs: metrics reset → train → calculate_all_groups
                         → validate → calculate_all_groups → epoch_metrics.json → early stopping →
                         CheckpointManager.save_checkpoint(epoch_{n}.pth, best.pth) → scheduler.step(val loss)
  test                   train_multimodal.py:866-917  load best.pth, validate_epoch on each test split
  CheckpointManager      experiment_utils/checkpoints.py:13-120

What differs is where the per-batch work happens: the reference synchronises on every batch
(``loss.item()`` and the predictions' ``.cpu()``); here each batch is ONE gather launch
(data.DeviceLoader writing into the step's static inputs) plus ONE graph replay that also records
the batch loss and the confusion counts (tspm_classify_update), and the host reads the epoch's
losses and counts once.  Epoch loss = ``np.mean`` of the per-batch fp32 losses as Python floats, as
the reference computes it; metrics via metrics.DeviceMetricRecorder (same keys and values as the
reference's MetricRecorder).
"""
from __future__ import annotations

import json
import time
from pathlib import Path
from typing import Any, Dict, Iterable, Optional, Tuple

import numpy as np
import torch

from . import _lib as L
from .metrics import ClassificationLog, DeviceMetricRecorder
from .modules import modality_key
from .step import FusedEvalStep, FusedTrainStep

# the AVMNIST YAML's metric block (configs/avmnist/centralised/train_avmnist_resnet.yaml:105-166)
AVMNIST_METRICS = {
    "metrics": {
        "accuracy": {"function": "sklearn.metrics.accuracy_score", "kwargs": {}},
        "balanced_accuracy": {"function": "sklearn.metrics.balanced_accuracy_score", "kwargs": {}},
        **{f"{m}_{avg}": {"function": f"sklearn.metrics.{fn}", "kwargs": {"average": avg, "zero_division": 0}}
           for m, fn in (("f1", "f1_score"), ("precision", "precision_score"), ("recall", "recall_score"))
           for avg in ("macro", "micro", "weighted")},
        "ConfusionMatrix": {"function": "sklearn.metrics.confusion_matrix", "kwargs": {"labels": list(range(10))}},
    },
    "groups": {"classification": ["accuracy", "balanced_accuracy", "f1_macro", "f1_micro", "f1_weighted",
                                  "precision_macro", "precision_micro", "precision_weighted", "recall_macro",
                                  "recall_micro", "recall_weighted", "ConfusionMatrix"]},
}


# the MOSI / MOSEI UTT-Fusion YAMLs' metric block (configs/mosi/centralised/utt_fusion_base_training.yaml:151-162)
MOSI_METRICS = {
    "metrics": {
        "MSA": {"function": "metrics.msa_binary_classification", "kwargs": {}, "level": "epoch"},
        "ConfusionMatrix": {"function": "sklearn.metrics.confusion_matrix", "kwargs": {"labels": [0, 1, 2]},
                            "level": "epoch"},
    },
    "groups": {"classification": ["MSA", "ConfusionMatrix"]},
}


def check_early_stopping(val_metrics: Dict[str, Any], best_metrics: Optional[Dict[str, Any]], patience: int,
                         min_delta: float, wait: int, mode: str = "minimize",
                         target_metric: str = "loss") -> Tuple[bool, bool, int]:
    """train_multimodal.py:329-377: (is_best, should_continue, wait)."""
    if best_metrics is None:
        return True, True, 0
    value, best = val_metrics.get(target_metric), best_metrics.get(target_metric)
    if value is None or best is None:
        raise ValueError(f"Metric '{target_metric}' not found in val_metrics or best_metrics.")
    if (mode == "minimize" and value < best - min_delta) or (mode == "maximize" and value > best + min_delta):
        return True, True, 0
    wait += 1
    return False, wait < patience, wait


class CheckpointManager:
    """experiment_utils/checkpoints.py:13-120 — same files (``epoch_{n}.pth``, ``best.pth``) and dict
    keys (``model_state_dict``, ``optimizer_state_dict``, ``scheduler_state_dict``); state_dict keys and
    OIHW shapes are the reference's, so checkpoints load on either side."""

    def __init__(self, model_dir, save_metric: str = "loss", mode: str = "minimize", device: str = "cuda"):
        self.model_dir = Path(model_dir)
        self.save_metric, self.mode, self.device = save_metric, mode, device
        self.best_metric = float("inf") if mode == "minimize" else float("-inf")
        self.best_epoch = -1
        self.model_dir.mkdir(parents=True, exist_ok=True)

    def is_better(self, current: float) -> bool:
        return current < self.best_metric if self.mode == "minimize" else current > self.best_metric

    def save_checkpoint(self, model, optimizer, scheduler, epoch: int, metrics: Dict[str, float],
                        is_best: bool = False) -> None:
        state = {"model_state_dict": model.state_dict(), "optimizer_state_dict": optimizer.state_dict()}
        if scheduler is not None:
            state["scheduler_state_dict"] = scheduler.state_dict()
        torch.save(state, self.model_dir / f"epoch_{epoch}.pth")
        if is_best:
            torch.save(state, self.model_dir / "best.pth")
        value = metrics[self.save_metric]
        if self.is_better(value):
            self.best_metric, self.best_epoch = value, epoch

    def load_checkpoint(self, model, optimizer=None, scheduler=None, epoch: Optional[int] = None,
                        load_best: bool = False) -> Dict[str, Any]:
        name = "best.pth" if load_best else (f"epoch_{epoch}.pth" if epoch is not None else "last.pth")
        ck = torch.load(self.model_dir / name, map_location=self.device, weights_only=True)
        model.load_state_dict(ck["model_state_dict"])
        if optimizer is not None and "optimizer_state_dict" in ck:
            optimizer.load_state_dict(ck["optimizer_state_dict"])
        if scheduler is not None and "scheduler_state_dict" in ck:
            scheduler.load_state_dict(ck["scheduler_state_dict"])
        return ck


class EpochRunner:
    """train_epoch / validate_epoch on the fused steps.  ``loader`` yields collate_fn-style batch dicts
    on the device (data.DeviceLoader / the drop-in DataLoader); batches of the runner's size are fed
    through the static buffers of one captured graph, a smaller last batch through a second one."""

    def __init__(self, model, optimizer, loss_functions, metric_config=None, device=None, log_capacity: int = 1 << 16):
        self.model, self.optimizer, self.loss_functions = model, optimizer, loss_functions
        self.device = device or next(model.parameters()).device
        self.log = ClassificationLog(self.device, capacity=log_capacity)
        self.recorder = DeviceMetricRecorder(metric_config or AVMNIST_METRICS, self.log)
        self.train_steps: Dict[int, FusedTrainStep] = {}
        self.eval_steps: Dict[int, FusedEvalStep] = {}

    def _train_step(self, n: int) -> FusedTrainStep:
        st = self.train_steps.get(n)
        if st is None:
            st = FusedTrainStep(self.model, self.optimizer, self.loss_functions, n)
            self.train_steps[n] = st
        st.log = self.log
        return st

    def _eval_step(self, n: int) -> FusedEvalStep:
        st = self.eval_steps.get(n)
        if st is None:
            st = FusedEvalStep(self.model, self.loss_functions, n, self.log)
            self.eval_steps[n] = st
        st.log = self.log
        return st

    def _unpack(self, b):
        a, i = b[modality_key(b, "audio")], b[modality_key(b, "image")]
        g = b.get("pattern_ids")
        if g is None:
            g = self.log.group_ids(b["pattern_name"])
        return a, i, b["labels"], g

    def _finish(self, t0: float, loss: Optional[float] = None):
        conf, losses, _ = self.log.fetch()  # the epoch's only host synchronisation
        mean = ClassificationLog.mean_loss(losses)
        metrics = self.recorder.calculate_metrics_for_group("classification", loss=mean, conf=conf)
        return mean, time.time() - t0, metrics, len(losses)

    def train_epoch(self, loader: Iterable[Dict[str, Any]]):
        """→ (mean batch loss, seconds, metrics dict, batches)."""
        self.log.reset()
        t0 = time.time()
        for b in loader:
            a, i, lab, g = self._unpack(b)
            self._train_step(a.shape[0]).step(a, i, lab, g)
        return self._finish(t0)

    @torch.no_grad()
    def validate_epoch(self, loader: Iterable[Dict[str, Any]]):
        self.log.reset()
        t0 = time.time()
        self.model.eval()
        for b in loader:
            a, i, lab, g = self._unpack(b)
            self._eval_step(a.shape[0]).step(a, i, lab, g)
        return self._finish(t0)


class MosiEpochRunner:
    """train_epoch / validate_epoch (train_multimodal.py:438-541) for UttFusionModel on the fused steps, over the
    seven missing-modality patterns (data/mosi.py:61-69).  A batch is a collate_fn-style dict — batch-first
    tensors, or the time-major buffers of this runner's own steps when the loader gathered into them
    (``MosiDeviceLoader`` with ``step_for`` pointed here by ``loader_for``) — or, for valid / test, the
    pattern-grouped ``{pattern: sub-batch}`` of data/mosi.py:236-251; each group is one ``validation_step`` (one
    ``FusedMosiEvalStep`` replay: its loss is one entry of the epoch's loss log, its rows go to the confusion
    counts of their pattern).  Per-pattern metrics come from ``DeviceMetricRecorder`` with the YAML's MSA and
    confusion-matrix functions (keys ``MSA_Has0_Accuracy_ATV`` ...; metric_recorder.py:147-209)."""

    def __init__(self, model, optimizer, loss_functions, metric_config=None, device=None, log_capacity: int = 1 << 16):
        from .mosi_data import PATTERNS
        self.model, self.optimizer, self.loss_functions = model, optimizer, loss_functions
        self.device = device or next(model.parameters()).device
        self.log = ClassificationLog(self.device, groups=PATTERNS, classes=3, capacity=log_capacity)
        self.recorder = DeviceMetricRecorder(metric_config or MOSI_METRICS, self.log)
        self.eval_steps: Dict[Tuple[int, int], Any] = {}

    def train_step_for(self, b: int, t: int):
        st = self.model.fused_step(self.optimizer, self.loss_functions, b, t)
        if st.log is not self.log:
            st.log, st.graph = self.log, None  # the captured graph must record into this log
        return st

    def eval_step_for(self, b: int, t: int):
        """The cached FusedMosiEvalStep for (b, t) — rebuilt when the model's engine for that shape is no longer
        the one it captured (``UttFusionModel._apply`` drops the engines on .to() / re-materialisation)."""
        from .mosi import FusedMosiEvalStep
        st = self.eval_steps.get((b, t))
        if st is None or st.eng is not self.model._engine(b, t, self.device):
            st = FusedMosiEvalStep(self.model, self.loss_functions, b, t, self.log)
            self.eval_steps[(b, t)] = st
        return st

    def loader_for(self, loader, train: bool):
        """Point a ``MosiDeviceLoader`` at this runner's steps (batches gathered straight into their inputs)."""
        if hasattr(loader, "step_for"):
            loader.step_for = self.train_step_for if train else self.eval_step_for
        return loader

    def _run(self, st, b: Dict[str, Any]) -> None:
        st.eng.groups.copy_(self.log.group_ids(b.get("pattern_name") or b["pattern_names"]), non_blocking=True)
        if b.get("time_major") and b["audio"] is st.eng.A:
            st.run()
        else:
            st.step(b["audio"], b["video"], b["text"], b["label"])

    @staticmethod
    def _shape(b: Dict[str, Any]) -> Tuple[int, int]:
        return int(b["label"].numel()), int(b.get("steps") or b["audio"].shape[1])

    @staticmethod
    def _groups(b: Dict[str, Any]):
        if "label" in b:
            return [b]
        return list(b.values())  # {pattern: sub-batch}

    def _finish(self, t0: float):
        conf, losses, _ = self.log.fetch()  # the epoch's only host synchronisation
        mean = ClassificationLog.mean_loss(losses)
        metrics = self.recorder.calculate_metrics_for_group("classification", loss=mean, conf=conf)
        return mean, time.time() - t0, metrics, len(losses)

    def train_epoch(self, loader: Iterable[Dict[str, Any]]):
        """→ (mean batch loss, seconds, metrics dict, batches)."""
        self.log.reset()
        t0 = time.time()
        for b in self.loader_for(loader, True):
            for g in self._groups(b):
                self._run(self.train_step_for(*self._shape(g)), g)
        return self._finish(t0)

    @torch.no_grad()
    def validate_epoch(self, loader: Iterable[Dict[str, Any]]):
        self.log.reset()
        t0 = time.time()
        self.model.eval()
        try:
            for b in self.loader_for(loader, False):
                for g in self._groups(b):
                    self._run(self.eval_step_for(*self._shape(g)), g)
        finally:
            self.model.train()
        return self._finish(t0)


def runner_for(model, optimizer, loss_functions, metric_config=None):
    """The epoch runner of the model family: AVMNIST late fusion, or MOSI / MOSEI UTT-Fusion."""
    from .mosi import UttFusionModel
    if isinstance(model, UttFusionModel):
        return MosiEpochRunner(model, optimizer, loss_functions, metric_config)
    return EpochRunner(model, optimizer, loss_functions, metric_config)


def _epoch_block(loss: float, timing: float, n_batches: int, metrics: Dict[str, Any]) -> Dict[str, Any]:
    """One split's entry of epoch_metrics.json (train_multimodal.py:627-718)."""
    out: Dict[str, Any] = {"loss": loss, "timing": {"total_time": timing,
                                                    "avg_batch_time": timing / max(1, n_batches)}}
    for key, value in metrics.items():
        if key == "loss" or not isinstance(value, (int, float)):
            continue
        if key.startswith("f1_") and "_" in key:
            parts = key.split("_")
            name = parts[0] + "_" + parts[1]
            mod = parts[2] if len(parts) >= 3 else "IT"
            out.setdefault(mod, {})[name] = metrics[key]
        else:
            out.setdefault("metrics", {})[key] = value
    return out


def fit(model, optimizer, loss_functions, loaders: Dict[str, Any], epochs: int, *, metric_config=None,
        early_stopping: bool = True, patience: int = 10, min_delta: float = 1e-3, scheduler=None,
        checkpoint_dir=None, metrics_path=None, save_metric: str = "loss", mode: str = "minimize",
        on_epoch=None, fail_on_nonfinite: bool = True) -> Dict[str, Any]:
    """_train_loop + test (train_multimodal.py:554-917) for the AVMNIST late-fusion model and the MOSI / MOSEI
    UTT-Fusion model (``runner_for``; its loaders: ``mosi_data.MOSI.loader(...)``).  ``loaders``:
    "train", "validation" and optionally "test" → iterables of device batches (a DeviceLoader is
    re-iterated each epoch; call ``set_epoch`` in ``on_epoch`` for DistributedSampler order).
    ``fail_on_nonfinite``: raise FloatingPointError as soon as an epoch's mean training loss is NaN / inf
    (checked at the epoch's one host synchronisation; SURVEY §5 — the reference only turns three numpy
    RuntimeWarnings into errors, train_multimodal.py:46-60, and would keep training on NaN weights)."""
    runner = runner_for(model, optimizer, loss_functions, metric_config)
    ckpt = CheckpointManager(checkpoint_dir, save_metric, mode) if checkpoint_dir is not None else None
    history: Dict[str, Any] = {"train": [], "validation": [], "epoch_metrics": []}
    best, wait = None, 0
    mfile = Path(metrics_path) / "epoch_metrics.json" if metrics_path is not None else None
    if mfile is not None:
        mfile.parent.mkdir(parents=True, exist_ok=True)
    for epoch in range(1, epochs + 1):
        if on_epoch is not None:
            on_epoch(epoch)
        tr_loss, tr_time, tr_metrics, tr_n = runner.train_epoch(loaders["train"])
        if fail_on_nonfinite and not np.isfinite(tr_loss):
            raise FloatingPointError(f"non-finite mean training loss {tr_loss} at epoch {epoch}")
        tr_metrics = dict(tr_metrics, loss=tr_loss)
        va_loss, va_time, va_metrics, va_n = runner.validate_epoch(loaders["validation"])
        va_metrics = dict(va_metrics, loss=va_loss)
        history["train"].append(tr_metrics)
        history["validation"].append(va_metrics)
        history["epoch_metrics"].append({"epoch": epoch, "train": _epoch_block(tr_loss, tr_time, tr_n, tr_metrics),
                                         "validation": _epoch_block(va_loss, va_time, va_n, va_metrics)})
        if mfile is not None:
            with open(mfile, "w") as f:
                json.dump(history["epoch_metrics"], f, indent=4, default=lambda o: np.asarray(o).tolist())
        is_best, cont, wait = check_early_stopping(va_metrics, best, patience, min_delta, wait, mode, save_metric)
        if is_best:
            best = dict(va_metrics)
            if ckpt is not None:
                ckpt.save_checkpoint(model, optimizer, scheduler, epoch, va_metrics, is_best=True)
        if early_stopping and not cont:
            break
        if scheduler is not None:
            if isinstance(scheduler, torch.optim.lr_scheduler.ReduceLROnPlateau):
                scheduler.step(va_metrics["loss"])
            else:
                scheduler.step()
    if "test" in loaders:
        if ckpt is not None and (ckpt.model_dir / "best.pth").exists():
            ckpt.load_checkpoint(model, load_best=True)
        te_loss, te_time, te_metrics, _ = runner.validate_epoch(loaders["test"])
        history["test"] = dict(te_metrics, loss=te_loss)
    history["best"] = best
    return history
