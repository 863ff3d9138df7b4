"""Monomodal encoder pre-training on the HIP path (BASELINE.json configs[1]:
ResNet18 audio encoder, batch 256, one MI355X).

Drop-in for ``MonomodalEncoder`` of MML_Suite/train_monomodal.py:64-418 — the wrapper that
train_monomodal.py builds around the YAML's encoder (``!ResNet18`` audio / ``!ResNet34`` image,
configs/avmnist/mono/train_{audio,image}_encoder_resnet.yaml) with ``classifier = nn.Linear(output_dim,
num_classes)``.  The best encoder's ``state_dict`` is saved as ``encoder_{modality}_best.pth``, the file the
pretrained late-fusion config loads (train_monomodal.py:789-802, train_multimodal.py:156-204).

* :class:`MonomodalEncoder` — same constructor, attribute names (``encoder``, ``classifier``),
  ``state_dict`` keys, ``forward`` / ``get_encoder`` / ``train_step`` / ``validation_step`` signatures and
  return dicts (``{"loss", "metrics": {"loss", "accuracy"}}``) as the reference.
* :class:`FusedMonoStep` — ``train_step`` as one HIP graph: encoder forward (libtspm schedule) →
  classifier → cross-entropy → classifier backward → encoder backward → FusedAdam, with the
  ``argmax(logits, 1)`` predictions written on the device (``tspm_classify_update_ex``, logits mode).
* :class:`FusedMonoEvalStep` — ``validation_step`` as one HIP graph (eval-mode BatchNorm).
* :func:`select_modality_key` — the reference's choice of the batch key (train_monomodal.py:103-128).
* :class:`MonoEpochRunner` / :func:`fit_monomodal` — the epoch loop of ``train_monomodal``
  (train_monomodal.py:536-884) on those steps, one host read per epoch.
"""
from __future__ import annotations

import math
import os
import time
from pathlib import Path
from typing import Any, Dict, Iterable, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib as L
from ._lib import linear_bwd
from .engine import EncoderEngine, prepare_encoder_layout
from .metrics import ClassificationLog, DeviceMetricRecorder
from .optim import FusedAdam
from .step import _ce_weight, shared_batches_tracked

ARGMAX_LOGITS = 1  # TSPM_ARGMAX_LOGITS (include/tspm.h)
# keys train_monomodal.py:110-112 never treats as a modality (+ this package's device pattern index)
_RESERVED = ("labels", "label", "genres", "imdb_ids", "pattern_name", "missing_masks", "sample_idx", "pattern_ids")


def _exp_name(config) -> str:
    if isinstance(config, str):
        return config
    exp = getattr(config, "experiment", None)
    return str(getattr(exp, "name", "") or "")


def select_modality_key(batch: Dict[Any, Any], experiment_name: str = ""):
    """train_monomodal.py:103-128: skip the bookkeeping keys; with "AVMNIST_Image_Encoder" /
    "AVMNIST_Audio_Encoder" in the experiment name take the first key whose ``str`` names IMAGE /
    AUDIO, otherwise the LAST remaining key.  ``str(Modality.X)`` comes from the un-vendored
    ``modalities`` package (unpinned), so the name test is case-insensitive here."""
    key = None
    for k in batch.keys():
        ks = str(k)
        if ks in _RESERVED or ks.endswith("_missing_index") or ks.endswith("_reverse"):
            continue
        up = ks.upper()
        if "AVMNIST_Image_Encoder" in experiment_name and "IMAGE" in up:
            return k
        if "AVMNIST_Audio_Encoder" in experiment_name and "AUDIO" in up:
            return k
        key = k
    if key is None:
        raise ValueError(f"No modality data found in batch. Available keys: {list(batch.keys())}")
    return key


def _as_tensor(raw) -> torch.Tensor:
    """train_monomodal.py:137-191: a tensor, or a list of tensors / numbers / arrays (stacked).  Lists
    of file paths are not taken: load the corpus with tspm_amd.data.AVMNIST (HBM-resident)."""
    if torch.is_tensor(raw):
        return raw
    if isinstance(raw, list):
        if raw and isinstance(raw[0], str):
            raise L.TspmError("file-path batches: load the corpus with tspm_amd.data.AVMNIST instead")
        items = []
        for it in raw:
            if torch.is_tensor(it):
                items.append(it)
            elif isinstance(it, (int, float)):
                items.append(torch.tensor(it))
            elif isinstance(it, np.ndarray):
                items.append(torch.from_numpy(it))
            else:
                raise TypeError(f"Unsupported data type: {type(it)}")
        return torch.stack(items)
    raise TypeError(f"Unsupported modality data type: {type(raw)}")


def _labels_of(batch: Dict[Any, Any]) -> torch.Tensor:
    """train_monomodal.py:196-219."""
    for k in ("label", "labels", "genres"):
        if k in batch:
            raw = batch[k]
            if isinstance(raw, list):
                if raw and isinstance(raw[0], str):
                    raise TypeError("Cannot convert string labels to tensor without label mapping")
                return torch.tensor(raw)
            return raw
    raise ValueError(f"No labels found in batch. Available keys: {list(batch.keys())}")


def _device_log(metric_recorder) -> Optional[ClassificationLog]:
    return metric_recorder.log if isinstance(metric_recorder, DeviceMetricRecorder) else None


class _LinearFn(torch.autograd.Function):
    """``classifier`` (nn.Linear) on libtspm: tspm_linear_fwd / _bwd_weight / _bwd_data."""

    @staticmethod
    def forward(ctx, x, w, b):
        n, fin = x.shape
        fout = w.shape[0]
        y = torch.empty(n, fout, device=x.device, dtype=torch.float32)
        L.check(L.lib().tspm_linear_fwd(n, fin, fout, x.data_ptr(), fin, w.data_ptr(), b.data_ptr(), 0, None, 1.0,
                                        y.data_ptr(), fout, L.stream_handle()), "classifier fwd")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous().float()
        n, fin = x.shape
        fout = w.shape[0]
        lib, sh = L.lib(), L.stream_handle()
        gw, gb, gx = torch.empty_like(w), torch.empty(fout, device=g.device), torch.empty_like(x)
        L.check(lib.tspm_linear_bwd_weight(n, fin, fout, x.data_ptr(), fin, g.data_ptr(), fout, gw.data_ptr(),
                                           gb.data_ptr(), sh), "classifier wgrad")
        L.check(lib.tspm_linear_bwd_data(n, fin, fout, g.data_ptr(), fout, w.data_ptr(), gx.data_ptr(), fin, sh),
                "classifier dgrad")
        return gx, gw, gb


class _MonoBuffers:
    """Static device buffers + graph bookkeeping shared by the fused train and eval steps."""

    def _init_buffers(self, model, x_shape: Tuple[int, ...], log) -> None:
        enc, cls = model.encoder, model.classifier
        self.model, self.log = model, log
        dev = next(model.parameters()).device
        self.device = dev
        self.N = int(x_shape[0])
        self.hid, self.K = cls.in_features, cls.out_features
        if self.hid != enc.hidden_dim:
            raise L.TspmError(f"classifier input {self.hid} != encoder hidden_dim {enc.hidden_dim}")
        f32 = dict(device=dev, dtype=torch.float32)
        self.X = torch.zeros(x_shape, **f32)
        self.labels = torch.zeros(self.N, dtype=torch.int64, device=dev)
        self.emb = torch.empty(self.N, self.hid, **f32)
        self.logits = torch.empty(self.N, self.K, **f32)
        self.loss = torch.zeros(1, **f32)
        self.preds = torch.zeros(self.N, dtype=torch.int64, device=dev)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._graph_log = None
        self.calls = 0

    def _classify(self, lib, sh: int) -> None:
        log = self.log
        L.check(lib.tspm_classify_update_ex(
            self.N, self.K, self.logits.data_ptr(), self.labels.data_ptr(), None, len(log.groups) if log else 1,
            log.conf.data_ptr() if log else None, self.preds.data_ptr(), self.loss.data_ptr(),
            log.loss_log.data_ptr() if log else None, log.counters.data_ptr() if log else None,
            log.capacity if log else 0, ARGMAX_LOGITS, sh), "classify_update")

    def _replay_or_enqueue(self) -> None:
        if self._graph_log is not self.log:  # the metrics log is baked into the captured graph
            self.graph, self._graph_log = None, self.log
        if not self.use_graph or self.calls == 0:
            self._enqueue()
        else:
            if self.graph is None:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with L.graph_capture(g):
                    self._enqueue()
                self.graph = g
            self.graph.replay()
        self.calls += 1

    def load_batch(self, x: torch.Tensor, labels: torch.Tensor) -> None:
        if x.data_ptr() != self.X.data_ptr():
            self.X.copy_(x.reshape(self.X.shape), non_blocking=True)
        if labels.data_ptr() != self.labels.data_ptr():
            self.labels.copy_(labels.reshape(-1), non_blocking=True)

    def batch_accuracy(self) -> torch.Tensor:
        """mean(pred == label) of the last batch, as a device scalar (no host synchronisation)."""
        return (self.preds == self.labels).float().mean()


class FusedMonoStep(_MonoBuffers):
    """MonomodalEncoder.train_step (train_monomodal.py:97-260) as one HIP graph:

        encoder fwd → classifier → CE → argmax(logits) → classifier bwd → encoder bwd → FusedAdam

    Weight gradients go straight into FusedAdam's flat gradient buffer (overwrite — no zero_grad
    pass).  First call eager, second captures, later calls copy the batch into the static buffers
    (no copy when the caller gathered into them) and replay."""

    def __init__(self, model, optimizer: FusedAdam, loss_functions, x_shape, use_graph: bool = True, log=None):
        self.ce_weight = _ce_weight(loss_functions)
        if self.ce_weight is None:
            raise L.TspmError("FusedMonoStep: the loss group must be a single cross-entropy term")
        if not isinstance(optimizer, FusedAdam):
            raise L.TspmError("FusedMonoStep needs tspm_amd.FusedAdam")
        x_shape = tuple(int(v) for v in x_shape)
        self._init_buffers(model, x_shape, log)
        self.opt = optimizer
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        model.train()
        prepare_encoder_layout(model.encoder)
        for p in model.parameters():
            if p.requires_grad and p.grad is None:
                raise L.TspmError("FusedMonoStep: parameter without a FusedAdam gradient view")
        self.eng = EncoderEngine(model.encoder, self.N, x_shape[-2], x_shape[-1], self.device)
        f32 = dict(device=self.device, dtype=torch.float32)
        self.dlogits = torch.empty(self.N, self.K, **f32)
        self.demb = torch.empty(self.N, self.hid, **f32)
        self.stats = torch.zeros(4, **f32)
        self.nbt = shared_batches_tracked(model, self.device)
        self._sig = (id(optimizer), id(loss_functions), x_shape)

    def matches(self, x: torch.Tensor, optimizer, loss_functions) -> bool:
        return self._sig == (id(optimizer), id(loss_functions), tuple(x.shape))

    def _enqueue(self) -> None:
        lib = L.lib()
        sh = torch.cuda.current_stream().cuda_stream
        n, hid, K = self.N, self.hid, self.K
        cls = self.model.classifier
        self.eng.forward(self.X, self.emb, hid, train=True, bump_batches_tracked=False)
        L.check(lib.tspm_linear_fwd(n, hid, K, self.emb.data_ptr(), hid, cls.weight.data_ptr(), cls.bias.data_ptr(), 0,
                                    None, 1.0, self.logits.data_ptr(), K, sh), "classifier fwd")
        L.check(lib.tspm_cross_entropy(n, K, self.logits.data_ptr(), self.labels.data_ptr(), self.loss.data_ptr(),
                                       self.dlogits.data_ptr(), self.ce_weight, self.stats.data_ptr(), sh),
                "cross_entropy")
        self._classify(lib, sh)
        linear_bwd(n, hid, K, self.emb.data_ptr(), hid, self.dlogits.data_ptr(), K, cls.weight.data_ptr(),
                   cls.weight.grad.data_ptr(), cls.bias.grad.data_ptr(), self.demb.data_ptr(), hid, sh)
        self.eng.backward(self.demb, hid)
        L.counters_add(self.nbt)
        self.opt.launch(sh)

    def run(self) -> None:
        """One training step on the batch in the static input buffers."""
        self.model.train()
        self.opt.sync_hyper()
        self._replay_or_enqueue()
        self.opt.note_steps(1)

    def step(self, x: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
        self.load_batch(x, labels)
        self.run()
        return {"loss": self.loss, "logits": self.logits, "preds": self.preds}


class FusedMonoEvalStep(_MonoBuffers):
    """MonomodalEncoder.validation_step (train_monomodal.py:262-418) as one HIP graph: eval-mode
    encoder forward (BatchNorm running statistics), classifier, weighted CE, argmax(logits)."""

    def __init__(self, model, loss_functions, x_shape, log=None, use_graph: bool = True):
        self.ce_weight = _ce_weight(loss_functions)
        if self.ce_weight is None:
            raise L.TspmError("FusedMonoEvalStep: the loss group must be a single cross-entropy term")
        x_shape = tuple(int(v) for v in x_shape)
        self._init_buffers(model, x_shape, log)
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        self.eng = model.encoder.engine_for(self.X)

    def _enqueue(self) -> None:
        lib = L.lib()
        sh = torch.cuda.current_stream().cuda_stream
        n, hid, K = self.N, self.hid, self.K
        cls = self.model.classifier
        self.eng.forward(self.X, self.emb, hid, train=False)
        L.check(lib.tspm_linear_fwd(n, hid, K, self.emb.data_ptr(), hid, cls.weight.data_ptr(), cls.bias.data_ptr(), 0,
                                    None, 1.0, self.logits.data_ptr(), K, sh), "eval classifier")
        L.check(lib.tspm_cross_entropy(n, K, self.logits.data_ptr(), self.labels.data_ptr(), self.loss.data_ptr(),
                                       None, self.ce_weight, None, sh), "eval cross_entropy")
        self._classify(lib, sh)

    def run(self) -> None:
        self.model.eval()
        self._replay_or_enqueue()

    def step(self, x: torch.Tensor, labels: torch.Tensor) -> Dict[str, torch.Tensor]:
        self.load_batch(x, labels)
        self.run()
        return {"loss": self.loss, "logits": self.logits, "preds": self.preds}


class MonomodalEncoder(nn.Module):
    """train_monomodal.py:64-95 drop-in: ``encoder`` + ``classifier``, executed on libtspm."""

    def __init__(self, encoder: nn.Module, output_dim: int, num_classes: int):
        super().__init__()
        self.encoder = encoder
        self.classifier = nn.Linear(output_dim, num_classes)
        self._fused: Optional[FusedMonoStep] = None
        self._eval_steps: Dict[Tuple, FusedMonoEvalStep] = {}

    def forward(self, x):
        if isinstance(x, list):
            x = torch.stack(x)
        encoded = self.encoder(x)
        if encoded.dim() > 2:  # train_monomodal.py:83-86
            encoded = encoded.reshape(encoded.shape[0], -1)
        if not encoded.is_cuda:
            raise L.TspmError("MonomodalEncoder (tspm_amd) runs on the MI355X only (there is no CPU fallback)")
        return _LinearFn.apply(encoded.contiguous().float(), self.classifier.weight, self.classifier.bias)

    def get_encoder(self) -> nn.Module:
        return self.encoder

    # -- steps ------------------------------------------------------------------------------------
    def _inputs(self, batch, config, device):
        key = select_modality_key(batch, _exp_name(config))
        raw = batch[f"{key}_original"] if f"{key}_original" in batch else batch[key]
        x = _as_tensor(raw).to(device, non_blocking=True).float()
        labels = _labels_of(batch).to(device, non_blocking=True)
        return key, x, labels

    def _hip_encoder(self) -> bool:
        from .modules import ResNetEncoder
        return isinstance(self.encoder, ResNetEncoder)

    def train_step_fused(self, x: torch.Tensor, labels: torch.Tensor, optimizer, loss_functions,
                         log: Optional[ClassificationLog] = None) -> FusedMonoStep:
        """Run one fused step on device tensors and return the step (its loss / logits / preds buffers)."""
        if self._fused is None or not self._fused.matches(x, optimizer, loss_functions):
            self._fused = FusedMonoStep(self, optimizer, loss_functions, tuple(x.shape))
        self._fused.log = log
        self._fused.step(x, labels)
        return self._fused

    def eval_step_for(self, loss_functions, x_shape, log=None) -> FusedMonoEvalStep:
        key = tuple(x_shape)
        st = self._eval_steps.get(key)
        if st is None or st.ce_weight != _ce_weight(loss_functions):
            st = FusedMonoEvalStep(self, loss_functions, key, log)
            self._eval_steps[key] = st
        st.log = log
        return st

    def train_step(self, batch, optimizer, loss_functions, device, metric_recorder, config=None, **kwargs):
        """train_monomodal.py:97-260.  Fused HIP graph with FusedAdam and the single cross-entropy loss
        group; otherwise the reference's autograd sequence on the HIP encoder / classifier."""
        key, x, labels = self._inputs(batch, config, device)
        dlog = _device_log(metric_recorder)
        fused = (not os.environ.get("TSPM_DISABLE_FUSED_STEP") and isinstance(optimizer, FusedAdam)
                 and self._hip_encoder() and _ce_weight(loss_functions) is not None and x.is_cuda
                 and labels.dim() == 1 and x.dim() in (3, 4))
        if fused:
            st = self.train_step_fused(x, labels, optimizer, loss_functions, dlog)
            loss_t, preds = st.loss, st.preds
        else:
            optimizer.zero_grad()
            logits = self.forward(x)
            loss_t = loss_functions(logits, labels)["total_loss"]
            loss_t.backward()
            optimizer.step()
            with torch.no_grad():
                preds = torch.argmax(logits, dim=1) if labels.dim() == 1 else torch.sigmoid(logits) > 0.5
        return self._finish(metric_recorder, dlog, key, preds, labels, loss_t)

    def validation_step(self, batch, loss_functions, device, metric_recorder, config=None, **kwargs):
        """train_monomodal.py:262-418 (the caller puts the model in eval mode, as train_monomodal does)."""
        with torch.no_grad():
            key, x, labels = self._inputs(batch, config, device)
            dlog = _device_log(metric_recorder)
            if (not self.training and self._hip_encoder() and _ce_weight(loss_functions) is not None and x.is_cuda
                    and labels.dim() == 1 and x.dim() in (3, 4)):
                st = self.eval_step_for(loss_functions, tuple(x.shape), dlog)
                st.step(x, labels)
                loss_t, preds = st.loss, st.preds
            else:
                logits = self.forward(x)
                loss_t = loss_functions(logits, labels)["total_loss"]
                preds = torch.argmax(logits, dim=1) if labels.dim() == 1 else torch.sigmoid(logits) > 0.5
            return self._finish(metric_recorder, dlog, key, preds, labels, loss_t)

    @staticmethod
    def _finish(metric_recorder, dlog, key, preds, labels, loss_t):
        with torch.no_grad():
            if metric_recorder is not None and dlog is None:
                for group_name in metric_recorder.config.groups:
                    metric_recorder.update_group(group_name=group_name, predictions=preds, targets=labels,
                                                 modality=str(key))
            loss = float(loss_t.item() if torch.is_tensor(loss_t) else loss_t)
            metrics = {"loss": loss}
            if labels.dim() == 1:
                metrics["accuracy"] = (preds == labels).float().mean().item()
        return {"loss": loss, "metrics": metrics}


# ------------------------------------------------------------------------------------------------
# Epoch harness (train_monomodal.py:536-884)
# ------------------------------------------------------------------------------------------------
def modality_of_experiment(name: str) -> str:
    """train_monomodal.py:793-798: the first of image/text/audio/video among the name's '_' parts."""
    for part in name.lower().split("_"):
        if part in ("image", "text", "audio", "video"):
            return part
    return "unknown"


class MonoEpochRunner:
    """Train / validation epochs of train_monomodal (train_monomodal.py:658-753) on the fused steps.
    Per batch: the batch (device tensors, e.g. a data.DeviceLoader's gather) + one graph replay; the
    per-batch losses and confusion counts stay on the device (``tspm_classify_update_ex``) and per-batch
    accuracies are device scalars, all read once per epoch.  Epoch dict = the reference's
    ``avg_*_metrics``: ``loss`` / ``accuracy`` = np.mean over the batches, updated with the flattened
    metric-recorder results (keys ``f"{metric}_{MODALITY}"``)."""

    def __init__(self, model: MonomodalEncoder, optimizer, loss_functions, experiment_name: str,
                 metric_config=None, device=None, log_capacity: int = 1 << 16):
        from .harness import AVMNIST_METRICS
        self.model, self.optimizer, self.loss_functions = model, optimizer, loss_functions
        self.experiment_name = experiment_name
        self.device = device or next(model.parameters()).device
        self.metric_config = metric_config or AVMNIST_METRICS
        self.log_capacity = log_capacity
        self.log: Optional[ClassificationLog] = None
        self.recorder: Optional[DeviceMetricRecorder] = None
        self.train_steps: Dict[Tuple, FusedMonoStep] = {}

    def _ensure_log(self, key) -> None:
        if self.log is None:
            self.log = ClassificationLog(self.device, groups=(str(key),), capacity=self.log_capacity)
            self.recorder = DeviceMetricRecorder(self.metric_config, self.log)

    def _finish(self, t0: float, accs: List[torch.Tensor]) -> Tuple[Dict[str, Any], float]:
        conf, losses, _ = self.log.fetch()  # the epoch's host synchronisation
        acc = torch.stack(accs).cpu().tolist() if accs else []
        mean = ClassificationLog.mean_loss(losses)
        out: Dict[str, Any] = {"loss": mean}
        if acc:
            out["accuracy"] = float(np.mean(acc))
        for g in self.recorder.groups:
            out.update(self.recorder.calculate_metrics_for_group(g, loss=mean, conf=conf))
        return out, time.time() - t0

    def _batches(self, loader):
        started = False
        for b in loader:
            key, x, lab = self.model._inputs(b, self.experiment_name, self.device)
            self._ensure_log(key)
            if not started:
                self.log.reset()
                started = True
            yield x, lab
        if not started:
            raise ValueError("empty loader")

    def train_epoch(self, loader: Iterable[Dict[str, Any]]):
        """→ (epoch metrics dict, seconds)."""
        t0 = time.time()
        accs: List[torch.Tensor] = []
        self.model.train()
        for x, lab in self._batches(loader):
            shape = tuple(x.shape)
            st = self.train_steps.get(shape)
            if st is None:
                st = FusedMonoStep(self.model, self.optimizer, self.loss_functions, shape)
                self.train_steps[shape] = st
            st.log = self.log
            st.step(x, lab)
            accs.append(st.batch_accuracy())
        return self._finish(t0, accs)

    @torch.no_grad()
    def validate_epoch(self, loader: Iterable[Dict[str, Any]]):
        t0 = time.time()
        accs: List[torch.Tensor] = []
        self.model.eval()
        for x, lab in self._batches(loader):
            st = self.model.eval_step_for(self.loss_functions, tuple(x.shape), self.log)
            st.step(x, lab)
            accs.append(st.batch_accuracy())
        return self._finish(t0, accs)


def fit_monomodal(model: MonomodalEncoder, optimizer, loss_functions, loaders: Dict[str, Any], epochs: int, *,
                  experiment_name: str, model_output_path=None, save_metric: str = "loss",
                  early_stopping: bool = True, patience: int = 10, scheduler_factory=None,
                  metric_config=None) -> Dict[str, Any]:
    """``train_monomodal`` (train_monomodal.py:536-884) on the HIP steps: per epoch train → validate →
    best by ``save_metric`` (strictly lower loss / higher accuracy, no min_delta) → on improvement
    ``epoch_{n}.pth`` + ``best.pth`` (model + optimizer state) and ``encoder_{modality}_best.pth``
    (the encoder's state_dict, the pretrained late-fusion hand-off) → early stopping after
    ``patience`` epochs without improvement → ``scheduler_factory(optimizer)`` built afresh and stepped
    every epoch (the reference re-creates its scheduler each epoch, train_monomodal.py:810-815, so a
    ReduceLROnPlateau never accumulates patience — reproduced, not fixed) → test on the best model."""
    from .harness import CheckpointManager
    runner = MonoEpochRunner(model, optimizer, loss_functions, experiment_name, metric_config)
    out_dir = Path(model_output_path) if model_output_path is not None else None
    ckpt = CheckpointManager(out_dir, save_metric, "minimize" if save_metric == "loss" else "maximize") \
        if out_dir is not None else None
    history: Dict[str, Any] = {"metrics_history": {"train": [], "validation": [], "test": []},
                               "timing_history": {"train": [], "validation": []}}
    best_loss, best_acc, wait = math.inf, 0.0, 0
    modality = modality_of_experiment(experiment_name)
    encoder_path = None
    for epoch in range(epochs):
        tr, tr_t = runner.train_epoch(loaders["train"])
        va, va_t = runner.validate_epoch(loaders["validation"])
        history["metrics_history"]["train"].append(tr)
        history["metrics_history"]["validation"].append(va)
        history["timing_history"]["train"].append(tr_t)
        history["timing_history"]["validation"].append(va_t)
        cur_loss, cur_acc = va["loss"], va.get("accuracy", 0)
        is_best = False
        if save_metric == "loss" and cur_loss < best_loss:
            best_loss, is_best, wait = cur_loss, True, 0
        elif save_metric != "loss" and cur_acc > best_acc:
            best_acc, is_best, wait = cur_acc, True, 0
        else:
            wait += 1
        if is_best and ckpt is not None:
            ckpt.save_checkpoint(model, optimizer, None, epoch, va, is_best=True)
            encoder_path = out_dir / f"encoder_{modality}_best.pth"
            torch.save(model.get_encoder().state_dict(), encoder_path)
        if early_stopping and wait >= patience:
            break
        if scheduler_factory is not None:
            sched = scheduler_factory(optimizer)
            if isinstance(sched, torch.optim.lr_scheduler.ReduceLROnPlateau):
                sched.step(cur_loss)
            else:
                sched.step()
    if "test" in loaders:
        if ckpt is not None and (ckpt.model_dir / "best.pth").exists():
            ckpt.load_checkpoint(model, load_best=True)
        te, te_t = runner.validate_epoch(loaders["test"])
        history["metrics_history"]["test"] = te
        history["timing_history"]["test"] = [te_t]
    history["best_val_loss"] = best_loss
    history["best_val_accuracy"] = best_acc
    history["encoder_path"] = str(encoder_path) if encoder_path is not None else None
    return history
