"""Input stage of the MOSI UTT-Fusion step: the corpus resident in HBM, padded batches assembled on device.

Replaces the reference's host data path for BASELINE.json configs[4]:

    DataLoader(MOSI(...), batch_size, shuffle, collate_fn=dataset.collate_fn)       config/data_config.py:270-290
      → MultimodalSentimentDataset.__getitem__: pattern (random.choice for train,
        pattern-major for valid/test), modality × missing mask                        data/mosi.py:159-196,
                                                                                       data/base_dataset.py:61-74,91-99
      → _collate_train_batch: torch.stack(labels), pad_sequence(batch_first, 0.0)
        per modality; eval batches grouped by pattern                                  data/mosi.py:198-247

Here every modality is packed once into HBM as ragged rows (``data`` [sum(len), F] f32 + per-sample
offsets and lengths), and a batch is one ``tspm_seq_gather`` launch per modality: index gather, zero
padding to the batch's longest sequence (pad_sequence), the pattern's modality mask and the labels —
written either batch-first (the reference's collate layout, for ``collate_fn``) or time-major straight
into a ``FusedMosiStep``'s input buffers (``device_loader(..., step=...)``: no copy at all).

The reference's own MOSI pickles (aligned_50.pkl) hold DENSE arrays — every sample of a split has the
same length per modality — so its pad_sequence is the identity there; ragged corpora (``lengths``) are
padded exactly as pad_sequence pads them.  Known reference defect, not reproduced: _collate_train_batch
reads ``b[""]`` (data/mosi.py:216), a key no sample has, so the reference's own collate raises KeyError;
this collate returns the batch the rest of that function builds.

Pattern semantics follow the MOSI configs (configs/mosi/centralised/utt_fusion_base_training.yaml:72-139:
every modality named in the pattern has missing_rate 0.0, the others are absent), i.e. modality m is
kept iff its letter is in the pattern.  Training patterns are drawn per sample from a seeded torch
generator (the reference uses Python's ``random.choice`` per ``__getitem__``: same distribution, a
different stream).
"""
from __future__ import annotations

import os
import pickle
from typing import Any, Dict, Iterator, List, Optional, Sequence

import numpy as np
import torch

from . import _lib as L

MODALITIES = ("audio", "video", "text")
_PICKLE_KEYS = {"audio": "audio", "video": "vision", "text": "text"}  # data/mosi.py:135-138
PATTERNS = ["atv", "at", "av", "tv", "a", "t", "v"]  # data/mosi.py:61-69 order


def pattern_keep(pattern: str) -> Dict[str, float]:
    """1.0 for every modality whose first letter is in ``pattern`` (configs/mosi/*: missing_rate 0.0)."""
    return {m: 1.0 if m[0] in pattern else 0.0 for m in MODALITIES}


class MosiCorpus:
    """One split: per modality ragged rows packed as [sum(lengths), F] float32 + offsets + lengths; labels."""

    def __init__(self, seqs: Dict[str, Sequence[np.ndarray]], labels: np.ndarray):
        self.labels = np.ascontiguousarray(np.asarray(labels))
        n = self.labels.shape[0]
        self.data, self.offsets, self.lengths, self.feat = {}, {}, {}, {}
        for m in MODALITIES:
            rows = seqs[m]
            if len(rows) != n:
                raise ValueError(f"{m}: {len(rows)} sequences for {n} labels")
            lens = np.array([np.asarray(r).shape[0] for r in rows], dtype=np.int32)
            feat = int(np.asarray(rows[0]).shape[-1])
            self.data[m] = np.ascontiguousarray(np.concatenate([np.asarray(r, np.float32).reshape(-1, feat)
                                                                for r in rows]) if n else np.zeros((0, feat), np.float32))
            self.offsets[m] = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if n else np.zeros(0, np.int64)
            self.lengths[m] = lens
            self.feat[m] = feat

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    @classmethod
    def from_split(cls, split_data: Dict[str, Any], labels_key: str = "classification_labels",
                   lengths: Optional[Dict[str, np.ndarray]] = None) -> "MosiCorpus":
        """The reference pickle's split dict (``audio``/``vision``/``text`` dense [N, T, F] arrays and the
        labels; data/mosi.py:134-152).  ``lengths`` optionally trims each sample to its true length."""
        seqs = {}
        for m in MODALITIES:
            arr = np.asarray(split_data[_PICKLE_KEYS[m]], dtype=np.float32)
            if lengths is not None and m in lengths:
                seqs[m] = [arr[i, :int(lengths[m][i])] for i in range(arr.shape[0])]
            else:
                seqs[m] = list(arr)
        lab = np.asarray(split_data[labels_key])
        lab = lab.astype(np.float32 if "regression" in labels_key else np.int64).reshape(lab.shape[0], -1)
        return cls(seqs, lab[:, 0] if lab.shape[1] == 1 else lab)


def synthetic_mosi_corpus(n: int, seed: int = 1234, steps: int = 50, min_len: Optional[int] = None,
                          feats=(5, 20, 768)) -> MosiCorpus:
    """MOSI-shaped synthetic split: audio 5-d, video 20-d, text 768-d, 3 classes.  ``min_len``: ragged
    lengths uniform in [min_len, steps] (shared by the three modalities, as in the aligned data); None:
    dense ``steps``-long sequences (aligned_50)."""
    g = np.random.default_rng(seed)
    lens = np.full(n, steps, np.int32) if min_len is None else g.integers(min_len, steps + 1, n).astype(np.int32)
    seqs = {m: [g.standard_normal((int(l), f), dtype=np.float32) for l in lens] for m, f in zip(MODALITIES, feats)}
    return MosiCorpus(seqs, g.integers(0, 3, n).astype(np.int64))


class DeviceMosiCorpus:
    """The packed corpus in HBM; ``gather`` = one tspm_seq_gather per modality."""

    def __init__(self, corpus: MosiCorpus, device: torch.device):
        self.n = len(corpus)
        self.device = device
        self.feat = dict(corpus.feat)
        self.host_lengths = {m: corpus.lengths[m] for m in MODALITIES}
        self.data = {m: torch.from_numpy(corpus.data[m]).to(device) for m in MODALITIES}
        self.offsets = {m: torch.from_numpy(corpus.offsets[m]).to(device) for m in MODALITIES}
        self.lengths = {m: torch.from_numpy(corpus.lengths[m]).to(device) for m in MODALITIES}
        self.labels = torch.from_numpy(np.ascontiguousarray(corpus.labels)).to(device)
        if self.labels.dtype != torch.int64:
            raise L.TspmError("device gather carries int64 class labels (classification_labels)")

    def steps_for(self, index_host: np.ndarray, pad_to: int = 0) -> int:
        """pad_sequence's padded length, the longest sequence of the batch — per modality in the reference
        (data/mosi.py:225-230); the HIP step runs the three modalities over one common length, so the
        per-modality maxima must agree (aligned data) or all be covered by ``pad_to``."""
        if not len(index_host):
            return pad_to
        mx = [int(self.host_lengths[m][index_host].max()) for m in MODALITIES]
        if max(mx) > pad_to and len(set(mx)) > 1:
            raise L.TspmError(f"unaligned batch: per-modality longest sequences {dict(zip(MODALITIES, mx))} differ "
                              "(pad_sequence pads each to its own length); pass pad_to >= all of them")
        return max(max(mx), pad_to)

    def gather(self, index: torch.Tensor, steps_pad: int, out: Dict[str, torch.Tensor], time_major: bool,
               masks: Optional[Dict[str, torch.Tensor]] = None, labels_out: Optional[torch.Tensor] = None) -> None:
        """Write the batch ``index`` (device int64) into ``out[m]``: [T, B, F] (time_major) or [B, T, F]."""
        lib, sh = L.lib(), L.stream_handle()
        b = int(index.numel())
        for j, m in enumerate(MODALITIES):
            f, dst = self.feat[m], out[m]
            shape = (steps_pad, b, f) if time_major else (b, steps_pad, f)
            if tuple(dst.shape) != shape or not dst.is_contiguous() or dst.dtype != torch.float32:
                raise L.TspmError(f"{m}: output {tuple(dst.shape)} != {shape} (contiguous f32)")
            st_t, st_b = (b * f, f) if time_major else (f, steps_pad * f)
            mk = masks.get(m) if masks else None
            L.check(lib.tspm_seq_gather(b, index.data_ptr(), self.n, self.data[m].data_ptr(), self.offsets[m].data_ptr(),
                                        self.lengths[m].data_ptr(), f, steps_pad, dst.data_ptr(), st_t, st_b,
                                        None if mk is None else mk.data_ptr(), self.labels.data_ptr() if j == 0 else None,
                                        labels_out.data_ptr() if (j == 0 and labels_out is not None) else None, sh),
                    "seq_gather")


class MOSI(torch.utils.data.Dataset):
    """data/mosi.py:17-301 (MultimodalSentimentDataset / MOSI) drop-in over a device-resident corpus."""

    VALID_SPLITS = ["train", "valid", "test"]
    NUM_CLASSES = 3
    AVAILABLE_MODALITIES = {m: m for m in MODALITIES}

    def __init__(self, data_fp=None, split: str = "train", target_modality: Any = "multimodal", *,
                 missing_patterns=None, selected_patterns: Optional[List[str]] = None,
                 labels_key: str = "classification_labels", aligned: bool = False, length: Optional[int] = None,
                 num_classes: Optional[int] = None, batch_size: int = 1, corpus: Optional[MosiCorpus] = None,
                 device=None, seed: int = 0, allow_pickle: bool = False) -> None:
        split = split.lower()
        if split not in self.VALID_SPLITS:
            raise AssertionError(f"Invalid split provided, must be one of {self.VALID_SPLITS}")
        self.split, self.labels_key, self.aligned = split, labels_key, aligned
        self.length = length if aligned else None
        if num_classes is not None:
            self.NUM_CLASSES = num_classes
        tm = str(getattr(target_modality, "value", target_modality)).lower().split(".")[-1]
        if tm != "multimodal":
            raise NotImplementedError("MOSI HIP path: target_modality multimodal (the UTT-Fusion configs)")
        self.selected_patterns = list(selected_patterns) if selected_patterns is not None else list(PATTERNS)
        bad = set(self.selected_patterns) - set(PATTERNS)
        if bad:
            raise ValueError(f"Invalid patterns: {bad}")
        self.missing_patterns = missing_patterns
        self._batch_size = batch_size
        self.allow_pickle = allow_pickle
        if corpus is None:
            corpus = self._load(data_fp)
        self.corpus = corpus
        self.num_samples = len(corpus)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self._dev: Optional[DeviceMosiCorpus] = None
        self._gen = torch.Generator().manual_seed(seed)
        self._keep = torch.tensor([[pattern_keep(p)[m] for m in MODALITIES] for p in PATTERNS], dtype=torch.float32)

    def _load(self, data_fp) -> MosiCorpus:
        """An .npz of the reference's split keys (``<split>/audio``, ``<split>/vision``, ...; read with
        allow_pickle=False), or — only with ``allow_pickle=True``, for a data file the user trusts — the
        reference's own split pickle (data/mosi.py:122-152: {"train"/"valid"/"test": {...}}), which
        executes code when loaded."""
        if data_fp is None:
            raise ValueError("MOSI: data_fp or corpus is required")
        path = os.fspath(data_fp)
        if not os.path.exists(path):
            raise FileNotFoundError(f"Data file not found: {path}")
        if path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as z:
                split = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith(self.split + "/")}
        else:
            if not self.allow_pickle:
                raise ValueError(f"{path}: pickled dataset files run code when loaded; convert it to .npz or pass "
                                 "allow_pickle=True for a file you trust")
            with open(path, "rb") as f:
                raw = pickle.load(f)  # noqa: S301 (explicit opt-in; data/mosi.py:125-126)
            if self.split not in raw:
                raise KeyError(f"Split '{self.split}' not found in data")
            split = raw[self.split]
        if self.labels_key not in split:
            raise KeyError(f"Labels key '{self.labels_key}' not found in data")
        # The reference keeps the dense [N, T, F] arrays even for unaligned files and never trims them to
        # audio_lengths / vision_lengths (data/mosi.py:134-152: lengths are metadata only); so here.
        corpus = MosiCorpus.from_split(split, self.labels_key, None)
        if not self.aligned and "audio_lengths" in split:
            corpus.true_lengths = {"audio": np.asarray(split["audio_lengths"]).astype(np.int64),
                                   "video": np.asarray(split["vision_lengths"]).astype(np.int64)}
        return corpus

    # -- reference Dataset API ----------------------------------------------------------------------
    def __len__(self) -> int:
        return self.num_samples if self.split == "train" else self.num_samples * len(self.selected_patterns)

    @property
    def device_corpus(self) -> DeviceMosiCorpus:
        if self._dev is None:
            self._dev = DeviceMosiCorpus(self.corpus, self.device)
        return self._dev

    def _resolve(self, items: Sequence[int]):
        items = np.asarray(items, dtype=np.int64)
        if self.split == "train":
            pid = torch.randint(len(self.selected_patterns), (len(items),), generator=self._gen).numpy()
            return items, pid
        return items % self.num_samples, items // self.num_samples

    def __getitems__(self, items: Sequence[int]):
        return [("__tspm_batch__", np.asarray(items, dtype=np.int64))]

    def __getitem__(self, idx: int):
        return ("__tspm_batch__", np.asarray([idx], dtype=np.int64))

    def collate_fn(self, batch) -> Dict[str, Any]:
        """data/mosi.py:198-247 on the device: padded batch-first tensors [B, T_max, F] per modality (one
        tspm_seq_gather each), labels, pattern names; valid/test batches grouped by pattern."""
        items = np.concatenate([b[1] for b in batch])
        rows, pid = self._resolve(items)
        if self.split == "train":
            return self._collate(rows, pid)
        out = {}
        for p in dict.fromkeys(pid.tolist()):
            sel = pid == p
            out[self.selected_patterns[p]] = self._collate(rows[sel], pid[sel])
        return out

    def _masks(self, pid: np.ndarray) -> Dict[str, torch.Tensor]:
        """Per-row keep factors of the modalities some row of the batch drops (None = all kept)."""
        k = self._keep[[PATTERNS.index(self.selected_patterns[p]) for p in pid]]
        return {m: k[:, j].contiguous().to(self.device, non_blocking=True)
                for j, m in enumerate(MODALITIES) if not bool((k[:, j] == 1.0).all())}

    def _collate(self, rows: np.ndarray, pid: np.ndarray, step=None, pad_to: int = 0) -> Dict[str, Any]:
        dc = self.device_corpus
        b, tpad = len(rows), dc.steps_for(rows, pad_to)
        index = torch.from_numpy(rows).to(self.device, non_blocking=True)
        masks = self._masks(pid)
        names = [self.selected_patterns[p] for p in pid]
        if step is not None:
            e = step.eng
            if (e.B, e.T) != (b, tpad):
                raise L.TspmError(f"step planned for (B={e.B}, T={e.T}), batch is (B={b}, T={tpad})")
            dc.gather(index, tpad, {"audio": e.A, "video": e.V, "text": e.X}, True, masks, e.labels)
            return {"audio": e.A, "video": e.V, "text": e.X, "label": e.labels, "pattern_name": names,
                    "steps": tpad, "time_major": True}
        out = {m: torch.empty(b, tpad, dc.feat[m], device=self.device) for m in MODALITIES}
        lab = torch.empty(b, dtype=torch.int64, device=self.device)
        dc.gather(index, tpad, out, False, masks, lab)
        return {"audio": out["audio"], "video": out["video"], "text": out["text"], "label": lab,
                "pattern_name": names, "pattern_names": names, "steps": tpad}

    def device_loader(self, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                      generator: Optional[torch.Generator] = None, step_for=None,
                      pad_to: int = 0, group_patterns: Optional[bool] = None) -> Iterator[Dict[str, Any]]:
        """One epoch of batches gathered on device.  ``step_for(B, T) -> FusedMosiStep`` (or
        ``FusedMosiEvalStep``): gather each batch time-major straight into that step's input buffers.
        ``pad_to``: pad every batch to at least this many steps (the aligned length, e.g. 50 for aligned_50:
        one captured step shape for the whole epoch; pad_sequence pads to the batch maximum, which equals it
        on the reference's dense data).  ``group_patterns`` (default: valid / test splits, as collate_fn):
        each batch is ``{pattern: sub-batch}`` in first-seen order (data/mosi.py:236-251)."""
        n = len(self)
        grouped = (self.split != "train") if group_patterns is None else bool(group_patterns)
        order = torch.randperm(n, generator=generator).numpy() if shuffle else np.arange(n)
        for s in range(0, n, batch_size):
            items = order[s:s + batch_size]
            if drop_last and len(items) < batch_size:
                break
            rows, pid = self._resolve(items)
            parts = ([(self.selected_patterns[p], pid == p) for p in dict.fromkeys(pid.tolist())] if grouped
                     else [(None, slice(None))])
            out = {}
            for name, sel in parts:
                r, q = rows[sel], pid[sel]
                if step_for is not None:
                    t = self.device_corpus.steps_for(r, pad_to)
                    out[name] = self._collate(r, q, step_for(len(r), t), pad_to)
                    if grouped:
                        yield {name: out[name]}  # the step's buffers are reused: hand each group over at once
                        out = {}
                else:
                    out[name] = self._collate(r, q, None, pad_to)
            if out:
                yield out if grouped else out[None]

    def loader(self, batch_size: int, shuffle: bool = False, drop_last: bool = False, seed: Optional[int] = None,
               step_for=None, pad_to: int = 0, group_patterns: Optional[bool] = None) -> "MosiDeviceLoader":
        """A re-iterable epoch loader (one ``device_loader`` pass per ``iter``), as a DataLoader is."""
        return MosiDeviceLoader(self, batch_size, shuffle, drop_last, seed, step_for, pad_to, group_patterns)

    def get_split(self) -> str:
        return self.split

    def get_selected_patterns(self) -> List[str]:
        return self.selected_patterns

    def get_missing_patterns(self):
        return self.missing_patterns

    @staticmethod
    def get_num_classes(is_classification: bool = True) -> int:
        return 3 if is_classification else 1


class MOSEI(MOSI):
    """data/mosi.py:270-283 (CMU-MOSEI: the same MultimodalSentimentDataset, 3 classes) — the dataset of
    configs/mosei/centralised/utt_fusion_train_mosei.yaml (74-d audio, 35-d video, 768-d text)."""


class MosiDeviceLoader:
    """Re-iterable wrapper of ``MOSI.device_loader`` (a DataLoader is iterated once per epoch): epoch e draws
    its shuffle from ``torch.Generator().manual_seed(seed + e)``; ``step_for`` may be replaced before an epoch
    (the harness points it at its own train / eval steps)."""

    def __init__(self, ds: MOSI, batch_size: int, shuffle: bool, drop_last: bool, seed: Optional[int], step_for,
                 pad_to: int, group_patterns: Optional[bool]):
        self.ds, self.batch_size, self.shuffle, self.drop_last = ds, batch_size, shuffle, drop_last
        self.seed, self.step_for, self.pad_to, self.group_patterns = seed, step_for, pad_to, group_patterns
        self.epoch = 0

    def __len__(self) -> int:
        n = len(self.ds)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        gen = None
        if self.shuffle:
            gen = torch.Generator()
            gen.manual_seed((self.seed if self.seed is not None else 0) + self.epoch)
        self.epoch += 1
        return self.ds.device_loader(self.batch_size, self.shuffle, self.drop_last, gen, self.step_for, self.pad_to,
                                     self.group_patterns)
