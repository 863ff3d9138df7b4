"""Input stage: the AVMNIST corpus resident in HBM, batches assembled on device.

Replaces the reference's host data path for the AVMNIST late-fusion step:

    DataLoader(AVMNIST(...), batch_size, shuffle, collate_fn=dataset.collate_fn)      config/data_config.py:270-290
      → AVMNIST.__getitem__ per sample                                                data/avmnist.py:193-224
          → _load_audio: torch.load(path) f32 [32,94]                                 data/avmnist.py:164-176
          → _load_image: torch.load(path) uint8 [28,28] → cm.gist_earth → PIL "L"
                         → PILToTensor → ToDtype(float32, scale=True)                  data/avmnist.py:178-191
          → get_samples: modality = original × missing-pattern mask                   data/base_dataset.py:61-74
      → collate_fn: torch.stack                                                       data/avmnist.py:248-277

Here the corpus (audio f32, image uint8 — the LUT is applied per batch —, labels int64; 12,824 B
per sample, ≈0.8 GB for all 60k AVMNIST training samples) is uploaded to HBM once, and a batch is ONE
``tspm_avmnist_gather`` launch (index gather + colormap LUT + 1/255 + pattern masks + labels).

Two ways in, same batches:

* drop-in: ``resolve_dataset_name("AVMNIST")`` → :class:`AVMNIST` (this module); the reference's own
  ``DataLoader(dataset, batch_size, shuffle, collate_fn=dataset.collate_fn)`` then calls
  ``dataset.__getitems__(indices)`` (torch's batched-fetch hook) and ``collate_fn`` launches the
  gather — per batch one ≈2 KB pinned H2D of indices/masks, no per-sample work;
* :meth:`AVMNIST.device_loader` — the epoch's order (RandomSampler / DistributedSampler semantics)
  and masks go to HBM in one copy per epoch; each batch is one launch, nothing crosses PCIe.

Corpus files: the reference's CSV (``audio``/``image``/``label`` columns of per-sample ``.pt`` paths,
data/avmnist.py:135-150), read with safe loaders only (``torch.load(weights_only=True)``; numpy
image arrays through torch's allow-list of numpy's array constructors), or this package's packed
format (``pack``/``load``: ``avmnist_corpus.json`` + raw ``audio.f32`` / ``image.u8`` / ``labels.i64``,
memory-mapped).  There is no CPU path: every batch is produced by the HIP kernel.
"""
from __future__ import annotations

import json
import os
import random
from concurrent.futures import ThreadPoolExecutor
from typing import Any, Dict, Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib as L

MODALITIES = ("audio", "image")
AUDIO_SHAPE = (32, 94)
IMAGE_SHAPE = (28, 28)
CORPUS_META = "avmnist_corpus.json"
_LUT_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gist_earth_L.lut")


# ------------------------------------------------------------------------------------------------
# Host corpus
# ------------------------------------------------------------------------------------------------
def _np_safe_globals() -> list:
    """numpy's array-reconstruction callables (data constructors only) for torch's weights-only
    unpickler: the reference saved its images as pickled numpy arrays (data/avmnist.py:188 loads
    them with weights_only=False, which this package never does)."""
    out = [np.ndarray, np.dtype]
    try:
        from numpy._core.multiarray import _reconstruct
        out.append(_reconstruct)
        # the reference's files were pickled under numpy 1.x, which names the function by its old
        # module path; torch matches allow-list entries by that name
        out.append((_reconstruct, "numpy.core.multiarray._reconstruct"))
    except ImportError:  # pragma: no cover - numpy 1.x
        pass
    try:
        from numpy.core.multiarray import _reconstruct as r1  # numpy-1.x pickles name this path
        out.append(r1)
    except Exception:  # pragma: no cover
        pass
    for n in ("UInt8DType", "Float32DType", "Float64DType", "Int64DType", "Int32DType", "Int16DType", "UInt16DType"):
        t = getattr(getattr(np, "dtypes", None), n, None)
        if t is not None:
            out.append(t)
    return out


def load_sample_file(path: str) -> np.ndarray:
    """One per-sample ``.pt`` (tensor or pickled numpy array) via the weights-only unpickler.  Call it
    inside ``torch.serialization.safe_globals(_np_safe_globals())`` for numpy arrays (the allow-list is
    process-wide state, so :meth:`AVMNISTCorpus.from_csv` enters it once around its thread pool)."""
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, torch.Tensor):
        return obj.numpy()
    return np.asarray(obj)


class AVMNISTCorpus:
    """Host-side corpus: ``audio`` f32 [N, 32, 94], ``image`` uint8 [N, 28, 28], ``labels`` int64 [N]."""

    def __init__(self, audio: np.ndarray, image: np.ndarray, labels: np.ndarray):
        audio = np.ascontiguousarray(audio, dtype=np.float32)
        image = np.ascontiguousarray(image)
        labels = np.ascontiguousarray(labels, dtype=np.int64).reshape(-1)
        if image.dtype != np.uint8:
            raise ValueError(f"images must be uint8 colormap indices (got {image.dtype})")
        n = labels.shape[0]
        if audio.shape[0] != n or image.shape[0] != n:
            raise ValueError(f"corpus arrays disagree on N: audio {audio.shape}, image {image.shape}, labels {n}")
        self.audio, self.image, self.labels = audio, image, labels

    def __len__(self) -> int:
        return int(self.labels.shape[0])

    @property
    def audio_shape(self) -> Tuple[int, ...]:
        return tuple(self.audio.shape[1:])

    @property
    def image_shape(self) -> Tuple[int, ...]:
        return tuple(self.image.shape[1:])

    def subset(self, rows: Sequence[int]) -> "AVMNISTCorpus":
        r = np.asarray(rows, dtype=np.int64)
        return AVMNISTCorpus(self.audio[r], self.image[r], self.labels[r])

    # -- reference CSV ------------------------------------------------------------------------------
    @classmethod
    def from_csv(cls, data_fp: str, audio_column: str = "audio", image_column: str = "image",
                 labels_column: str = "label", split_indices: Optional[Sequence[int]] = None,
                 workers: int = 8) -> "AVMNISTCorpus":
        """data/avmnist.py:135-150 (+ the loaders :164-191, minus the colormap which runs on device)."""
        import pandas as pd
        df = pd.read_csv(data_fp)
        if split_indices is not None:
            df = df.iloc[list(split_indices)].reset_index(drop=True)
        missing = [c for c in (audio_column, image_column, labels_column) if c not in df.columns]
        if missing:
            raise ValueError(f"Missing required columns: {missing}")
        base = os.path.dirname(os.path.abspath(data_fp))

        def resolve(p: str) -> str:
            return p if os.path.isabs(p) or os.path.exists(p) else os.path.join(base, p)

        apaths = [resolve(str(p)) for p in df[audio_column]]
        ipaths = [resolve(str(p)) for p in df[image_column]]
        with torch.serialization.safe_globals(_np_safe_globals()), ThreadPoolExecutor(max(1, workers)) as ex:
            audio = list(ex.map(load_sample_file, apaths))
            image = list(ex.map(load_sample_file, ipaths))
        a = np.stack([np.asarray(x, dtype=np.float32) for x in audio]) if audio else \
            np.zeros((0,) + AUDIO_SHAPE, np.float32)
        im = []
        for p, x in zip(ipaths, image):
            x = np.asarray(x)
            if x.dtype != np.uint8:
                if np.issubdtype(x.dtype, np.integer) and x.min(initial=0) >= 0 and x.max(initial=0) <= 255:
                    x = x.astype(np.uint8)
                else:
                    # cm.gist_earth(float) is a different (interpolating) map; only integer
                    # colormap indices are on this path
                    raise ValueError(f"{p}: image must hold integer colormap indices 0..255 (got {x.dtype})")
            im.append(x)
        i = np.stack(im) if im else np.zeros((0,) + IMAGE_SHAPE, np.uint8)
        return cls(a, i, df[labels_column].to_numpy(dtype=np.int64))

    # -- packed format ------------------------------------------------------------------------------
    def save(self, out_dir: str) -> None:
        os.makedirs(out_dir, exist_ok=True)
        self.audio.tofile(os.path.join(out_dir, "audio.f32"))
        self.image.tofile(os.path.join(out_dir, "image.u8"))
        self.labels.astype("<i8").tofile(os.path.join(out_dir, "labels.i64"))
        meta = {"format": "tspm-avmnist-corpus", "version": 1, "n": len(self),
                "audio_shape": list(self.audio_shape), "image_shape": list(self.image_shape)}
        with open(os.path.join(out_dir, CORPUS_META), "w") as f:
            json.dump(meta, f)

    @classmethod
    def load(cls, path: str, split_indices: Optional[Sequence[int]] = None) -> "AVMNISTCorpus":
        d = os.path.dirname(path) if path.endswith(".json") else path
        with open(os.path.join(d, CORPUS_META)) as f:
            meta = json.load(f)
        if meta.get("format") != "tspm-avmnist-corpus" or meta.get("version") != 1:
            raise ValueError(f"{d}: not a version-1 packed AVMNIST corpus")
        n = int(meta["n"])
        a = np.memmap(os.path.join(d, "audio.f32"), dtype="<f4", mode="r", shape=(n, *meta["audio_shape"]))
        i = np.memmap(os.path.join(d, "image.u8"), dtype=np.uint8, mode="r", shape=(n, *meta["image_shape"]))
        lab = np.fromfile(os.path.join(d, "labels.i64"), dtype="<i8", count=n)
        c = cls(a, i, lab) if split_indices is None else AVMNISTCorpus(a, i, lab).subset(split_indices)
        return c

    @classmethod
    def open(cls, data_fp: str, split_indices: Optional[Sequence[int]] = None, **csv_kw) -> "AVMNISTCorpus":
        if os.path.isdir(data_fp) or str(data_fp).endswith(".json"):
            return cls.load(str(data_fp), split_indices)
        return cls.from_csv(str(data_fp), split_indices=split_indices, **csv_kw)


def pack(csv_path: str, out_dir: str, **csv_kw) -> AVMNISTCorpus:
    """Convert a reference-format CSV corpus into the packed format (one-off)."""
    c = AVMNISTCorpus.from_csv(csv_path, **csv_kw)
    c.save(out_dir)
    return c


def synthetic_corpus(n: int, seed: int = 1234) -> AVMNISTCorpus:
    """AVMNIST-shaped synthetic corpus (SURVEY.md §8(d) "Synthetic inputs"; no dataset download here):
    audio f32 [n,32,94] = 10**clip(N(0.108, 5.85), log10 2.2e-9, log10 1.52e7) (the log-moments of real
    AVMNIST spectrogram files), image uint8 [n,28,28] with 81 % zeros and U{1..255} elsewhere, labels
    U{0..9}; numpy ``default_rng(seed)``, the same draws as the parity tests' generator."""
    import math
    rng = np.random.default_rng(seed)
    la = np.clip(rng.normal(0.108, 5.85, size=(n,) + AUDIO_SHAPE), math.log10(2.2e-9), math.log10(1.52e7))
    audio = (10.0 ** la).astype(np.float32)
    u8 = rng.integers(1, 256, size=(n,) + IMAGE_SHAPE).astype(np.uint8)
    u8[rng.random((n,) + IMAGE_SHAPE) < 0.81] = 0
    labels = rng.integers(0, 10, size=(n,)).astype(np.int64)
    return AVMNISTCorpus(audio, u8, labels)


def default_lut() -> np.ndarray:
    """The 256-entry uint8 map of ``cm.gist_earth`` → RGBA·255 → PIL ``convert("L")`` (package data,
    identical to tests/golden/lut_gist_earth_L.bin generated from matplotlib + PIL)."""
    with open(_LUT_FILE, "rb") as f:
        lut = np.frombuffer(f.read(), dtype=np.uint8)
    if lut.shape != (256,):
        raise ValueError(f"{_LUT_FILE}: expected 256 bytes")
    return lut


# ------------------------------------------------------------------------------------------------
# Device corpus + gather
# ------------------------------------------------------------------------------------------------
class DeviceCorpus:
    """The corpus in HBM plus the colormap LUT; :meth:`gather` is the one-launch batch assembly."""

    def __init__(self, corpus: AVMNISTCorpus, device: torch.device, lut: Optional[np.ndarray] = None):
        if device.type != "cuda":
            raise L.TspmError(f"DeviceCorpus needs a ROCm device (got {device}); the input stage has no CPU path")
        L.lib()
        self.device = device
        self.n = len(corpus)
        self.audio_shape, self.image_shape = corpus.audio_shape, corpus.image_shape
        self.audio_elems = int(np.prod(self.audio_shape))
        self.image_elems = int(np.prod(self.image_shape))
        self.audio = torch.from_numpy(np.ascontiguousarray(corpus.audio)).to(device)
        self.image = torch.from_numpy(np.ascontiguousarray(corpus.image)).to(device)
        self.labels = torch.from_numpy(np.ascontiguousarray(corpus.labels)).to(device)
        lut = default_lut() if lut is None else np.ascontiguousarray(lut, dtype=np.uint8)
        self.lut = torch.from_numpy(lut.copy()).to(device)

    def gather(self, index: torch.Tensor, audio_mask: Optional[torch.Tensor] = None,
               image_mask: Optional[torch.Tensor] = None, want_audio: bool = True, want_image: bool = True,
               out: Optional[Tuple[Optional[torch.Tensor], Optional[torch.Tensor], Optional[torch.Tensor]]] = None,
               stream: Optional[torch.cuda.Stream] = None):
        """audio [B, *audio_shape] f32, image [B, 1, *image_shape] f32, labels [B] int64 for the
        corpus rows ``index`` (int64 device tensor), each modality × its per-row mask (if given)."""
        if index.device != self.device or index.dtype != torch.int64 or not index.is_contiguous():
            raise L.TspmError("index must be a contiguous int64 tensor on the corpus device")
        b = index.numel()
        for m, name in ((audio_mask, "audio_mask"), (image_mask, "image_mask")):
            if m is not None and (m.device != self.device or m.dtype != torch.float32 or m.numel() < b
                                  or not m.is_contiguous()):
                raise L.TspmError(f"{name} must be a contiguous float32 device tensor with >= {b} entries")
        if out is None:
            a = torch.empty((b,) + self.audio_shape, device=self.device) if want_audio else None
            im = torch.empty((b, 1) + self.image_shape, device=self.device) if want_image else None
            lab = torch.empty(b, dtype=torch.int64, device=self.device)
        else:
            a, im, lab = out
            a, im = (a if want_audio else None), (im if want_image else None)
            for t, e, dt in ((a, self.audio_elems, torch.float32), (im, self.image_elems, torch.float32),
                             (lab, 1, torch.int64)):
                if t is not None and (t.device != self.device or t.dtype != dt or t.numel() != b * e
                                      or not t.is_contiguous()):
                    raise L.TspmError("gather output buffer has the wrong device/dtype/size/layout")
        L.check(L.lib().tspm_avmnist_gather(
            b, index.data_ptr(), self.n, self.audio.data_ptr(), self.audio_elems, self.image.data_ptr(),
            self.image_elems, self.labels.data_ptr(), self.lut.data_ptr(), L.ptr(audio_mask), L.ptr(image_mask),
            L.ptr(a), L.ptr(im), L.ptr(lab), L.stream_handle(stream)), "tspm_avmnist_gather")
        return a, im, lab


# ------------------------------------------------------------------------------------------------
# Dataset with the reference's interface
# ------------------------------------------------------------------------------------------------
def _modality_name(m: Any) -> str:
    for attr in ("value", "name"):
        v = getattr(m, attr, None)
        if isinstance(v, str):
            return v.lower()
    return str(m).lower().split(".")[-1]


def _default_keys() -> Dict[str, Any]:
    """Batch keys: the reference's ``modalities.Modality`` members when that package is importable
    (it is un-vendored), else the plain strings — ``modules.modality_key`` accepts both."""
    try:
        from modalities import Modality  # type: ignore
        return {"audio": Modality.AUDIO, "image": Modality.IMAGE}
    except Exception:
        return {"audio": "audio", "image": "image"}


class _BatchRequest(list):
    """What :meth:`AVMNIST.__getitems__` returns: the batch's dataset indices, resolved by
    :meth:`AVMNIST.collate_fn` in one gather launch."""

    def __init__(self, owner: "AVMNIST", items: Sequence[int]):
        super().__init__(int(i) for i in items)
        self.owner = owner


class _Staging:
    """Ring of pinned host buffers for the per-batch index + mask upload (one H2D per batch)."""

    def __init__(self, device: torch.device, slots: int = 4):
        self.device, self.slots, self.k = device, slots, 0
        self.bufs: Dict[int, List[Tuple[torch.Tensor, torch.Tensor, torch.cuda.Event]]] = {}

    def upload(self, index: np.ndarray, am: np.ndarray, im: np.ndarray, pid: np.ndarray):
        b = index.shape[0]
        ring = self.bufs.get(b)
        if ring is None:
            ring = [(torch.empty(20 * b, dtype=torch.uint8).pin_memory(),
                     torch.empty(20 * b, dtype=torch.uint8, device=self.device), torch.cuda.Event())
                    for _ in range(self.slots)]
            self.bufs[b] = ring
        host, dev, ev = ring[self.k % self.slots]
        self.k += 1
        ev.synchronize()  # the previous upload from this slot has left the host buffer
        host[:8 * b].view(torch.int64).numpy()[:] = index
        host[8 * b:12 * b].view(torch.float32).numpy()[:] = am
        host[12 * b:16 * b].view(torch.float32).numpy()[:] = im
        host[16 * b:].view(torch.int32).numpy()[:] = pid
        dev.copy_(host, non_blocking=True)
        ev.record()
        return (dev[:8 * b].view(torch.int64), dev[8 * b:12 * b].view(torch.float32),
                dev[12 * b:16 * b].view(torch.float32), dev[16 * b:].view(torch.int32))


class AVMNIST(torch.utils.data.Dataset):
    """Drop-in for ``data.avmnist.AVMNIST`` (MML_Suite/data/avmnist.py:20-277): same constructor,
    ``__len__``, pattern semantics, ``collate_fn`` output and ``get_pattern_batches``; batches are
    assembled on the GPU from the HBM-resident corpus.

    ``data_fp`` is the reference CSV or a packed corpus directory.  Extra keyword-only arguments:
    ``device`` (default: the current ROCm device, chosen at first use), ``lut`` (override the colormap
    table), ``keys`` (batch keys per modality), ``corpus`` (an :class:`AVMNISTCorpus` instead of a file).
    """

    NUM_CLASSES: int = 10
    VALID_SPLITS = ["train", "valid", "test"]
    AVAILABLE_MODALITIES = {"audio": "audio", "image": "image"}

    @staticmethod
    def get_full_modality() -> str:
        """data/avmnist.py:34-43."""
        return "".join(sorted(k[0] for k in AVMNIST.AVAILABLE_MODALITIES))

    @classmethod
    def get_all_possible_patterns(cls) -> List[str]:
        """data/base_dataset.py:113-122."""
        import itertools
        mods = list(cls.AVAILABLE_MODALITIES)
        pats = ["".join(m[0] for m in sorted(c)) for r in range(1, len(mods) + 1)
                for c in itertools.combinations(mods, r)]
        return sorted(pats)

    def __init__(self, data_fp=None, split: str = "train", target_modality: Any = "multimodal", *,
                 missing_patterns: Optional[Dict[str, Dict[Any, float]]] = None,
                 selected_patterns: Optional[List[str]] = None, audio_column: str = "audio",
                 image_column: str = "image", labels_column: str = "label",
                 split_indices: Optional[List[int]] = None, _id: int = 1, batch_size: int = 1,
                 device: Optional[torch.device] = None, lut: Optional[np.ndarray] = None,
                 keys: Optional[Dict[str, Any]] = None, corpus: Optional[AVMNISTCorpus] = None,
                 mask_seed: int = 0) -> None:
        split = split.lower()
        if split not in self.VALID_SPLITS:
            raise AssertionError(f"Invalid split provided, must be one of {self.VALID_SPLITS}")
        self.split = split
        self._id = _id
        self._batch_size = batch_size
        m_patterns = missing_patterns or {"ai": {"audio": 1.0, "image": 1.0}, "a": {"audio": 1.0, "image": 0.0},
                                          "i": {"audio": 0.0, "image": 1.0}}
        self.missing_patterns = {p: {_modality_name(m): float(v) for m, v in probs.items()}
                                 for p, probs in m_patterns.items()}
        allp = self.get_all_possible_patterns()
        if selected_patterns is not None:
            bad = set(selected_patterns) - set(allp)
            if bad:
                raise ValueError(f"Invalid patterns: {bad}\nValid patterns are: {allp}")
            self.selected_patterns = list(selected_patterns)
        else:
            self.selected_patterns = allp
        for p in self.selected_patterns:
            if p not in self.missing_patterns:
                raise ValueError(f"selected pattern {p!r} has no entry in missing_patterns")
        target = _modality_name(target_modality)
        if target not in ("audio", "image", "multimodal"):
            raise AssertionError("Invalid modality provided, must be one of [audio, image, multimodal]")
        self.target_modality = target
        if corpus is None:
            if data_fp is None:
                raise ValueError("data_fp (CSV or packed corpus directory) or corpus= is required")
            if not os.path.exists(str(data_fp)):
                raise FileNotFoundError(f"Data file not found: {data_fp}")
            corpus = AVMNISTCorpus.open(str(data_fp), split_indices, audio_column=audio_column,
                                        image_column=image_column, labels_column=labels_column)
        elif split_indices is not None:
            corpus = corpus.subset(split_indices)
        self.corpus = corpus
        self.num_samples = len(corpus)
        self.pattern_indices = {p: list(range(self.num_samples)) for p in self.selected_patterns}
        self.masks = self._initialise_missing_masks(len(self), mask_seed)
        self._device = device
        self._lut = lut
        self._dev: Optional[DeviceCorpus] = None
        self._staging: Optional[_Staging] = None
        self.keys = keys or _default_keys()
        self.current_pattern = None

    # -- reference semantics --------------------------------------------------------------------------
    def _initialise_missing_masks(self, length: int, seed: int) -> Dict[str, Dict[str, np.ndarray]]:
        """data/base_dataset.py:46-59.  Presence probability 1.0 / 0.0 → mask 1 / 0 (what the reference's
        un-vendored create_missing_mask yields for AVMNIST's patterns); a fractional probability draws
        Bernoulli(p) per sample with numpy (parity unpinned)."""
        rng = np.random.default_rng(seed)
        out = {}
        for p, probs in self.missing_patterns.items():
            out[p] = {}
            for m in MODALITIES:
                pr = probs.get(m, 1.0)
                out[p][m] = np.full(length, pr, np.float32) if pr in (0.0, 1.0) else \
                    (rng.random(length) < pr).astype(np.float32)
        return out

    def __len__(self) -> int:
        """data/avmnist.py:152-162."""
        return self.num_samples if self.split == "train" else self.num_samples * len(self.selected_patterns)

    def pattern_ids(self, names: Sequence[str]) -> np.ndarray:
        """Index of each pattern name in ``get_all_possible_patterns()`` (["a", "ai", "i"]) — the
        ``pattern_ids`` batch entry (int32, device) that keys the device-side metrics by pattern."""
        allp = self.get_all_possible_patterns()
        return np.fromiter((allp.index(n) for n in names), dtype=np.int32, count=len(names))

    def _resolve(self, items: Sequence[int]) -> Tuple[np.ndarray, List[str], np.ndarray, np.ndarray]:
        """data/base_dataset.py:76-92 + 137-150: dataset index → (pattern, sample) and its masks."""
        n, sel = self.num_samples, self.selected_patterns
        L_ = len(self)
        idx = np.asarray(items, dtype=np.int64).reshape(-1)
        if idx.size and (idx.min() < -L_ or idx.max() >= L_):
            raise IndexError(f"dataset index out of range for length {L_}")
        idx = np.where(idx < 0, idx + L_, idx)
        if self.split in ("train", "trn"):
            names = [random.choice(sel) for _ in range(idx.size)]  # one draw per item, as the reference
            samples = idx
        else:
            names = [sel[int(i) // n] for i in idx]
            samples = idx % n
        am = np.empty(idx.size, np.float32)
        im = np.empty(idx.size, np.float32)
        for p in set(names):
            rows = np.fromiter((k for k, q in enumerate(names) if q == p), dtype=np.int64)
            am[rows] = self.masks[p]["audio"][samples[rows]]
            im[rows] = self.masks[p]["image"][samples[rows]]
        return samples, names, am, im

    # -- device side ----------------------------------------------------------------------------------
    @property
    def device_corpus(self) -> DeviceCorpus:
        if self._dev is None:
            if not torch.cuda.is_available():
                raise L.TspmError("AVMNIST batches are assembled on the GPU; no ROCm device is available")
            dev = torch.device(self._device) if self._device is not None else \
                torch.device("cuda", torch.cuda.current_device())
            self._dev = DeviceCorpus(self.corpus, dev, self._lut)
        return self._dev

    def _want(self) -> Tuple[bool, bool]:
        t = self.target_modality
        return t in ("multimodal", "audio"), t in ("multimodal", "image")

    def _pack(self, a, im, lab, names, pids=None) -> Dict[Any, Any]:
        """collate_fn's output dict (data/avmnist.py:258-277), plus ``pattern_ids`` (int32 device
        tensor, see :meth:`pattern_ids`) for the device-side metrics."""
        out: Dict[Any, Any] = {"labels": lab, "pattern_name": list(names), "missing_masks": {}}
        if pids is not None:
            out["pattern_ids"] = pids
        if a is not None:
            out[self.keys["audio"]] = a
        if im is not None:
            out[self.keys["image"]] = im
        return out

    def _gather_batch(self, items: Sequence[int]) -> Dict[Any, Any]:
        dc = self.device_corpus
        samples, names, am, im = self._resolve(items)
        if self._staging is None:
            self._staging = _Staging(dc.device)
        if len(samples) == 0:
            raise ValueError("empty batch")
        idx_d, am_d, im_d, pid_d = self._staging.upload(samples, am, im, self.pattern_ids(names))
        wa, wi = self._want()
        a, imt, lab = dc.gather(idx_d, am_d, im_d, want_audio=wa, want_image=wi)
        if names:
            self.current_pattern = names[-1]
        return self._pack(a, imt, lab, names, pid_d)

    def __getitems__(self, items: Sequence[int]) -> _BatchRequest:
        """torch DataLoader's batched-fetch hook: defer the whole batch to :meth:`collate_fn`."""
        return _BatchRequest(self, items)

    def __getitem__(self, idx: int) -> Dict[Any, Any]:
        """One sample (data/avmnist.py:193-224) — a batch of one, unstacked."""
        b = self._gather_batch([idx])
        sample = {"labels": b["labels"][0], "pattern_name": b["pattern_name"][0], "missing_mask": {},
                  "sample_idx": int(self._resolve_sample(idx))}
        for m in MODALITIES:
            k = self.keys[m]
            if k in b:
                sample[k] = b[k][0]
        return sample

    def _resolve_sample(self, idx: int) -> int:
        return idx if self.split in ("train", "trn") else idx % self.num_samples

    def collate_fn(self, batch) -> Dict[Any, Any]:
        """data/avmnist.py:248-277.  A ``__getitems__`` request → one gather launch; a list of sample
        dicts (from ``dataset[i]``) → stacked on device like the reference."""
        if isinstance(batch, _BatchRequest):
            return batch.owner._gather_batch(batch)
        out: Dict[Any, Any] = {"labels": torch.stack([b["labels"] for b in batch]),
                               "pattern_name": [b["pattern_name"] for b in batch], "missing_masks": {}}
        for m in MODALITIES:
            k = self.keys[m]
            if k in batch[0]:
                out[k] = torch.stack([b[k] for b in batch])
        return out

    def get_pattern_batches(self, batch_size: int, **dataloader_kwargs) -> Dict[str, torch.utils.data.DataLoader]:
        """data/avmnist.py:226-246."""
        if self.split == "train":
            raise ValueError("Pattern-specific batches only available for validation/test")
        return {p: torch.utils.data.DataLoader(PatternView(self, p), batch_size=batch_size, shuffle=False,
                                               collate_fn=self.collate_fn, **dataloader_kwargs)
                for p in self.selected_patterns}

    def device_loader(self, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                      generator: Optional[torch.Generator] = None, *, rank: int = 0, world_size: int = 1,
                      distributed: Optional[bool] = None, seed: int = 0, pattern: Optional[str] = None,
                      out=None) -> "DeviceLoader":
        return DeviceLoader(self, batch_size, shuffle, drop_last, generator, rank=rank, world_size=world_size,
                            distributed=distributed, seed=seed, pattern=pattern, out=out)

    def get_split(self) -> str:
        return self.split

    def get_selected_patterns(self) -> List[str]:
        return self.selected_patterns

    def get_missing_patterns(self):
        return self.missing_patterns


class PatternView(torch.utils.data.Dataset):
    """data/pattern.py: the samples of one pattern of a valid/test split (index + pattern·N)."""

    def __init__(self, parent: AVMNIST, pattern: str):
        self.parent, self.pattern = parent, pattern
        self.offset = parent.selected_patterns.index(pattern) * parent.num_samples

    def __len__(self) -> int:
        return self.parent.num_samples

    def __getitems__(self, items: Sequence[int]) -> _BatchRequest:
        return _BatchRequest(self.parent, [int(i) + self.offset for i in items])

    def __getitem__(self, idx: int):
        return self.parent[int(idx) + self.offset]


class DeviceLoader:
    """Epoch iterator with no per-batch host→device traffic: the epoch's sample order (torch
    ``RandomSampler`` / ``SequentialSampler``, or ``DistributedSampler`` with ``world_size > 1``) and the
    per-item masks are resolved on the host and copied to HBM once; each batch is one gather launch.
    Batches equal those of ``DataLoader(dataset, batch_size, shuffle, drop_last, collate_fn=
    dataset.collate_fn)`` for the same item order.

    ``out=(audio, image, labels)``: full batches are written into these caller-owned buffers (e.g. a
    ``FusedTrainStep``'s static inputs, so the step consumes the gather's output in place) and the
    yielded dict holds those same tensors — consume each batch before advancing the iterator."""

    def __init__(self, dataset: AVMNIST, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                 generator: Optional[torch.Generator] = None, *, rank: int = 0, world_size: int = 1,
                 distributed: Optional[bool] = None, seed: int = 0, pattern: Optional[str] = None, out=None):
        if batch_size <= 0:
            raise ValueError("batch_size must be positive")
        self.out = out
        self.ds, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        self.generator, self.rank, self.world_size, self.seed = generator, rank, world_size, seed
        self.distributed = world_size > 1 if distributed is None else distributed
        self.pattern = pattern
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def _n_items(self) -> int:
        return self.ds.num_samples if self.pattern is not None else len(self.ds)

    def items(self) -> np.ndarray:
        """The epoch's item order, drawing from the RNGs exactly as ``iter(DataLoader(...))`` does: the
        loader's ``_base_seed`` int64 first (torch/utils/data/dataloader.py, from ``generator`` or the
        global torch RNG), then the sampler."""
        n = self._n_items()
        torch.empty((), dtype=torch.int64).random_(generator=self.generator)
        if self.distributed:
            sampler = torch.utils.data.DistributedSampler(range(n), num_replicas=self.world_size, rank=self.rank,
                                                          shuffle=self.shuffle, seed=self.seed,
                                                          drop_last=self.drop_last)
            sampler.set_epoch(self.epoch)
            order = np.fromiter(iter(sampler), dtype=np.int64)
        elif self.shuffle:
            order = np.fromiter(iter(torch.utils.data.RandomSampler(range(n), generator=self.generator)),
                                dtype=np.int64, count=n)
        else:
            order = np.arange(n, dtype=np.int64)
        if self.pattern is not None:
            order = order + self.ds.selected_patterns.index(self.pattern) * self.ds.num_samples
        return order

    def __len__(self) -> int:
        n = self._n_items()
        if self.distributed:
            n = (n // self.world_size) if (self.drop_last and n % self.world_size) else -(-n // self.world_size)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self) -> Iterator[Dict[Any, Any]]:
        order = self.items()
        nb = len(self)
        if nb == 0:
            return
        order = order[:nb * self.batch_size] if self.drop_last else order
        samples, names, am, im = self.ds._resolve(order)
        dc = self.ds.device_corpus
        idx_d = torch.from_numpy(samples).pin_memory().to(dc.device, non_blocking=True)
        am_d = torch.from_numpy(am).pin_memory().to(dc.device, non_blocking=True)
        im_d = torch.from_numpy(im).pin_memory().to(dc.device, non_blocking=True)
        pid_d = torch.from_numpy(self.ds.pattern_ids(names)).pin_memory().to(dc.device, non_blocking=True)
        wa, wi = self.ds._want()
        for b in range(nb):
            lo, hi = b * self.batch_size, min(len(order), (b + 1) * self.batch_size)
            out = self.out if (self.out is not None and hi - lo == self.batch_size) else None
            a, imt, lab = dc.gather(idx_d[lo:hi], am_d[lo:hi], im_d[lo:hi], want_audio=wa, want_image=wi, out=out)
            yield self.ds._pack(a, imt, lab, names[lo:hi], pid_d[lo:hi])
