"""ORACLE — CPU restatement of the AVMNIST input stage.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module (as the checker).  The product package never imports it.

Restated (reference = TArsenii/task-specific-pretraining-multimodal, paths under ``MML_Suite/``):

* pattern names             data/base_dataset.py:113-122 (``get_all_possible_patterns``: first letters
                            of each sorted modality combination, list sorted → ["a", "ai", "i"])
* default missing patterns  data/avmnist.py:73-77 (presence probability per modality and pattern)
* missing masks             data/base_dataset.py:46-59 + the un-vendored ``modalities.create_missing_mask``:
                            presence probability 1.0 → mask 1, 0.0 → mask 0 (deterministic, pinned);
                            fractional probabilities draw Bernoulli(presence) here — PARITY UNPINNED
                            (the un-vendored function's RNG use is unknown)
* index → (pattern, sample) data/base_dataset.py:76-92 (train: ``random.choice`` per item; valid/test:
                            ``idx // N`` selects the pattern, ``idx % N`` the sample) and ``__len__``
                            data/avmnist.py:152-162 (train N, else N × #patterns)
* sample assembly           data/avmnist.py:193-224 + data/base_dataset.py:61-74 (modality =
                            original × mask), ``_load_image`` data/avmnist.py:178-191 for an integer
                            uint8 image = ``LUT[u8]`` (gist_earth → RGBA·255 → PIL "L", the committed
                            tests/golden/lut_gist_earth_L.bin) then torchvision v2 ``ToDtype(float32,
                            scale=True)`` = ``to(float32).mul_(1/255)`` (torchvision is absent here; the
                            multiply-by-reciprocal form is restated from its ``to_dtype_image`` — a
                            division would differ by 1 ulp on 126 of the 256 values)
* ``collate_fn``            data/avmnist.py:248-277 (stack; ``missing_masks`` stays ``{}`` because
                            ``sample["missing_mask"]`` is never filled, :211)

Pinned by ``tests/golden/avmnist_data.npz``, produced by running the REAL reference dataset class
(``tests/golden/make_data_golden.py``) over a small corpus written in the reference's file format.
"""
from __future__ import annotations

import itertools
import random
from typing import Dict, List, Optional, Sequence

import numpy as np

MODALITIES = ("audio", "image")


def all_patterns(modalities: Sequence[str] = MODALITIES) -> List[str]:
    """data/base_dataset.py:113-122."""
    out = []
    for r in range(1, len(modalities) + 1):
        for combo in itertools.combinations(modalities, r):
            out.append("".join(m[0] for m in sorted(combo)))
    return sorted(out)


def default_missing_patterns() -> Dict[str, Dict[str, float]]:
    """data/avmnist.py:73-77 (values are presence probabilities)."""
    return {"ai": {"audio": 1.0, "image": 1.0}, "a": {"audio": 1.0, "image": 0.0}, "i": {"audio": 0.0, "image": 1.0}}


def missing_masks(patterns: Dict[str, Dict[str, float]], length: int, seed: int = 0) -> Dict[str, Dict[str, np.ndarray]]:
    """data/base_dataset.py:46-59: per pattern and modality a float mask of ``length`` entries."""
    rng = np.random.default_rng(seed)
    out = {}
    for p, probs in patterns.items():
        out[p] = {}
        for m, pr in probs.items():
            if pr in (0.0, 1.0):
                out[p][m] = np.full(length, pr, dtype=np.float32)
            else:  # parity unpinned (un-vendored create_missing_mask)
                out[p][m] = (rng.random(length) < pr).astype(np.float32)
    return out


def dataset_len(split: str, n: int, selected: Sequence[str]) -> int:
    """data/avmnist.py:152-162."""
    return n if split == "train" else n * len(selected)


def pattern_and_sample(idx: int, split: str, n: int, selected: Sequence[str], rnd: Optional[random.Random] = None):
    """data/base_dataset.py:76-92."""
    if split in ("train", "trn"):
        return (rnd or random).choice(list(selected)), idx
    return selected[idx // n], idx % n


def image_to_float(u8: np.ndarray, lut: np.ndarray) -> np.ndarray:
    """data/avmnist.py:186-191: LUT (the PIL colormap pipeline for integer input), then ToDtype scale."""
    return lut[u8].astype(np.float32) * np.float32(1.0 / 255.0)


def collate(audio: np.ndarray, image_u8: np.ndarray, labels: np.ndarray, lut: np.ndarray, items: Sequence[int],
            split: str, selected: Sequence[str], patterns: Optional[Dict[str, Dict[str, float]]] = None,
            target: str = "multimodal", rnd: Optional[random.Random] = None) -> Dict[str, object]:
    """``collate_fn([dataset[i] for i in items])`` (data/avmnist.py:193-224, 248-277)."""
    n = audio.shape[0]
    patterns = patterns or default_missing_patterns()
    masks = missing_masks(patterns, dataset_len(split, n, selected))
    a_rows, i_rows, labs, names = [], [], [], []
    for it in items:
        p, s = pattern_and_sample(int(it), split, n, selected, rnd)
        names.append(p)
        labs.append(labels[s])
        if target in ("multimodal", "audio"):
            a_rows.append(audio[s] * masks[p]["audio"][s])
        if target in ("multimodal", "image"):
            i_rows.append(image_to_float(image_u8[s], lut)[None] * masks[p]["image"][s])
    out: Dict[str, object] = {"labels": np.asarray(labs, dtype=np.int64), "pattern_name": names, "missing_masks": {}}
    if a_rows:
        out["audio"] = np.stack(a_rows).astype(np.float32)
    if i_rows:
        out["image"] = np.stack(i_rows).astype(np.float32)
    return out


def distributed_indices(n: int, world: int, rank: int, shuffle: bool, seed: int, epoch: int,
                        drop_last: bool = False) -> np.ndarray:
    """torch.utils.data.DistributedSampler.__iter__ (torch 2.x): permutation from a generator seeded
    with seed + epoch, padded by wrap-around (or truncated with drop_last) to a multiple of world,
    then every world-th index starting at rank."""
    import torch
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    if drop_last and n % world:
        num = n // world
    else:
        num = -(-n // world)
    total = num * world
    if not drop_last:
        pad = total - len(idx)
        if pad <= len(idx):
            idx += idx[:pad]
        else:
            idx += (idx * -(-pad // len(idx)))[:pad]
    else:
        idx = idx[:total]
    return np.asarray(idx[rank:total:world], dtype=np.int64)


def write_reference_files(root: str, audio: np.ndarray, image_u8: np.ndarray, labels: np.ndarray) -> str:
    """A corpus in the reference's on-disk layout (CSV of per-sample ``.pt`` paths: audio = saved
    float32 tensor, image = saved uint8 numpy array; data/avmnist.py:135-191).  Returns the CSV path."""
    import os
    import torch
    rows = ["audio,image,label"]
    for i in range(audio.shape[0]):
        ap, ip = os.path.join(root, f"audio_{i}.pt"), os.path.join(root, f"image_{i}.pt")
        torch.save(torch.from_numpy(np.ascontiguousarray(audio[i])), ap)
        torch.save(np.ascontiguousarray(image_u8[i]), ip)
        rows.append(f"{ap},{ip},{int(labels[i])}")
    csv = os.path.join(root, "corpus.csv")
    with open(csv, "w") as f:
        f.write("\n".join(rows) + "\n")
    return csv


def reference_host_batches(csv: str, batch: int, device=None):
    """The reference's per-batch host work, restated step by step for the CPU baseline: for every
    sample ``torch.load`` the audio file (data/avmnist.py:165-176), ``torch.load`` the image file, map
    it through ``cm.gist_earth`` → RGBA·255 → PIL ``convert("L")`` → ``PILToTensor`` → ``to(float32)
    .mul_(1/255)`` (:178-191), multiply both by the pattern mask (data/base_dataset.py:61-74), then
    ``collate_fn``'s ``torch.stack`` (:248-277) and — with ``device`` — the train step's
    ``.to(device)`` (models/avmnist.py:276-282).  Yields one batch dict at a time (no lru_cache hits:
    every path is read once, as in an epoch over a corpus far larger than the cache's 1000 entries)."""
    import pandas as pd
    import torch
    from matplotlib import cm
    from PIL import Image
    np_globals = [np.ndarray, np.dtype]
    from numpy._core.multiarray import _reconstruct
    np_globals += [_reconstruct, np.dtypes.UInt8DType]
    df = pd.read_csv(csv)
    one = torch.ones(())
    samples = []
    with torch.serialization.safe_globals(np_globals):
        for r in range(len(df)):
            a = torch.load(df["audio"].iloc[r], weights_only=True)
            img = np.array(torch.load(df["image"].iloc[r], weights_only=True))
            pil = Image.fromarray(np.uint8(cm.gist_earth(img) * 255)).convert("L")
            im = torch.from_numpy(np.array(pil))[None].to(torch.float32).mul_(1.0 / 255)
            samples.append({"audio": a * one, "image": im * one,
                            "labels": torch.tensor(int(df["label"].iloc[r]), dtype=torch.long)})
            if len(samples) == batch or r == len(df) - 1:
                b = {k: torch.stack([s[k] for s in samples]) for k in ("audio", "image", "labels")}
                if device is not None:
                    b = {k: v.to(device) for k, v in b.items()}
                samples = []
                yield b
