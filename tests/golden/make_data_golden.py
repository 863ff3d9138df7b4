"""Generate tests/golden/avmnist_data.npz by running the REAL reference input stage
(MML_Suite/data/avmnist.py ``AVMNIST`` dataset + ``collate_fn`` + data/base_dataset.py, via
``torch.utils.data.DataLoader``) over a small corpus written in the reference's file format
(CSV of per-sample ``.pt`` paths: audio = ``torch.save`` of a float32 [32,94] tensor, image =
``torch.save`` of a uint8 [28,28] numpy array, data/avmnist.py:135-191).

Run here (the reference is importable in this container; it never travels to the GPU box):

    python tests/golden/make_data_golden.py

Stubs for the un-vendored / absent packages are written to a temp dir (as make_golden.py does):
``modalities`` (Modality enum; ``create_missing_mask(n, batch, rates)`` returns 1 where a uniform draw
is >= the missing rate — deterministic for AVMNIST's 0.0 / 1.0 rates), ``torchvision.transforms.v2``
(``PILToTensor`` = ``torch.from_numpy(np.array(img))[None]``, ``ToDtype(float32, scale=True)`` =
``to(float32).mul_(1/255)``), ``h5py``.  The corpus itself comes from ``oracle.avmnist_ref.synthetic_batch``
(regenerable from the seed), so the fixture stores the outputs, not the inputs.
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile
import textwrap

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MML_Suite"
N = 6
SEED = 4321
BATCH = 4


def _write_stubs(root: str) -> None:
    files = {
        "modalities/__init__.py": """
            from enum import Enum
            class Modality(Enum):
                AUDIO = "audio"; IMAGE = "image"; TEXT = "text"; VIDEO = "video"; MULTIMODAL = "multimodal"
                @classmethod
                def from_str(cls, s):
                    return cls(str(s).lower())
                def __str__(self):
                    return self.value
            def add_modality(name):
                return Modality(name)
            def create_missing_mask(n_modalities, batch, rates):
                import torch
                g = torch.Generator().manual_seed(0)
                u = torch.rand(batch, n_modalities, generator=g)
                return (u >= torch.tensor(rates, dtype=torch.float32)).float()
            """,
        "h5py/__init__.py": "File = None\n",
        "torchvision/__init__.py": "",
        "torchvision/transforms/__init__.py": "",
        "torchvision/transforms/v2/__init__.py": """
            import numpy as np, torch
            class PILToTensor:
                def __call__(self, img):
                    return torch.from_numpy(np.array(img))[None]
            class ToDtype:
                def __init__(self, dtype, scale=False):
                    self.dtype, self.scale = dtype, scale
                def __call__(self, t):
                    return t.to(self.dtype).mul_(1.0 / 255) if self.scale else t.to(self.dtype)
            """,
    }
    try:
        import transformers  # noqa: F401
    except Exception:
        files["transformers/__init__.py"] = "class BertModel: pass\nclass BertTokenizer: pass\nclass BertConfig: pass\n"
    for rel, body in files.items():
        p = os.path.join(root, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(textwrap.dedent(body))


def write_corpus(root: str):
    """The corpus in the reference's file layout; returns (csv path, audio, image_u8, labels)."""
    sys.path.insert(0, REPO)
    from oracle import avmnist_ref as orc
    audio, _, labels, img_u8 = orc.synthetic_batch(N, seed=SEED)
    rows = ["audio,image,label"]
    for i in range(N):
        ap, ip = os.path.join(root, f"audio_{i}.pt"), os.path.join(root, f"image_{i}.pt")
        torch.save(audio[i].clone(), ap)
        torch.save(img_u8[i].numpy().copy(), ip)
        rows.append(f"{ap},{ip},{int(labels[i])}")
    csv = os.path.join(root, "corpus.csv")
    with open(csv, "w") as f:
        f.write("\n".join(rows) + "\n")
    return csv, audio.numpy(), img_u8.numpy(), labels.numpy()


# (split, target modality, selected patterns)
CASES = [("train", "MULTIMODAL", ["ai"]), ("valid", "MULTIMODAL", ["ai", "a", "i"]), ("test", "IMAGE", ["i", "ai"])]


def main() -> None:
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from data.avmnist import AVMNIST
    from modalities import Modality

    corpus_dir = tempfile.mkdtemp(prefix="tspm_avmnist_corpus_")
    csv, audio, img_u8, labels = write_corpus(corpus_dir)
    out = {"n": np.int64(N), "seed": np.int64(SEED), "batch": np.int64(BATCH)}
    for ci, (split, target, sel) in enumerate(CASES):
        ds = AVMNIST(csv, split, Modality[target], selected_patterns=sel)
        dl = torch.utils.data.DataLoader(ds, batch_size=BATCH, shuffle=False, collate_fn=ds.collate_fn)
        out[f"c{ci}_len"] = np.int64(len(ds))
        for bi, b in enumerate(dl):
            key = f"c{ci}_b{bi}"
            out[key + "_labels"] = b["labels"].numpy()
            out[key + "_pattern"] = np.array(b["pattern_name"])
            out[key + "_mask_keys"] = np.int64(len(b["missing_masks"]))
            for m in (Modality.AUDIO, Modality.IMAGE):
                if m in b:
                    t = b[m].contiguous()
                    out[f"{key}_{m.value}_shape"] = np.array(t.shape, dtype=np.int64)
                    out[f"{key}_{m.value}_sha256"] = np.array(hashlib.sha256(t.numpy().tobytes()).hexdigest())
                    if m is Modality.IMAGE:
                        out[f"{key}_image"] = t.numpy()
        out[f"c{ci}_batches"] = np.int64(bi + 1)
    dst = os.path.join(HERE, "avmnist_data.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, "keys:", len(out))


if __name__ == "__main__":
    main()
