"""Generate the golden vectors that pin the oracle (run HERE, in the survey/build container only).

It imports the REAL reference modules from ``/root/reference/MML_Suite`` (read-only) with throw-away
stubs for its un-vendored / absent imports (``modalities``, ``h5py``, ``torchvision.transforms.v2``,
and ``transformers`` only if it is not importable) written into a temporary directory outside both
repositories, runs the reference ``AVMNIST.train_step`` on CPU, and records:

* ``avmnist_step_b4.npz`` — seed-0 weights (checked by sha256 + sample values), a seeded synthetic
  batch (B=4), the dropout keep-masks the reference drew, logits / loss / embeddings of 3 consecutive
  train steps, per-parameter gradient norms + first/last values after step 1, post-step parameter
  checksums, BN running statistics, and an eval-mode forward;
* ``lut_gist_earth_L.bin`` — the 256-entry uint8 LUT of ``cm.gist_earth`` → RGBA·255 → PIL "L"
  (MML_Suite/data/avmnist.py:186-191).

It then runs ``oracle/avmnist_ref.py`` on the same inputs/masks and reports the max abs difference
(expected 0: bit-exact on CPU).  Nothing from the reference is copied into the repository; only
these numeric vectors are written.

Usage:  python tests/golden/make_golden.py
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
B = 4
N_STEPS = 3


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
                return Modality(str(name).lower())
            def create_missing_mask(n_modalities, batch, rates):
                import torch
                return torch.ones(batch, n_modalities)
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


def make_lut() -> np.ndarray:
    from matplotlib import cm
    from PIL import Image
    idx = np.arange(256, dtype=np.uint8).reshape(16, 16)
    img = Image.fromarray(np.uint8(cm.gist_earth(idx) * 255)).convert("L")
    return np.array(img, dtype=np.uint8).reshape(256)


class _NullRecorder:
    def update_group_all(self, *a, **k):
        pass


def main() -> None:
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from models.avmnist import AVMNIST
    from models.msa.networks.resnet import ResNet18, ResNet34
    from experiment_utils.loss import LossFunctionGroup
    from modalities import Modality

    sys.path.insert(0, REPO)
    from oracle import avmnist_ref as orc

    torch.set_num_threads(4)
    lut = make_lut()
    lut_t = torch.from_numpy(lut.astype(np.int64))
    with open(os.path.join(HERE, "lut_gist_earth_L.bin"), "wb") as f:
        f.write(lut.tobytes())

    # reference model, seeded construction order = YAML order (audio R18, image R34, AVMNIST)
    torch.manual_seed(0)
    ref_a = ResNet18(in_channels=1, hidden_dim=64)
    ref_i = ResNet34(in_channels=1, hidden_dim=128)
    ref = AVMNIST(ref_a, ref_i, 128, dropout=0.5, fusion_fn="concat")
    sd0 = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    h = hashlib.sha256()
    for k in sorted(sd0):
        h.update(k.encode()); h.update(sd0[k].contiguous().numpy().tobytes())
    print("state_dict entries:", len(sd0), "sha256:", h.hexdigest())

    audio, image, labels, img_u8 = orc.synthetic_batch(B, seed=1234, lut=lut_t)
    batch = {Modality.AUDIO: audio, Modality.IMAGE: image, "labels": labels, "pattern_name": ["ai"] * B,
             "missing_masks": {}}
    opt = torch.optim.Adam(ref.parameters(), lr=5e-4, weight_decay=1e-4)
    loss_fns = LossFunctionGroup.from_dict({"cross_entropy": {"loss_name": "cross_entropy", "weight": 1.0}})

    captured = {}

    def drop_hook(mod, inp, out):
        x = inp[0]
        keep = torch.where(x != 0, (out != 0), torch.ones_like(out, dtype=torch.bool))
        captured.setdefault("masks", []).append(keep.to(torch.uint8).clone())

    def net_hook(mod, inp, out):
        captured.setdefault("logits", []).append(out.detach().clone())
        captured.setdefault("fused", []).append(inp[0].detach().clone())

    ref.net[2].register_forward_hook(drop_hook)
    ref.net.register_forward_hook(net_hook)

    out = {}
    names = [n for n, _ in ref.named_parameters()]
    losses = []
    for step in range(N_STEPS):
        torch.manual_seed(100 + step)
        r = ref.train_step(batch, opt, loss_fns, torch.device("cpu"), _NullRecorder())
        losses.append(r["loss"])
        if step == 0:
            gnorm = np.array([p.grad.double().norm().item() for p in ref.parameters()])
            gfirst = np.stack([p.grad.reshape(-1)[:8].numpy() if p.numel() >= 8 else
                               np.pad(p.grad.reshape(-1).numpy(), (0, 8 - p.numel())) for p in ref.parameters()])
            glast = np.stack([p.grad.reshape(-1)[-8:].numpy() if p.numel() >= 8 else
                              np.pad(p.grad.reshape(-1).numpy(), (0, 8 - p.numel())) for p in ref.parameters()])
            out["grad_norm_step1"] = gnorm
            out["grad_first8_step1"] = gfirst.astype(np.float32)
            out["grad_last8_step1"] = glast.astype(np.float32)
            out["param_sum_step1"] = np.array([p.detach().double().sum().item() for p in ref.parameters()])
            out["param_abssum_step1"] = np.array([p.detach().double().abs().sum().item() for p in ref.parameters()])
            bn_keys = [k for k in ref.state_dict() if k.endswith("running_mean") or k.endswith("running_var")]
            out["bn_stat_sum_step1"] = np.array([ref.state_dict()[k].double().sum().item() for k in bn_keys])
            out["bn_stat_first8_step1"] = np.stack([ref.state_dict()[k][:8].numpy() for k in bn_keys])
    out["losses"] = np.array(losses, dtype=np.float64)
    out["logits"] = np.stack([t.numpy() for t in captured["logits"]])
    out["fused"] = np.stack([t.numpy() for t in captured["fused"]])
    out["keep_masks"] = np.stack([t.numpy() for t in captured["masks"]])
    out["param_sum_final"] = np.array([p.detach().double().sum().item() for p in ref.parameters()])
    ref.eval()
    with torch.no_grad():
        out["eval_logits"] = ref(A=audio, I=image).numpy()
    out["audio"] = audio.numpy(); out["image"] = image.numpy(); out["image_u8"] = img_u8.numpy()
    out["labels"] = labels.numpy()
    out["w_sample_first8"] = np.stack([sd0[n].reshape(-1)[:8].numpy() if sd0[n].numel() >= 8 else
                                       np.pad(sd0[n].reshape(-1).numpy(), (0, 8 - sd0[n].numel())) for n in names])
    out["param_names"] = np.array(names)
    out["state_dict_keys"] = np.array(list(sd0.keys()))
    out["state_dict_sha256"] = np.array(h.hexdigest())
    np.savez_compressed(os.path.join(HERE, "avmnist_step_b4.npz"), **out)
    print("losses:", losses)

    # ---- check the oracle restatement against what the reference produced -----------------------
    model = orc.build_oracle_avmnist(seed=0)
    assert list(model.state_dict().keys()) == list(sd0.keys()), "state_dict key mismatch"
    wdiff = max((model.state_dict()[k].double() - sd0[k].double()).abs().max().item() for k in sd0)
    oopt = orc.OracleAdam(list(model.parameters()), lr=5e-4, weight_decay=1e-4)
    od = []
    for step in range(N_STEPS):
        keep = torch.from_numpy(out["keep_masks"][step])
        r = orc.train_step(model, oopt, audio, image, labels, keep)
        od.append(abs(r["loss"].item() - losses[step]))
        od.append((r["logits"] - torch.from_numpy(out["logits"][step])).abs().max().item())
    pdiff = max(abs(a - b) for a, b in zip([p.detach().double().sum().item() for p in model.parameters()],
                                           out["param_sum_final"]))
    print(f"oracle vs reference: init max|dw|={wdiff:.3e} step max diff={max(od):.3e} param-sum diff={pdiff:.3e}")


if __name__ == "__main__":
    main()
