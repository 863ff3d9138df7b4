"""Golden vectors that pin oracle/monomodal_ref.py (run HERE, in the build container only).

Imports the REAL ``MML_Suite/train_monomodal.py`` (read-only; the throw-away stubs of make_golden.py
for its un-vendored imports, written to a temporary directory outside both repositories) and runs
``MonomodalEncoder.train_step`` three times and ``validation_step`` once on CPU, for the audio
(ResNet18, hidden 64) and the image (ResNet34, hidden 128) pre-training models of
configs/avmnist/mono/train_{audio,image}_encoder_resnet.yaml, on the seeded B=4 batch of
avmnist_step_b4.npz.  Records into ``avmnist_mono_b4.npz``: the seed-0 state_dict sha256 and keys,
per step the loss / accuracy / classifier logits / predictions handed to the metric recorder, step-1
gradient norms, final parameter sums, and the eval loss / logits / predictions.  Then re-runs the
oracle on the same inputs and prints the max difference (expected 0: bit-exact on CPU).  Only these
numeric vectors are written; nothing from the reference is copied.

The batches hold one modality key (plus labels / pattern names), so the reference's key choice
(train_monomodal.py:103-128, which depends on the un-vendored ``str(Modality)``) is unambiguous.

Usage:  python tests/golden/make_mono_golden.py
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MML_Suite"
B = 4
N_STEPS = 3


class _Recorder:
    """The metric_recorder surface train_step / validation_step use (config.groups, update_group)."""

    def __init__(self):
        self.config = SimpleNamespace(groups={"classification": ["accuracy"]})
        self.seen = []

    def update_group(self, group_name, predictions, targets, modality):
        self.seen.append((str(modality), predictions.detach().cpu().numpy().copy()))


def main() -> None:
    sys.path.insert(0, HERE)
    from make_golden import _write_stubs, make_lut
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    import train_monomodal as tm
    from experiment_utils.loss import LossFunctionGroup
    from models.msa.networks.resnet import ResNet18, ResNet34
    from modalities import Modality

    sys.path.insert(0, REPO)
    from oracle import avmnist_ref as orc
    from oracle import monomodal_ref as mref

    torch.set_num_threads(4)
    lut_t = torch.from_numpy(make_lut().astype(np.int64))
    audio, image, labels, _ = orc.synthetic_batch(B, seed=1234, lut=lut_t)
    loss_fns = LossFunctionGroup.from_dict({"cross_entropy": {"loss_name": "cross_entropy", "weight": 1.0}})
    cpu = torch.device("cpu")
    out = {"labels": labels.numpy()}
    cases = (("audio", ResNet18, 64, audio, Modality.AUDIO, "AVMNIST_Audio_Encoder_Resnet_Pretrain"),
             ("image", ResNet34, 128, image, Modality.IMAGE, "AVMNIST_Image_Encoder_Resnet_Pretrain"))
    for which, ctor, dim, x, mod, name in cases:
        torch.manual_seed(0)
        enc = ctor(in_channels=1, hidden_dim=dim)
        model = tm.MonomodalEncoder(encoder=enc, output_dim=dim, num_classes=10)
        sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        h = hashlib.sha256()
        for k in sorted(sd0):
            h.update(k.encode())
            h.update(sd0[k].contiguous().numpy().tobytes())
        opt = torch.optim.Adam(model.parameters(), lr=5e-4, weight_decay=1e-4)
        cfg = SimpleNamespace(experiment=SimpleNamespace(name=name))
        batch = {mod: x, "labels": labels, "pattern_name": [which[0]] * B, "missing_masks": {}}
        cap = []
        hook = model.classifier.register_forward_hook(lambda m, i, o: cap.append(o.detach().clone()))
        rec = _Recorder()
        losses, accs = [], []
        model.train()
        for s in range(N_STEPS):
            r = model.train_step(batch, opt, loss_fns, cpu, rec, cfg)
            losses.append(r["loss"])
            accs.append(r["metrics"]["accuracy"])
            if s == 0:
                out[f"{which}_grad_norm_step1"] = np.array([p.grad.double().norm().item() for p in model.parameters()])
        out[f"{which}_param_sum_final"] = np.array([p.detach().double().sum().item() for p in model.parameters()])
        model.eval()
        v = model.validation_step(batch, loss_fns, cpu, rec, cfg)
        hook.remove()
        out[f"{which}_losses"] = np.array(losses, dtype=np.float64)
        out[f"{which}_accuracy"] = np.array(accs, dtype=np.float64)
        out[f"{which}_logits"] = np.stack([c.numpy() for c in cap[:N_STEPS]])
        out[f"{which}_eval_logits"] = cap[N_STEPS].numpy()
        out[f"{which}_eval_loss"] = np.array(v["loss"], dtype=np.float64)
        out[f"{which}_preds"] = np.stack([p for _, p in rec.seen])  # 3 train steps + the eval step
        out[f"{which}_modality_str"] = np.array(rec.seen[0][0])
        out[f"{which}_x"] = x.numpy()
        out[f"{which}_state_dict_keys"] = np.array(list(sd0))
        out[f"{which}_state_dict_sha256"] = np.array(h.hexdigest())
        out[f"{which}_param_names"] = np.array([n for n, _ in model.named_parameters()])
        # ---- the oracle on the same inputs -------------------------------------------------------
        om = mref.build_oracle_monomodal(which, 0)
        assert list(om.state_dict()) == list(sd0), "state_dict key mismatch"
        d = [max((om.state_dict()[k].double() - sd0[k].double()).abs().max().item() for k in sd0)]
        oo = orc.OracleAdam(list(om.parameters()), lr=5e-4, weight_decay=1e-4)
        for s in range(N_STEPS):
            rr = mref.train_step(om, oo, x, labels)
            d.append(abs(rr["loss"].item() - losses[s]))
            d.append((rr["logits"] - cap[s]).abs().max().item())
            d.append(abs(rr["accuracy"].item() - accs[s]))
        ev = mref.validation_step(om, x, labels)
        d.append((ev["logits"] - cap[N_STEPS]).abs().max().item())
        d.append(abs(ev["loss"].item() - v["loss"]))
        print(f"{which}: losses {losses} accuracy {accs} modality key {rec.seen[0][0]!r} "
              f"oracle vs reference max diff {max(d):.3e}")
    np.savez_compressed(os.path.join(HERE, "avmnist_mono_b4.npz"), **out)


if __name__ == "__main__":
    main()
