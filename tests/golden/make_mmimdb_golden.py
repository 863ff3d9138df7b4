"""Generate ``mmimdb_step_b4.npz`` — golden vectors for the MMIMDb late-fusion step (run HERE only).

Imports the REAL reference modules (``models.mmimdb.MMIMDb``, ``MMIMDbModalityEncoder``,
``GatedBiModalNetwork``, ``MLPGenreClassifier``; ``experiment_utils.loss.LossFunctionGroup``) from
``/root/reference/MML_Suite`` with the same throw-away stubs as ``make_golden.py``, builds the model of
configs/mmimdb/centralised/mmimdb_baseline.yaml (image 4096→512, text 300→512, GMU 512/512, classifier
512/512/23) from ``torch.manual_seed(0)`` in YAML order, and runs 3 reference ``train_step`` calls at
B=4 on a seeded synthetic batch with Adam(lr 1e-5, wd 1e-3) and BCEWithLogits.  Records the dropout
masks the reference drew (forward hooks), logits, losses, per-parameter gradient norms and first/last
values after step 1, parameter sums after each step, BN running statistics and an eval-mode forward.
Then replays ``oracle/mmimdb_ref.py`` on the same masks and prints the differences (expected 0).
Only numeric vectors are written; no reference source is copied.

Usage:  python tests/golden/make_mmimdb_golden.py
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MML_Suite"
B = 4
N_STEPS = 3
LR, WD = 1e-5, 1e-3


class _NullRecorder:
    def update_group_all(self, *a, **k):
        pass


def _first_last(t: torch.Tensor, k: int = 8):
    f = t.reshape(-1)
    pad = lambda a: np.pad(a, (0, k - a.size)) if a.size < k else a
    return pad(f[:k].numpy()), pad(f[-k:].numpy())


def main() -> None:
    sys.path.insert(0, HERE)
    from make_golden import _write_stubs
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from models.mmimdb import MMIMDb, MMIMDbModalityEncoder, MLPGenreClassifier
    from models.gates import GatedBiModalNetwork
    from experiment_utils.loss import LossFunctionGroup
    from modalities import Modality

    sys.path.insert(0, REPO)
    from oracle import mmimdb_ref as orc
    from oracle.avmnist_ref import OracleAdam

    torch.set_num_threads(4)
    torch.manual_seed(0)
    ie = MMIMDbModalityEncoder(input_dim=4096, output_dim=512)
    te = MMIMDbModalityEncoder(input_dim=300, output_dim=512)
    gmu = GatedBiModalNetwork(input_one_dim=512, output_one_dim=512, input_two_dim=512, output_two_dim=512)
    clf = MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
    ref = MMIMDb(ie, te, gated_bimodal_network=gmu, classifier=clf)
    sd0 = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    h = hashlib.sha256()
    for k in sorted(sd0):
        h.update(k.encode()); h.update(sd0[k].contiguous().numpy().tobytes())
    print("state_dict entries:", len(sd0), "sha256:", h.hexdigest())

    image, text, labels = orc.synthetic_batch(B, seed=1234)
    batch = {Modality.IMAGE: image, Modality.TEXT: text, "label": labels, "pattern_name": ["it"] * B}
    opt = torch.optim.Adam(ref.parameters(), lr=LR, weight_decay=WD)
    loss_fns = LossFunctionGroup.from_dict({"bce": {"loss_name": "bce_with_logits", "loss_args": {}, "weight": 1.0}})

    captured = {"m1": [], "m2": [], "logits": []}

    def hook(key):
        def f(mod, inp, out):
            x = inp[0]
            keep = torch.where(x != 0, out != 0, torch.ones_like(out, dtype=torch.bool))
            captured[key].append(keep.to(torch.uint8).clone())
        return f

    ref.mm_mlp.net[2].register_forward_hook(hook("m1"))
    ref.mm_mlp.net[5].register_forward_hook(hook("m2"))
    ref.mm_mlp.register_forward_hook(lambda m, i, o: captured["logits"].append(o.detach().clone()))

    out, losses, psums = {}, [], []
    for step in range(N_STEPS):
        torch.manual_seed(200 + step)
        r = ref.train_step(batch, opt, loss_fns, torch.device("cpu"), _NullRecorder(), epoch=0)
        losses.append(r["loss"])
        psums.append([p.detach().double().sum().item() for p in ref.parameters()])
        if step == 0:
            out["grad_norm_step1"] = np.array([p.grad.double().norm().item() for p in ref.parameters()])
            fl = [_first_last(p.grad) for p in ref.parameters()]
            out["grad_first8_step1"] = np.stack([a for a, _ in fl]).astype(np.float32)
            out["grad_last8_step1"] = np.stack([b for _, b in fl]).astype(np.float32)
            bn_keys = [k for k in ref.state_dict() if k.endswith("running_mean") or k.endswith("running_var")]
            out["bn_stat_sum_step1"] = np.array([ref.state_dict()[k].double().sum().item() for k in bn_keys])
    out["losses"] = np.array(losses, dtype=np.float64)
    out["param_sums"] = np.array(psums)
    out["logits"] = np.stack([t.numpy() for t in captured["logits"]])
    out["keep1"] = np.stack([t.numpy() for t in captured["m1"]])
    out["keep2"] = np.stack([t.numpy() for t in captured["m2"]])
    ref.eval()
    with torch.no_grad():
        out["eval_logits"] = ref(I=image, T=text).numpy()
    out["image"] = image.numpy(); out["text"] = text.numpy(); out["labels"] = labels.numpy()
    out["param_names"] = np.array([n for n, _ in ref.named_parameters()])
    out["state_dict_keys"] = np.array(list(sd0.keys()))
    out["state_dict_sha256"] = np.array(h.hexdigest())
    np.savez_compressed(os.path.join(HERE, "mmimdb_step_b4.npz"), **out)
    print("losses:", losses)

    # ---- the oracle restatement on the same inputs / masks -------------------------------------
    model = orc.build_oracle_mmimdb(0)
    assert list(model.state_dict().keys()) == list(sd0.keys()), "state_dict key mismatch"
    wdiff = max((model.state_dict()[k].double() - sd0[k].double()).abs().max().item() for k in sd0)
    oopt = OracleAdam(list(model.parameters()), lr=LR, weight_decay=WD)
    d = []
    for step in range(N_STEPS):
        r = orc.train_step(model, oopt, image, text, labels, torch.from_numpy(out["keep1"][step]),
                           torch.from_numpy(out["keep2"][step]))
        d.append(abs(r["loss"].item() - losses[step]))
        d.append((r["logits"] - torch.from_numpy(out["logits"][step])).abs().max().item())
    print(f"oracle vs reference: init max|dw|={wdiff:.3e} max step diff={max(d):.3e}")


if __name__ == "__main__":
    main()
