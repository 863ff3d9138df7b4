"""Generate ``mmimdb_pool_b4.npz`` — golden vectors for the MMIMDb step with ``multimodal_pooling`` fusion
(run HERE only).

Imports the REAL reference modules (``models.mmimdb.MMIMDb`` with ``models.pooling.MultimodalPooling``,
``MMIMDbModalityEncoder``, ``MLPGenreClassifier``; ``experiment_utils.loss.LossFunctionGroup``) from
``/root/reference/MML_Suite`` with the throw-away stubs of ``make_golden.py``.  For each pooling type of
configs/mmimdb/centralised/pooling/mmimdb_pooling_{max,avg,sum,attention,gated}.yaml (hidden_dim 512,
dropout 0.1) it builds the model from ``torch.manual_seed(0)`` in YAML order (encoders, classifier, then
the pooling module inside MMIMDb.__init__), runs 2 reference ``train_step`` calls at B=4 with Adam(lr 1e-5,
wd 1e-3) and BCEWithLogits, and records the dropout masks the reference drew (pooling a / b, classifier
1 / 2), logits, losses, per-parameter gradient norms after step 1 and parameter sums after each step.
Then replays ``oracle/mmimdb_ref.py`` on the same masks and prints the differences (expected 0).  Only
numeric vectors are written.

Usage:  python tests/golden/make_mmimdb_pooling_golden.py
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MML_Suite"
B, N_STEPS = 4, 2
LR, WD = 1e-5, 1e-3
KINDS = ["max", "avg", "sum", "attention", "gated"]


class _NullRecorder:
    def update_group_all(self, *a, **k):
        pass


def main() -> None:
    sys.path.insert(0, HERE)
    from make_golden import _write_stubs
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from experiment_utils.loss import LossFunctionGroup
    from modalities import Modality
    from models.mmimdb import MLPGenreClassifier, MMIMDb, MMIMDbModalityEncoder

    sys.path.insert(0, REPO)
    from oracle import mmimdb_ref as orc
    from oracle.avmnist_ref import OracleAdam

    torch.set_num_threads(4)
    image, text, labels = orc.synthetic_batch(B, seed=4321)
    out = {"image": image.numpy(), "text": text.numpy(), "labels": labels.numpy()}
    for kind in KINDS:
        cfg = {"pooling_type": kind, "hidden_dim": 512, "dropout": 0.1}
        torch.manual_seed(0)
        ie = MMIMDbModalityEncoder(input_dim=4096, output_dim=512)
        te = MMIMDbModalityEncoder(input_dim=300, output_dim=512)
        clf = MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
        ref = MMIMDb(ie, te, multimodal_pooling=dict(cfg), classifier=clf)
        sd0 = {k: v.detach().clone() for k, v in ref.state_dict().items()}
        batch = {Modality.IMAGE: image, Modality.TEXT: text, "label": labels, "pattern_name": ["it"] * B}
        opt = torch.optim.Adam(ref.parameters(), lr=LR, weight_decay=WD)
        loss_fns = LossFunctionGroup.from_dict({"bce": {"loss_name": "bce_with_logits", "loss_args": {},
                                                        "weight": 1.0}})
        cap = {"pool": [], "m1": [], "m2": [], "logits": []}

        def hook(key):
            def f(mod, inp, o):
                if mod.training:
                    x = inp[0]
                    cap[key].append(torch.where(x != 0, o != 0, torch.ones_like(o, dtype=torch.bool)).to(torch.uint8))
            return f
        ref.fusion_module.dropout_layer.register_forward_hook(hook("pool"))  # called for a, then b
        ref.mm_mlp.net[2].register_forward_hook(hook("m1"))
        ref.mm_mlp.net[5].register_forward_hook(hook("m2"))
        ref.mm_mlp.register_forward_hook(lambda m, i, o: cap["logits"].append(o.detach().clone()) if m.training else None)
        losses, psums = [], []
        for step in range(N_STEPS):
            torch.manual_seed(500 + step)
            r = ref.train_step(batch, opt, loss_fns, torch.device("cpu"), _NullRecorder(), epoch=0)
            losses.append(r["loss"])
            psums.append([p.detach().double().sum().item() for p in ref.parameters()])
            if step == 0:
                out[f"{kind}/grad_norm_step1"] = np.array([p.grad.double().norm().item() for p in ref.parameters()])
        out[f"{kind}/losses"] = np.array(losses, dtype=np.float64)
        out[f"{kind}/param_sums"] = np.array(psums)
        out[f"{kind}/logits"] = np.stack([t.numpy() for t in cap["logits"]])
        pool = np.stack([t.numpy() for t in cap["pool"]]).reshape(N_STEPS, 2, B, -1)
        out[f"{kind}/keep_pool"] = pool
        out[f"{kind}/keep1"] = np.stack([t.numpy() for t in cap["m1"]])
        out[f"{kind}/keep2"] = np.stack([t.numpy() for t in cap["m2"]])
        out[f"{kind}/state_dict_keys"] = np.array(list(sd0.keys()))
        out[f"{kind}/param_names"] = np.array([n for n, _ in ref.named_parameters()])

        model = orc.build_oracle_mmimdb(0, pooling=cfg)
        assert list(model.state_dict().keys()) == list(sd0.keys()), (kind, "state_dict key mismatch")
        wdiff = max((model.state_dict()[k].double() - sd0[k].double()).abs().max().item() for k in sd0)
        oopt = OracleAdam(list(model.parameters()), lr=LR, weight_decay=WD)
        d = []
        for step in range(N_STEPS):
            kp = (torch.from_numpy(pool[step, 0]), torch.from_numpy(pool[step, 1]))
            r = orc.train_step(model, oopt, image, text, labels, torch.from_numpy(out[f"{kind}/keep1"][step]),
                               torch.from_numpy(out[f"{kind}/keep2"][step]), keep_pool=kp)
            d.append(abs(r["loss"].item() - losses[step]))
            d.append((r["logits"] - torch.from_numpy(out[f"{kind}/logits"][step])).abs().max().item())
        ps = [p.detach().double().sum().item() for p in model.parameters()]
        d.append(max(abs(a - b) for a, b in zip(ps, psums[-1])))
        print(f"{kind}: losses {losses}; oracle vs reference: init max|dw|={wdiff:.3e} max diff={max(d):.3e}")
    np.savez_compressed(os.path.join(HERE, "mmimdb_pool_b4.npz"), **out)


if __name__ == "__main__":
    main()
