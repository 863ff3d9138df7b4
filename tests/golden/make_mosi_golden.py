"""Generate ``mosi_step_b4.npz`` (or, with ``mosei``, ``mosei_step_b4.npz``) — golden vectors for the
UTT-Fusion step (run HERE only).

Imports the REAL reference modules (``models.msa.utt_fusion.UttFusionModel``, ``LSTMEncoder``,
``TextCNN``, ``FcClassifier``; ``experiment_utils.loss.LossFunctionGroup``) from
``/root/reference/MML_Suite`` with the throw-away stubs of ``make_golden.py``, builds the model of
configs/mosi/centralised/utt_fusion_base_training.yaml (LSTM 5→64 and 20→64 "last", TextCNN 768 → 3x128
(heights 3/4/5) → 64, FcClassifier 192 → 192/64/32 → 3, dropout 0.5, clip 1.0) from
``torch.manual_seed(0)`` in YAML order, and runs 3 reference ``train_step`` calls at B=4 (20 steps,
two samples zero-padded past their length as pad_sequence leaves them) with Adam(lr 1e-3, wd 1e-3) and
the cross-entropy loss group.  Records the dropout masks the reference drew (forward hooks on its
Dropout modules), logits, losses, the pre-clip total gradient norms clip_grad_norm_ returned,
per-parameter (clipped) gradient norms and first/last values after step 1, parameter sums after each
step and an eval-mode forward.  Then replays ``oracle/mosi_ref.py`` on the same masks and prints the
differences (expected 0: bit-exact on CPU).  Only numeric vectors are written.

``mosei``: the model of configs/mosei/centralised/utt_fusion_train_mosei.yaml instead (LSTM 74→64 and
35→64 "maxpool", TextCNN dropout 0.7, FcClassifier 192 → 96/48 → 3 with use_bn and dropout 0.66, clip 0.5,
Adam lr 2e-4 / wd 1e-5); the classifier's BatchNorm1d running statistics after each step are recorded too.

Usage:  python tests/golden/make_mosi_golden.py [mosei]
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
B, STEPS, N_STEPS = 4, 20, 3
LENGTHS = [20, 13, 20, 7]


class _NullRecorder:
    def update_group_all(self, *a, **k):
        pass


def _first_last(t: torch.Tensor, k: int = 8):
    f = t.reshape(-1)
    pad = lambda a: np.pad(a, (0, k - a.size)) if a.size < k else a  # noqa: E731
    return pad(f[:k].numpy()), pad(f[-k:].numpy())


def main(which: str = "mosi") -> None:
    sys.path.insert(0, HERE)
    from make_golden import _write_stubs
    stubdir = tempfile.mkdtemp(prefix="tspm_refstubs_")
    _write_stubs(stubdir)
    sys.path[:0] = [stubdir, REF]
    os.environ.setdefault("EXP_PATH", tempfile.mkdtemp(prefix="tspm_exp_"))
    import config.multimodal_training_config  # noqa: F401  (import order: train_multimodal.py:14)
    from experiment_utils.loss import LossFunctionGroup
    from modalities import Modality
    from models.msa.networks.classifier import FcClassifier
    from models.msa.networks.lstm import LSTMEncoder
    from models.msa.networks.textcnn import TextCNN
    from models.msa.utt_fusion import UttFusionModel

    sys.path.insert(0, REPO)
    from oracle import mosi_ref as orc

    cfg = orc.MOSEI if which == "mosei" else orc.MOSI
    LR, WD = cfg.lr, cfg.weight_decay
    torch.set_num_threads(4)
    torch.manual_seed(0)
    netA = LSTMEncoder(input_size=cfg.audio_dim, hidden_size=64, embd_method=cfg.embd_method)
    netV = LSTMEncoder(input_size=cfg.video_dim, hidden_size=64, embd_method=cfg.embd_method)
    netT = TextCNN(input_size=768, embd_size=64, dropout=cfg.text_dropout, in_channels=1, out_channels=128,
                   kernel_heights=[3, 4, 5])
    netC = FcClassifier(input_dim=192, layers=list(cfg.cls_layers), output_dim=3, dropout=cfg.cls_dropout,
                        use_bn=cfg.use_bn)
    ref = UttFusionModel(netA, netV, netT, netC, clip=cfg.clip)
    sd0 = {k: v.detach().clone() for k, v in ref.state_dict().items()}
    h = hashlib.sha256()
    for k in sorted(sd0):
        h.update(k.encode()); h.update(sd0[k].contiguous().numpy().tobytes())
    print("state_dict entries:", len(sd0), "sha256:", h.hexdigest())

    A, V, T, y = orc.synthetic_batch(B, STEPS, seed=1234, lengths=LENGTHS, cfg=cfg)
    batch = {Modality.AUDIO: A, Modality.VIDEO: V, Modality.TEXT: T, "label": y, "pattern_name": ["atv"] * B}
    opt = torch.optim.Adam(ref.parameters(), lr=LR, weight_decay=WD)
    loss_fns = LossFunctionGroup.from_dict({"cross_entropy": {"loss_name": "cross_entropy", "loss_args": {},
                                                               "weight": 1.0}})
    ncls = len(cfg.cls_layers)
    cap = {"text": [], "logits": [], "norm": [], **{f"cls{j}": [] for j in range(ncls)}}

    def hook(key):
        def f(mod, inp, out):
            x = inp[0]
            if mod.training:  # the eval forward does not drop
                keep = torch.where(x != 0, out != 0, torch.ones_like(out, dtype=torch.bool))
                cap[key].append(keep.to(torch.uint8).clone())
        return f
    drops = [i for i, m in enumerate(ref.netC.module) if isinstance(m, torch.nn.Dropout)]
    assert len(drops) == ncls
    if not cfg.use_bn:
        ref.netT.dropout.register_forward_hook(hook("text"))
        for j, idx in enumerate(drops):
            ref.netC.module[idx].register_forward_hook(hook(f"cls{j}"))
    else:
        # Dropout after BatchNorm1d: an input can be exactly 0 (a dead channel normalises to beta = 0) while
        # the mask still zeroes its gradient, so the mask cannot be read back from (input, output).  Draw it
        # explicitly instead, with ATen's dropout arithmetic (x * (bernoulli / (1 - p))), and record it.
        names = {id(ref.netT.dropout): "text", **{id(ref.netC.module[i]): f"cls{j}" for j, i in enumerate(drops)}}

        def drop_forward(mod, x):
            if not mod.training or mod.p == 0:
                return x
            keep = torch.rand(x.shape) >= mod.p
            cap[names[id(mod)]].append(keep.to(torch.uint8).clone())
            return x * (keep.to(x.dtype) / (1.0 - mod.p))
        for mod in (ref.netT.dropout, *[ref.netC.module[i] for i in drops]):
            mod.forward = drop_forward.__get__(mod)
    bns = [m for m in ref.netC.module if isinstance(m, torch.nn.BatchNorm1d)]
    ref.netC.register_forward_hook(lambda m, i, o: cap["logits"].append(o.detach().clone()) if m.training else None)
    orig_clip = torch.nn.utils.clip_grad_norm_

    def rec_clip(params, max_norm, *a, **k):
        n = orig_clip(params, max_norm, *a, **k)
        cap["norm"].append(float(n))
        return n
    torch.nn.utils.clip_grad_norm_ = rec_clip

    out, losses, psums, bnstats = {}, [], [], []
    for step in range(N_STEPS):
        torch.manual_seed(300 + step)
        r = ref.train_step(batch, opt, loss_fns, torch.device("cpu"), _NullRecorder())
        losses.append(r["loss"])
        psums.append([p.detach().double().sum().item() for p in ref.parameters()])
        bnstats.append([float(t.double().sum()) for bn in bns for t in (bn.running_mean, bn.running_var)] +
                       [int(bn.num_batches_tracked) for bn in bns])
        if step == 0:
            out["grad_norm_step1"] = np.array([p.grad.double().norm().item() for p in ref.parameters()])
            fl = [_first_last(p.grad) for p in ref.parameters()]
            out["grad_first8_step1"] = np.stack([a for a, _ in fl]).astype(np.float32)
            out["grad_last8_step1"] = np.stack([b for _, b in fl]).astype(np.float32)
    torch.nn.utils.clip_grad_norm_ = orig_clip
    out["losses"] = np.array(losses, dtype=np.float64)
    out["total_norms"] = np.array(cap["norm"], dtype=np.float64)
    out["param_sums"] = np.array(psums)
    if bns:
        out["bn_stat_sums"] = np.array(bnstats, dtype=np.float64)
    out["logits"] = np.stack([t.numpy() for t in cap["logits"]])
    keys = ["text"] + [f"cls{j}" for j in range(ncls)]
    for k in keys:
        out[f"keep_{k}"] = np.stack([t.numpy() for t in cap[k]])
    ref.eval()
    with torch.no_grad():
        out["eval_logits"] = ref(A, V, T).numpy()
    out["audio"], out["video"], out["text"], out["labels"] = A.numpy(), V.numpy(), T.numpy(), y.numpy()
    out["lengths"] = np.array(LENGTHS, dtype=np.int32)
    out["param_names"] = np.array([n for n, _ in ref.named_parameters()])
    out["state_dict_keys"] = np.array(list(sd0.keys()))
    out["state_dict_sha256"] = np.array(h.hexdigest())
    np.savez_compressed(os.path.join(HERE, f"{which}_step_b4.npz"), **out)
    print("losses:", losses, "norms:", cap["norm"])

    # ---- the oracle restatement on the same inputs / masks -------------------------------------
    model = orc.build_oracle_utt(0, cfg=cfg)
    assert list(model.state_dict().keys()) == list(sd0.keys()), "state_dict key mismatch"
    wdiff = max((model.state_dict()[k].double() - sd0[k].double()).abs().max().item() for k in sd0)
    oopt = orc.OracleAdam(list(model.parameters()), lr=LR, weight_decay=WD)
    d = []
    for step in range(N_STEPS):
        keeps = {k: torch.from_numpy(out[f"keep_{k}"][step]) for k in keys}
        r = orc.train_step(model, oopt, A, V, T, y, keeps)
        d.append(abs(r["loss"].item() - losses[step]))
        d.append((r["logits"] - torch.from_numpy(out["logits"][step])).abs().max().item())
        d.append(abs(float(r["total_norm"]) - cap["norm"][step]))
    print(f"oracle vs reference: init max|dw|={wdiff:.3e} max step diff={max(d):.3e}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "mosi")
