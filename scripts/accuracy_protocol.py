"""Accuracy parity on the reference's OWN training protocol (verdict r3 item 6; BASELINE north star "final
accuracy within ±0.2 pp of the reference after equal epochs").

The reference's loop (MML_Suite/train_multimodal.py:554-917 with configs/avmnist/centralised/
train_avmnist_resnet.yaml): up to 20 epochs; after every training epoch a validation epoch over the patterns
ai / a / i (`selected_patterns` of the validation split; a pattern zeroes the absent modality,
data/base_dataset.py:76-92) whose mean batch loss drives `check_early_stopping` (patience 10, min_delta
1e-3 — TrainingConfig's default, multimodal_training_config.py:48; mode minimize on `loss`) — a strictly
better loss saves `best.pth` — and `ReduceLROnPlateau` (the YAML's `scheduler_kwargs` never reach the
scheduler: get_scheduler passes `training.scheduler_args`, empty, multimodal_training_config.py:177, so
torch's defaults: factor 0.1, patience 10, threshold 1e-4 rel); after the loop `best.pth` is reloaded and the
test split is evaluated (:862-917, :889).

Data: the reference's own sample files, paired as in scripts/accuracy_parity.py (24,000 train / 6,000 test
pairs, test speakers 48-59).  The validation split is carved speaker-disjoint from the train pairs: speakers
40-47 (4,000 pairs, 12,000 items over the 3 patterns); training uses speakers 0-39 (20,000 pairs).

Pre-registered end point: TEST ACCURACY OF best.pth on pattern "ai" (both modalities), paired over runs
(same initial weights, batch order and dropout masks on both sides), TOST at ±0.2 pp (90 % interval).
Secondary: test accuracy over all three patterns, best epoch, stop epoch.

  python scripts/accuracy_protocol.py reference --device cuda --seeds 0      # GPU box (ATen reference)
  python scripts/accuracy_protocol.py ours --seeds 0                         # GPU box (HIP path)
  python scripts/accuracy_protocol.py pt_reference|pt_ours --seeds 0         # pretrained encoders (10 mono epochs)
  python scripts/accuracy_protocol.py compare --out profiles/r4_accuracy_parity.json [--pt]
"""
from __future__ import annotations

import argparse
import copy
import glob
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
import accuracy_parity as AP  # noqa: E402  (data pairing, batch orders, dropout masks, pretraining orders)

EPOCHS, PATIENCE, MIN_DELTA = 20, 10, 1e-3
PLATEAU = dict(factor=0.1, patience=10, threshold=1e-4)  # torch.optim.lr_scheduler.ReduceLROnPlateau defaults
LR, WD = 5e-4, 1e-4
PATTERNS = (("ai", 1.0, 1.0), ("a", 1.0, 0.0), ("i", 0.0, 1.0))
SPLIT_K = 2000  # per digit: k < 2000 -> speakers 0-39 (train), 2000 <= k < 2400 -> speakers 40-47 (validation)


SMOKE = os.environ.get("ACC_SMOKE") == "1"  # plumbing check: a few batches per split, 2 epochs


def split_rows():
    per = AP.TRAIN_PER_DIGIT
    train = np.array([d * per + k for d in range(10) for k in range(SPLIT_K)], np.int64)
    val = np.array([d * per + k for d in range(10) for k in range(SPLIT_K, per)], np.int64)
    if SMOKE:
        train, val = train[::50], val[::40]
    return train, val


def pattern_items(rows: np.ndarray):
    """(rows, audio mask, image mask, pattern id) of the 3-pattern evaluation set, pattern-major (idx // N)."""
    r = np.concatenate([rows] * len(PATTERNS))
    am = np.concatenate([np.full(len(rows), a, np.float32) for _, a, _ in PATTERNS])
    im = np.concatenate([np.full(len(rows), i, np.float32) for _, _, i in PATTERNS])
    pid = np.concatenate([np.full(len(rows), k, np.int64) for k in range(len(PATTERNS))])
    return r, am, im, pid


def check_early_stopping(loss, best, wait):
    """train_multimodal.py:329-376, mode minimize on `loss`: (is_best, should_continue, wait)."""
    if best is None or loss < best - MIN_DELTA:
        return True, True, 0
    wait += 1
    return False, wait < PATIENCE, wait


class Plateau:
    """torch.optim.lr_scheduler.ReduceLROnPlateau(mode='min') with the defaults, on a plain lr value."""

    def __init__(self, lr):
        self.lr, self.best, self.bad = lr, float("inf"), 0

    def step(self, loss):
        if loss < self.best * (1.0 - PLATEAU["threshold"]):
            self.best, self.bad = loss, 0
        else:
            self.bad += 1
        if self.bad > PLATEAU["patience"]:
            new = self.lr * PLATEAU["factor"]
            if self.lr - new > 1e-8:
                self.lr = new
            self.bad = 0
        return self.lr


def _protocol(train_epoch, eval_items, set_lr, get_state, set_state, epochs=2 if SMOKE else EPOCHS):
    """The reference's _train_loop + test with early stopping / plateau / best reload, on callbacks."""
    tr_rows, va_rows = split_rows()
    va = pattern_items(va_rows)
    best, wait, best_state, best_epoch = None, 0, None, None
    sched = Plateau(LR)
    curve = []
    for ep in range(epochs):
        t0 = time.time()
        tr_loss = train_epoch(ep, tr_rows)
        va_loss, va_acc = eval_items("train", *va)
        is_best, cont, wait = check_early_stopping(va_loss, best, wait)
        if is_best:
            best, best_state, best_epoch = va_loss, get_state(), ep + 1
        curve.append({"epoch": ep + 1, "train_loss": tr_loss, "val_loss": va_loss,
                      "val_accuracy": va_acc, "lr": sched.lr, "is_best": is_best,
                      "seconds": round(time.time() - t0, 2)})
        print(json.dumps(curve[-1]), flush=True)
        if not cont:
            break
        set_lr(sched.step(va_loss))
    set_state(best_state)
    te_rows = np.arange(AP.TEST_PER_DIGIT * 10, dtype=np.int64)[::60 if SMOKE else 1]
    te = pattern_items(te_rows)
    te_loss, te_acc = eval_items("test", *te)
    return {"curve": curve, "best_epoch": best_epoch, "stop_epoch": len(curve), "best_val_loss": best,
            "test_loss": te_loss, "test_accuracy": te_acc}


# ------------------------------------------------------------------------------------------------ reference
def _ref_setup(device):
    from oracle import avmnist_eval_ref as eref
    from oracle import avmnist_ref as orc
    tr, te = AP._load()
    dev = torch.device(device)
    lut = torch.from_numpy(AP._lut().astype(np.int64))

    def tensors(c, rows, am=None, im=None):
        a = torch.from_numpy(np.asarray(c.audio[rows]))
        i = (lut[torch.from_numpy(np.asarray(c.image[rows])).long()].float() * (1.0 / 255.0)).unsqueeze(1)
        if am is not None:
            a = a * torch.from_numpy(am)[:, None, None]
            i = i * torch.from_numpy(im)[:, None, None, None]
        return a.to(dev), i.to(dev), torch.from_numpy(np.asarray(c.labels[rows])).to(dev)
    return orc, eref, tr, te, dev, tensors


def _ref_run(seed, device, model, opts, orc, eref, tr, te, dev, tensors):
    class _All:
        def step(self):
            for o in opts:
                o.step()

    def train_epoch(ep, rows):
        order = rows[AP._order(len(rows), ep, seed).numpy()]
        losses = []
        model.train()
        for b in range(0, len(order), AP.BATCH):
            a, i, lab = tensors(tr, order[b:b + AP.BATCH])
            keep = AP._keep(seed, ep, b // AP.BATCH, lab.numel()).to(dev)
            losses.append(orc.train_step(model, _All(), a, i, lab, keep)["loss"].detach())
        return float(np.mean([x.item() for x in losses]))

    @torch.no_grad()
    def eval_items(split, rows, am, im, pid):
        c = tr if split == "train" else te
        model.eval()
        losses, correct = [], np.zeros(len(PATTERNS), np.int64)
        for b in range(0, len(rows), AP.BATCH):
            sl = slice(b, b + AP.BATCH)
            a, i, lab = tensors(c, rows[sl], am[sl], im[sl])
            r = eref.validation_step(model, a, i, lab)
            losses.append(float(r["loss"]))
            ok = (r["preds"] == lab).cpu().numpy()
            np.add.at(correct, pid[sl], ok)
        n = len(rows) // len(PATTERNS)
        acc = {p: float(correct[k]) / n for k, (p, _, _) in enumerate(PATTERNS)}
        acc["all"] = float(correct.sum()) / len(rows)
        return float(np.mean(losses)), acc

    def set_lr(lr):
        for o in opts:
            o.lr = lr

    def get_state():
        return copy.deepcopy(model.state_dict())

    def set_state(sd):
        model.load_state_dict(sd)
    return _protocol(train_epoch, eval_items, set_lr, get_state, set_state)


def reference(seed, device="cuda"):
    orc, eref, tr, te, dev, tensors = _ref_setup(device)
    model = orc.build_oracle_avmnist(seed).to(dev)
    opts = [orc.OracleAdam(list(model.parameters()), lr=LR, weight_decay=WD)]
    res = _ref_run(seed, device, model, opts, orc, eref, tr, te, dev, tensors)
    _save("reference", seed, res, "reference (oracle = the reference's torch code, ATen/MIOpen on the MI355X)")


def pt_reference(seed, device="cuda", mono_epochs=1 if SMOKE else 10):
    from oracle import monomodal_ref as mref
    orc, eref, tr, te, dev, tensors = _ref_setup(device)
    tr_rows, _ = split_rows()
    sds, mono = {}, []
    for modality in ("audio", "image"):
        mm = mref.build_oracle_monomodal(modality, seed + 100).to(dev)
        opt = orc.OracleAdam(list(mm.parameters()), lr=LR, weight_decay=WD)
        for ep in range(mono_epochs):
            order = tr_rows[AP._mono_order(len(tr_rows), modality, ep, seed).numpy()]
            for b in range(0, len(order), AP.BATCH):
                a, i, lab = tensors(tr, order[b:b + AP.BATCH])
                mref.train_step(mm, opt, a if modality == "audio" else i, lab)
        sds[modality] = {k: v.detach().clone() for k, v in mm.encoder.state_dict().items()}
        mono.append(modality)
    model = orc.build_oracle_avmnist(seed).to(dev)
    model.audio_encoder.load_state_dict(sds["audio"])
    model.image_encoder.load_state_dict(sds["image"])
    opts = [orc.OracleAdam(list(model.parameters()), lr=LR, weight_decay=WD)]  # the reference's ONE group
    res = _ref_run(seed, device, model, opts, orc, eref, tr, te, dev, tensors)
    _save("pt_reference", seed, res, "reference, pretrained encoders (10 monomodal epochs each)")


# ------------------------------------------------------------------------------------------------ ours
def _ours_run(seed, model, opt, dtr, dte):
    from tspm_amd.step import FusedEvalStep
    import tspm_amd
    dev = next(model.parameters()).device
    steps, evals = {}, {}

    def train_epoch(ep, rows):
        order = torch.from_numpy(rows[AP._order(len(rows), ep, seed).numpy()]).to(dev)
        losses = []
        for b in range(0, len(order), AP.BATCH):
            idx = order[b:b + AP.BATCH].contiguous()
            n = idx.numel()
            st = steps.get(n) or steps.setdefault(n, tspm_amd.FusedTrainStep(model, opt, None, n))
            dtr.gather(idx, out=(st.A, st.I, st.labels))
            st.keep_override = AP._keep(seed, ep, b // AP.BATCH, n).to(dev, non_blocking=True)
            st.run()
            losses.append(st.loss.clone())
        return float(np.mean([x.item() for x in losses]))

    @torch.no_grad()
    def eval_items(split, rows, am, im, pid):
        c = dtr if split == "train" else dte
        rows_d, am_d, im_d = (torch.from_numpy(x).to(dev) for x in (rows, am, im))
        pid_d = torch.from_numpy(pid).to(dev)
        losses, correct = [], torch.zeros(len(PATTERNS), dtype=torch.int64, device=dev)
        for b in range(0, len(rows), AP.BATCH):
            sl = slice(b, b + AP.BATCH)
            idx = rows_d[sl].contiguous()
            n = idx.numel()
            ev = evals.get(n) or evals.setdefault(n, FusedEvalStep(model, None, n))
            c.gather(idx, am_d[sl].contiguous(), im_d[sl].contiguous(), out=(ev.A, ev.I, ev.labels))
            ev.run()
            losses.append(ev.loss.clone())
            correct.index_add_(0, pid_d[sl], (ev.preds == ev.labels).long())
        correct = correct.cpu().numpy()
        n = len(rows) // len(PATTERNS)
        acc = {p: float(correct[k]) / n for k, (p, _, _) in enumerate(PATTERNS)}
        acc["all"] = float(correct.sum()) / len(rows)
        return float(np.mean([x.item() for x in losses])), acc

    def set_lr(lr):
        for g in opt.param_groups:
            g["lr"] = lr

    def get_state():
        return {k: v.detach().clone() for k, v in model.state_dict().items()}

    def set_state(sd):
        with torch.no_grad():
            for k, v in model.state_dict().items():
                v.copy_(sd[k])  # in place: the captured graphs keep their buffers
    return _protocol(train_epoch, eval_items, set_lr, get_state, set_state)


def _ours_setup():
    from tspm_amd.data import DeviceCorpus
    dev = torch.device("cuda", 0)
    tr, te = AP._load()
    return dev, DeviceCorpus(tr, dev), DeviceCorpus(te, dev)


def ours(seed):
    import tspm_amd
    dev, dtr, dte = _ours_setup()
    torch.manual_seed(seed)  # the reference side's build_oracle_avmnist(seed)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=LR, weight_decay=WD)
    _save("ours", seed, _ours_run(seed, model, opt, dtr, dte), "ours (HIP path, MI355X)")


def pt_ours(seed, mono_epochs=1 if SMOKE else 10):
    import tspm_amd
    from tspm_amd.monomodal import FusedMonoStep, MonomodalEncoder
    dev, dtr, dte = _ours_setup()
    tr_rows, _ = split_rows()
    sds = {}
    for modality in ("audio", "image"):
        torch.manual_seed(seed + 100)
        enc, dim = ((tspm_amd.ResNet18(1, 64), 64) if modality == "audio" else (tspm_amd.ResNet34(1, 128), 128))
        mm = MonomodalEncoder(enc, dim, 10).to(dev)
        opt = tspm_amd.FusedAdam(mm.parameters(), lr=LR, weight_decay=WD)
        steps = {}
        for ep in range(mono_epochs):
            order = torch.from_numpy(tr_rows[AP._mono_order(len(tr_rows), modality, ep, seed).numpy()]).to(dev)
            for b in range(0, len(order), AP.BATCH):
                idx = order[b:b + AP.BATCH].contiguous()
                a, i, lab = dtr.gather(idx, want_audio=modality == "audio", want_image=modality == "image")
                x = a if modality == "audio" else i
                st = steps.get(x.shape[0]) or steps.setdefault(x.shape[0], FusedMonoStep(mm, opt, None, x.shape))
                st.step(x, lab)
        sds[modality] = {k: v.detach().clone() for k, v in mm.encoder.state_dict().items()}
    torch.manual_seed(seed)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    model.audio_encoder.load_state_dict(sds["audio"])
    model.image_encoder.load_state_dict(sds["image"])
    opt = tspm_amd.FusedAdam(model.parameters(), lr=LR, weight_decay=WD)
    _save("pt_ours", seed, _ours_run(seed, model, opt, dtr, dte), "ours, pretrained encoders (10 monomodal epochs each)")


def _save(side, seed, res, desc):
    os.makedirs(AP.OUT, exist_ok=True)
    with open(os.path.join(AP.OUT, f"accproto_{side}_s{seed}.json"), "w") as f:
        json.dump(dict(res, side=desc, seed=seed), f, indent=1)
    print(json.dumps({"seed": seed, "best_epoch": res["best_epoch"], "stop_epoch": res["stop_epoch"],
                      "test_accuracy": res["test_accuracy"]}), flush=True)


# ------------------------------------------------------------------------------------------------ compare
def compare(out_path, pt=False, seed_range=None):
    from scipy import stats
    rs, os_ = ("pt_reference", "pt_ours") if pt else ("reference", "ours")

    def runs(side):
        return {json.load(open(p))["seed"]: json.load(open(p))
                for p in sorted(glob.glob(os.path.join(AP.OUT, f"accproto_{side}_s*.json")))}
    ref, our = runs(rs), runs(os_)
    seeds = sorted(set(ref) & set(our))
    if seed_range is not None:  # a pre-registered seed block, analysed alone (round 6: 200-295)
        seeds = [s for s in seeds if seed_range[0] <= s <= seed_range[1]]

    def tost(o, r):
        d = 100 * (np.asarray(o) - np.asarray(r))
        m, sd = float(d.mean()), float(d.std(ddof=1))
        se = sd / np.sqrt(len(d))
        t90 = float(stats.t.ppf(0.95, len(d) - 1))
        t95 = float(stats.t.ppf(0.975, len(d) - 1))
        return {"delta_pp": round(m, 3), "paired_sd_pp": round(sd, 3), "median_delta_pp": round(float(np.median(d)), 3),
                "ci90_pp": [round(m - t90 * se, 3), round(m + t90 * se, 3)],
                "ci95_pp": [round(m - t95 * se, 3), round(m + t95 * se, 3)],
                "equivalent_at_0.2pp": bool(m - t90 * se > -0.2 and m + t90 * se < 0.2)}
    doc = {"what": __doc__.split("\n\n")[0], "protocol": {"epochs": EPOCHS, "early_stopping_patience": PATIENCE,
                                                          "min_delta": MIN_DELTA, "plateau": PLATEAU, "lr": LR,
                                                          "weight_decay": WD, "batch": AP.BATCH,
                                                          "validation": "speakers 40-47 of the train pairs, patterns "
                                                                        "ai/a/i (12,000 items)",
                                                          "train": "speakers 0-39 (20,000 pairs)",
                                                          "test": "speakers 48-59 (6,000 pairs x 3 patterns)"},
           "setting": "pretrained encoders (10 monomodal epochs each), one Adam group" if pt else "from scratch",
           "seeds": seeds, "paired_runs": len(seeds),
           "endpoint": "test accuracy of best.pth, pattern ai (pre-registered)"}
    for key in ("ai", "all"):
        o = [our[s]["test_accuracy"][key] for s in seeds]
        r = [ref[s]["test_accuracy"][key] for s in seeds]
        doc[f"test_accuracy_{key}"] = {"reference_mean": round(float(np.mean(r)), 5), "ours_mean": round(float(np.mean(o)), 5),
                                       "paired": tost(o, r), "reference": r, "ours": o}
    doc["best_epoch"] = {"reference": [ref[s]["best_epoch"] for s in seeds], "ours": [our[s]["best_epoch"] for s in seeds]}
    doc["stop_epoch"] = {"reference": [ref[s]["stop_epoch"] for s in seeds], "ours": [our[s]["stop_epoch"] for s in seeds]}
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: doc[k] for k in ("paired_runs", "test_accuracy_ai")}, indent=1)[:2000])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["reference", "ours", "pt_reference", "pt_ours", "compare"])
    ap.add_argument("--seeds", default="0")
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--out", default=None)
    ap.add_argument("--pt", action="store_true")
    ap.add_argument("--seed-range", default=None, help="compare: only seeds lo-hi (inclusive)")
    a = ap.parse_args()
    if a.cmd == "compare":
        compare(a.out, a.pt, tuple(int(x) for x in a.seed_range.split("-")) if a.seed_range else None)
        return
    for s in (int(x) for x in a.seeds.split(",")):
        if a.cmd == "reference":
            reference(s, a.device)
        elif a.cmd == "pt_reference":
            pt_reference(s, a.device)
        elif a.cmd == "ours":
            ours(s)
        else:
            pt_ours(s)


if __name__ == "__main__":
    main()
