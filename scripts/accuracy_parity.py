"""Accuracy after equal epochs, reference vs the HIP path, on a REAL-data AVMNIST subset
(BASELINE.json north star: "final accuracy within ±0.2 pp of the reference after equal epochs").

The reference's split CSVs are absent (``$EXP_PATH/DATA`` is gitignored), so this
script defines its own pairing of the reference's sample files (MML_Suite/AVMNIST/dataset): for each
digit d, the k-th spectrogram of d (``{d}_{speaker}_{rep}.pt`` sorted by speaker, repetition) is paired
with the k-th MNIST image labelled d (``{idx}_{idx}_{d}.pt`` sorted by idx).  Train = the first
TRAIN_PER_DIGIT pairs of every digit, test = the next TEST_PER_DIGIT.  Files are read with the
weights-only unpickler only (data.load_sample_file).

Both sides train the late-fusion model (ResNet18 audio + ResNet34 image + MLP head, dropout 0.5) from
the seed-0 weights, batch 128 over the same sample order (torch.randperm, generator seeded per epoch),
Adam lr 5e-4 / wd 1e-4, E epochs, and measure test accuracy (eval mode, pattern "ai",
argmax of the softmax) after every epoch:

  reference — oracle/avmnist_ref.py on the CPU, i.e. the reference's AVMNIST.train_step (bit-exact to it
              on CPU, tests/test_oracle_golden.py); its dropout masks come from torch.bernoulli
  ours      — tspm_amd.FusedTrainStep / FusedEvalStep on the MI355X; dropout masks from the device RNG

Dropout masks (and fp32 summation order) differ between the sides, so the trajectories are two
independent training runs of the same recipe on the same data; the comparison is of their accuracy.

  python scripts/accuracy_parity.py prepare                  # here: reference files -> data_cache/
  python scripts/accuracy_parity.py reference --epochs 6     # here, CPU
  python scripts/accuracy_parity.py ours --epochs 6          # GPU box
  python scripts/accuracy_parity.py compare                  # -> profiles/r1_v7_accuracy_parity.json
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
DATASET = "/root/reference/MML_Suite/AVMNIST/dataset"
CACHE = os.path.join(REPO, "data_cache", "avmnist_real_subset")
OUT = os.path.join(REPO, "gpurun_out")
TRAIN_PER_DIGIT, TEST_PER_DIGIT = 400, 100
BATCH = 128


def prepare() -> None:
    from tspm_amd.data import AVMNISTCorpus, _np_safe_globals, load_sample_file
    specs = {d: [] for d in range(10)}
    for p in glob.glob(os.path.join(DATASET, "spectrograms", "*.pt")):
        d, spk, rep = (int(v) for v in os.path.basename(p)[:-3].split("_"))
        specs[d].append((spk, rep, p))
    imgs = {d: [] for d in range(10)}
    for p in glob.glob(os.path.join(DATASET, "images", "*.pt")):
        idx, _, d = (int(v) for v in os.path.basename(p)[:-3].split("_"))
        imgs[d].append((idx, p))
    need = TRAIN_PER_DIGIT + TEST_PER_DIGIT
    split = {"train": [], "test": []}
    for d in range(10):
        a = [p for _, _, p in sorted(specs[d])][:need]
        i = [p for _, p in sorted(imgs[d])][:need]
        for k in range(need):
            split["train" if k < TRAIN_PER_DIGIT else "test"].append((a[k], i[k], d))
    with torch.serialization.safe_globals(_np_safe_globals()):
        for name, rows in split.items():
            audio = np.stack([np.asarray(load_sample_file(a), np.float32) for a, _, _ in rows])
            image = np.stack([np.asarray(load_sample_file(i)).astype(np.uint8) for _, i, _ in rows])
            labels = np.array([d for _, _, d in rows], np.int64)
            AVMNISTCorpus(audio, image, labels).save(os.path.join(CACHE, name))
            print(name, audio.shape, image.shape, np.bincount(labels), flush=True)


def _load():
    from tspm_amd.data import AVMNISTCorpus
    return AVMNISTCorpus.load(os.path.join(CACHE, "train")), AVMNISTCorpus.load(os.path.join(CACHE, "test"))


def _lut() -> np.ndarray:
    from tspm_amd.data import default_lut
    return default_lut()


def _order(n: int, epoch: int) -> torch.Tensor:
    return torch.randperm(n, generator=torch.Generator().manual_seed(1000 + epoch))


def reference(epochs: int, seed: int) -> None:
    from oracle import avmnist_eval_ref as eref
    from oracle import avmnist_ref as orc
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    tr, te = _load()
    lut = torch.from_numpy(_lut().astype(np.int64))

    def tensors(c, rows):
        a = torch.from_numpy(np.asarray(c.audio[rows]))
        i = (lut[torch.from_numpy(np.asarray(c.image[rows])).long()].float() * (1.0 / 255.0)).unsqueeze(1)
        return a, i, torch.from_numpy(np.asarray(c.labels[rows]))
    model = orc.build_oracle_avmnist(0)
    opt = orc.OracleAdam(list(model.parameters()), lr=5e-4, weight_decay=1e-4)
    torch.manual_seed(seed)  # the dropout masks' RNG (weights stay the seed-0 ones)
    curve = []
    for ep in range(epochs):
        t0 = time.time()
        order = _order(len(tr), ep).numpy()
        losses = []
        model.train()
        for b in range(0, len(order), BATCH):
            a, i, lab = tensors(tr, order[b:b + BATCH])
            losses.append(orc.train_step(model, opt, a, i, lab)["loss"].item())
        model.eval()
        correct = 0
        for b in range(0, len(te), BATCH):
            rows = np.arange(b, min(len(te), b + BATCH))
            a, i, lab = tensors(te, rows)
            correct += int((eref.validation_step(model, a, i, lab)["preds"] == lab).sum())
        curve.append({"epoch": ep + 1, "train_loss": float(np.mean(losses)), "test_accuracy": correct / len(te),
                      "seconds": round(time.time() - t0, 1)})
        print(json.dumps(curve[-1]), flush=True)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"accuracy_reference_s{seed}.json"), "w") as f:
        json.dump({"side": "reference (oracle on CPU)", "dropout_seed": seed, "curve": curve}, f, indent=1)


def ours(epochs: int, seed: int) -> None:
    import tspm_amd
    from tspm_amd.data import DeviceCorpus
    from tspm_amd.step import FusedEvalStep
    dev = torch.device("cuda", 0)
    tr, te = _load()
    dtr, dte = DeviceCorpus(tr, dev), DeviceCorpus(te, dev)
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    model._rng_seed = 7919 * (seed + 1)  # the device dropout RNG's key (weights stay the seed-0 ones)
    steps, evals = {}, {}
    curve = []
    for ep in range(epochs):
        t0 = time.time()
        order = _order(len(tr), ep).to(dev)
        losses = []
        for b in range(0, len(tr), BATCH):
            idx = order[b:b + BATCH].contiguous()
            n = idx.numel()
            st = steps.get(n) or steps.setdefault(n, tspm_amd.FusedTrainStep(model, opt, None, n))
            dtr.gather(idx, out=(st.A, st.I, st.labels))
            st.run()
            losses.append(st.loss.clone())
        correct = torch.zeros((), dtype=torch.int64, device=dev)
        for b in range(0, len(te), BATCH):
            idx = torch.arange(b, min(len(te), b + BATCH), device=dev)
            n = idx.numel()
            ev = evals.get(n) or evals.setdefault(n, FusedEvalStep(model, None, n))
            dte.gather(idx, out=(ev.A, ev.I, ev.labels))
            ev.run()
            correct += (ev.preds == ev.labels).sum()
        torch.cuda.synchronize()
        curve.append({"epoch": ep + 1, "train_loss": float(np.mean([x.item() for x in losses])),
                      "test_accuracy": int(correct) / len(te), "seconds": round(time.time() - t0, 2)})
        print(json.dumps(curve[-1]), flush=True)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"accuracy_ours_s{seed}.json"), "w") as f:
        json.dump({"side": "ours (HIP path, MI355X)", "dropout_seed": seed, "curve": curve}, f, indent=1)


def compare(out_path: str) -> None:
    def runs(side):
        out = {}
        for p in sorted(glob.glob(os.path.join(OUT, f"accuracy_{side}_s*.json"))):
            d = json.load(open(p))
            out[d["dropout_seed"]] = d["curve"]
        return out
    ref, our = runs("reference"), runs("ours")
    n = min(min(len(c) for c in ref.values()), min(len(c) for c in our.values()))
    rows = []
    for k in range(n):
        ra = [c[k]["test_accuracy"] for c in ref.values()]
        oa = [c[k]["test_accuracy"] for c in our.values()]
        rows.append({"epoch": k + 1, "reference_test_accuracy": ra, "ours_test_accuracy": oa,
                     "reference_mean": round(float(np.mean(ra)), 5), "ours_mean": round(float(np.mean(oa)), 5),
                     "delta_mean_pp": round(100 * (float(np.mean(oa)) - float(np.mean(ra))), 2),
                     "reference_train_loss": [round(c[k]["train_loss"], 5) for c in ref.values()],
                     "ours_train_loss": [round(c[k]["train_loss"], 5) for c in our.values()]})
    last = rows[-1]
    doc = {"what": "late-fusion AVMNIST, real-data subset of the reference's sample files "
                   f"({TRAIN_PER_DIGIT * 10} train / {TEST_PER_DIGIT * 10} test pairs, own pairing: the "
                   "reference's split CSVs are absent), seed-0 weights, same batch order, batch 128, Adam "
                   "5e-4 / 1e-4, dropout 0.5; one run per dropout seed and side (masks drawn independently)",
           "reference_seeds": sorted(ref), "ours_seeds": sorted(our),
           "test_samples": TEST_PER_DIGIT * 10, "one_sample_pp": round(100 / (TEST_PER_DIGIT * 10), 3),
           "final": {"epoch": last["epoch"], "reference_mean": last["reference_mean"], "ours_mean": last["ours_mean"],
                     "delta_mean_pp": last["delta_mean_pp"],
                     "reference_seed_spread_pp": round(100 * (max(last["reference_test_accuracy"]) -
                                                              min(last["reference_test_accuracy"])), 2),
                     "ours_seed_spread_pp": round(100 * (max(last["ours_test_accuracy"]) -
                                                         min(last["ours_test_accuracy"])), 2)},
           "epochs": rows}
    # less noisy summary: per run, the mean test accuracy of the last 3 epochs; then mean and standard
    # error over the runs of each side
    def tail3(curves):
        v = np.array([np.mean([c[k]["test_accuracy"] for k in range(n - 3, n)]) for c in curves.values()])
        return float(v.mean()), float(v.std(ddof=1) / np.sqrt(len(v))) if len(v) > 1 else float("nan")
    (rm, rse), (om, ose) = tail3(ref), tail3(our)
    doc["last3_epochs"] = {"reference_mean": round(rm, 5), "reference_stderr": round(rse, 5), "ours_mean": round(om, 5),
                           "ours_stderr": round(ose, 5), "delta_pp": round(100 * (om - rm), 2),
                           "delta_stderr_pp": round(100 * float(np.hypot(rse, ose)), 2)}
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc["final"], indent=1))
    print(json.dumps(doc["last3_epochs"], indent=1))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("what", choices=["prepare", "reference", "ours", "compare"])
    ap.add_argument("--epochs", type=int, default=6)
    ap.add_argument("--seeds", default="0", help="comma-separated dropout seeds (one run each)")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r1_v7_accuracy_parity.json"))
    a = ap.parse_args()
    if a.what == "prepare":
        prepare()
    elif a.what == "reference":
        for sd in a.seeds.split(","):
            reference(a.epochs, int(sd))
    elif a.what == "ours":
        for sd in a.seeds.split(","):
            ours(a.epochs, int(sd))
    else:
        compare(a.out)


if __name__ == "__main__":
    main()
