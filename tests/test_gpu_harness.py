"""Evaluation + epoch harness on the GPU: tspm_classify_update against the numpy/torch oracle, the
FusedEvalStep against the oracle's eval forward, in-graph train metrics, EpochRunner epochs against a
plain per-batch loop (losses bit-exact, metrics equal to raw-array sklearn), and fit() files."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import avmnist_eval_ref as eref
from oracle import avmnist_ref as orc

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm()).item()


def test_classify_update_vs_oracle(gpu):
    from tspm_amd.metrics import ClassificationLog
    g = torch.Generator().manual_seed(0)
    log = ClassificationLog(gpu, groups=("a", "ai", "i"), capacity=8)
    ref_conf = np.zeros((3, 10, 10), np.int64)
    losses = []
    for n in (128, 37, 1):
        logits = torch.randn(n, 10, generator=g) * 3
        logits[0, 3] = logits[0, 7] = logits[0].max() + 1  # exact tie: first index wins
        labels = torch.randint(0, 10, (n,), generator=g)
        labels[-1] = 11 if n > 1 else labels[-1]           # out-of-range label: not counted
        groups = torch.randint(0, 3, (n,), generator=g, dtype=torch.int32)
        loss = torch.rand(1, generator=g)
        losses.append(float(loss))
        pred = torch.empty(n, dtype=torch.int64, device=gpu)
        log.update(logits.to(gpu), labels.to(gpu), groups.to(gpu), loss.to(gpu), pred_out=pred)
        want = eref.predictions(logits)
        assert torch.equal(pred.cpu(), want) and int(want[0]) == 3
        ref_conf += eref.confusion(labels.numpy(), want.numpy(), groups.numpy(), 3)
    conf, ll, samples = log.fetch()
    assert np.array_equal(conf, ref_conf)
    assert ll.tolist() == [np.float32(x) for x in losses] and samples == 166
    log.reset()
    assert log.fetch()[0].sum() == 0 and len(log.fetch()[1]) == 0


def _models(dev, dropout=0.5):
    import tspm_amd
    torch.manual_seed(0)
    m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=dropout).to(dev)
    return m, orc.build_oracle_avmnist(0)


@pytest.mark.parametrize("batch", [64, 37])
def test_fused_eval_step_vs_oracle(gpu, batch):
    from tspm_amd.metrics import ClassificationLog
    from tspm_amd.step import FusedEvalStep
    model, ref = _models(gpu)
    # non-trivial running statistics
    for m in list(model.modules()) + list(ref.modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            gg = torch.Generator().manual_seed(m.num_features)
            rm, rv = torch.randn(m.num_features, generator=gg) * 0.1, torch.rand(m.num_features, generator=gg) + 0.5
            m.running_mean.copy_(rm)
            m.running_var.copy_(rv)
    audio, image, labels, _ = orc.synthetic_batch(batch, seed=99)
    log = ClassificationLog(gpu)
    st = FusedEvalStep(model, None, batch, log)
    groups = torch.full((batch,), 1, dtype=torch.int32)
    for _ in range(3):  # eager, capture, replay
        out = st.step(audio.to(gpu), image.to(gpu), labels.to(gpu), groups.to(gpu))
    r = eref.validation_step(ref, audio, image, labels)
    assert rel(out["logits"], r["logits"]) < 1e-4
    assert abs(out["loss"].item() - r["loss"].item()) <= 1e-4 * abs(r["loss"].item())
    top2 = r["logits"].topk(2, dim=1).values
    clear = (top2[:, 0] - top2[:, 1]) > 1e-3 * top2[:, 0].abs().clamp_min(1)
    assert torch.equal(out["preds"].cpu()[clear], r["preds"][clear])
    conf, ll, n = log.fetch()
    assert n == 3 * batch and len(ll) == 3 and conf.sum() == 3 * batch and conf[1].sum() == 3 * batch
    assert ll[0] == ll[1] == ll[2]  # eager / captured / replayed evaluations agree bit-exactly


def test_train_step_log_matches_step_logits(gpu):
    from tspm_amd.metrics import ClassificationLog
    import tspm_amd
    model, _ = _models(gpu)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    st = tspm_amd.FusedTrainStep(model, opt, None, 32)
    log = ClassificationLog(gpu)
    st.log = log
    want = np.zeros((3, 10, 10), np.int64)
    losses = []
    for s in range(4):
        audio, image, labels, _ = orc.synthetic_batch(32, seed=10 + s)
        groups = torch.tensor([s % 3] * 32, dtype=torch.int32)
        out = st.step(audio.to(gpu), image.to(gpu), labels.to(gpu), groups.to(gpu))
        preds = eref.predictions(out["logits"].cpu())
        want += eref.confusion(labels.numpy(), preds.numpy(), groups.numpy(), 3)
        losses.append(out["loss"].item())
    conf, ll, n = log.fetch()
    assert np.array_equal(conf, want) and ll.tolist() == losses and n == 128


def _loaders(gpu, n_train=96, n_val=40, bs=32):
    from tspm_amd.data import AVMNIST, synthetic_corpus
    tr = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=synthetic_corpus(n_train, 5),
                 device=gpu)
    va = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"],
                 corpus=synthetic_corpus(n_val, 6), device=gpu)
    return tr, va


def test_epoch_runner_equals_plain_loop(gpu):
    import sklearn.metrics as skm
    import tspm_amd
    from tspm_amd.harness import AVMNIST_METRICS, EpochRunner
    tr, va = _loaders(gpu)
    # run A: the harness
    mA, _ = _models(gpu)
    oA = tspm_amd.FusedAdam(mA.parameters(), lr=5e-4, weight_decay=1e-4)
    runner = EpochRunner(mA, oA, None)
    lossA, _, trm, nb = runner.train_epoch(tr.device_loader(32, shuffle=True, generator=torch.Generator().manual_seed(1)))
    vlossA, _, vam, vnb = runner.validate_epoch(va.device_loader(32))
    # run B: plain per-batch calls (the reference's loop shape) on an identical model
    mB, _ = _models(gpu)
    oB = tspm_amd.FusedAdam(mB.parameters(), lr=5e-4, weight_decay=1e-4)
    stB = tspm_amd.FusedTrainStep(mB, oB, None, 32)
    lossesB, tp, tt = [], [], []
    for b in tr.device_loader(32, shuffle=True, generator=torch.Generator().manual_seed(1)):
        out = stB.step(b["audio"], b["image"], b["labels"])
        lossesB.append(out["loss"].item())
        tp.append(eref.predictions(out["logits"].cpu()).numpy())
        tt.append(b["labels"].cpu().numpy())
    assert nb == 3 and lossA == float(np.mean(lossesB))
    for p, q in zip(mA.parameters(), mB.parameters()):
        assert torch.equal(p, q)
    vl, preds, targs, pats = [], [], [], []
    for b in va.device_loader(32):
        r = mB.validation_step(b, None, gpu, None, return_test_info=True)
        vl.append(r["loss"])
        preds.append(r["predictions"]), targs.append(r["labels"]), pats.extend(b["pattern_name"])
    assert vnb == 4 and vlossA == float(np.mean(vl))
    preds, targs, pats = np.concatenate(preds), np.concatenate(targs), np.array(pats)
    for p in ("a", "ai", "i"):
        sel = pats == p
        for name, spec in AVMNIST_METRICS["metrics"].items():
            fn = getattr(skm, spec["function"].rsplit(".", 1)[1])
            want = fn(targs[sel], preds[sel], **spec["kwargs"])
            got = vam[f"{name}_{p.upper()}"]
            assert np.array_equal(np.asarray(got), np.asarray(want)), (name, p)
    tt, tp = np.concatenate(tt), np.concatenate(tp)
    assert trm["accuracy_AI"] == skm.accuracy_score(tt, tp)
    assert trm["f1_macro_AI"] == skm.f1_score(tt, tp, average="macro", zero_division=0)


def test_fit_writes_reference_files(gpu, tmp_path):
    import tspm_amd
    from tspm_amd.harness import fit
    tr, va = _loaders(gpu)
    model, _ = _models(gpu)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    sched = torch.optim.lr_scheduler.ReduceLROnPlateau(opt, mode="min", factor=0.5, patience=5, min_lr=1e-5)
    loaders = {"train": tr.device_loader(32, shuffle=True), "validation": va.device_loader(32),
               "test": va.device_loader(32)}
    h = fit(model, opt, None, loaders, epochs=2, scheduler=sched, checkpoint_dir=tmp_path / "models",
            metrics_path=tmp_path / "metrics")
    assert len(h["train"]) == 2 and "test" in h and "accuracy_AI" in h["test"]
    em = json.load(open(tmp_path / "metrics" / "epoch_metrics.json"))
    assert [e["epoch"] for e in em] == [1, 2]
    assert set(em[0]["validation"]) >= {"loss", "timing", "AI", "A", "I", "metrics"}
    assert "f1_macro" in em[0]["validation"]["AI"] and "accuracy_AI" in em[0]["validation"]["metrics"]
    ck = torch.load(tmp_path / "models" / "best.pth", weights_only=True)
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "scheduler_state_dict"}
    assert len(ck["model_state_dict"]) == 346
    assert os.path.exists(tmp_path / "models" / "epoch_1.pth")
    fresh, _ = _models(gpu)
    fresh.load_state_dict(ck["model_state_dict"])


def test_fit_fails_fast_on_nonfinite_loss(gpu):
    """A NaN in one training sample makes that batch's loss NaN: fit stops at the end of the epoch
    with FloatingPointError instead of training on (checkpointing) NaN weights."""
    import tspm_amd
    from tspm_amd.data import AVMNIST, synthetic_corpus
    from tspm_amd.harness import fit
    c = synthetic_corpus(64, 5)
    c.audio[3, 0, 0] = float("nan")
    tr = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=c, device=gpu)
    _, va = _loaders(gpu)
    model, _ = _models(gpu)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    loaders = {"train": tr.device_loader(32, shuffle=False), "validation": va.device_loader(32)}
    with pytest.raises(FloatingPointError):
        fit(model, opt, None, loaders, epochs=2)
