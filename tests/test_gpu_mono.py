"""Monomodal pre-training step (train_monomodal.MonomodalEncoder; BASELINE.json configs[1]) on the HIP
path against the CPU oracle (oracle/monomodal_ref.py, pinned bit-exact to the real reference by
tests/golden/make_mono_golden.py).  Criterion as tests/test_gpu_model.py (tests/parity.py): fp64
oracle with our ReLU / max-pool decisions forced (flips proven near-ties), logits rel-L2 <= 1e-4,
gradients rel-L2 <= 1e-3 and cosine >= 0.9999 and within 4x the fp32 reference's error, no relaxed
branch; every step checked from our own state; Adam exact."""
import numpy as np
import pytest
import torch

import tspm_amd
from oracle import avmnist_ref as orc
from oracle import monomodal_ref as mref
from parity import (GRAD_REL, Tally, check_adam, check_grad, check_out, engine_decisions, flip_report, flips_summary,
                    pair_from, rel_l2, snapshot)
from tspm_amd.monomodal import FusedMonoEvalStep, FusedMonoStep

pytestmark = pytest.mark.gpu
NAMES = {"audio": "AVMNIST_Audio_Encoder_Resnet_Pretrain", "image": "AVMNIST_Image_Encoder_Resnet_Pretrain"}


def _ours(which, dev, seed):
    torch.manual_seed(seed)
    enc = tspm_amd.ResNet18(1, 64) if which == "audio" else tspm_amd.ResNet34(1, 128)
    return tspm_amd.MonomodalEncoder(enc, 64 if which == "audio" else 128, 10).to(dev)


def _batch(which, n, seed):
    audio, image, labels, _ = orc.synthetic_batch(n, seed=seed)
    return (audio if which == "audio" else image), labels


def _clear(logits64):
    top2 = logits64.topk(2, dim=1).values
    return (top2[:, 0] - top2[:, 1]) > 1e-3 * top2[:, 0].abs().clamp_min(1)


def _check_mono_step(ours, st, which, seed, x, labels, out, tally, ref32_logits=None, ref32_loss=None):
    """One step of ours (just run, starting from the state the oracle pair was anchored to) against the
    forced fp32 / fp64 oracle steps."""
    o32, o64 = st._pair
    forced = engine_decisions(st.eng, "enc.")
    t32, t64 = orc.MaskTrace(forced), orc.MaskTrace(forced)
    r32 = mref.train_step(o32, None, x, labels, t32)
    r64 = mref.train_step(o64, None, x.double(), labels, t64)
    rep = flip_report(t64, forced)
    check_out("logits", out["logits"], r32["logits"] if ref32_logits is None else ref32_logits, r64["logits"], tally)
    check_out("loss", out["loss"], (r32["loss"] if ref32_loss is None else ref32_loss).reshape(1),
              r64["loss"].reshape(1), tally)
    p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
    for n, p in ours.named_parameters():
        check_grad(f"grad {n}", p.grad, p32[n].grad, p64[n].grad, tally)
    s32, s64 = o32.state_dict(), o64.state_dict()
    for k, v in ours.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            check_out(k, v, s32[k], s64[k], tally, bound=GRAD_REL)
    clear = _clear(r64["logits"])
    assert torch.equal(out["preds"].cpu()[clear], r64["preds"][clear])
    return rep


@pytest.mark.parametrize("which,batch", [("audio", 32), ("audio", 256), ("image", 64)])
def test_fused_mono_step_vs_oracle(gpu, which, batch):
    ours = _ours(which, gpu, 3)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    x, labels = _batch(which, batch, 1234)
    st = FusedMonoStep(ours, opt, None, tuple(x.shape))
    tally = Tally()
    for s in range(3):  # eager, capture, replay
        st._pair = pair_from(ours, lambda: mref.build_oracle_monomodal(which, 3))
        before = snapshot(ours, opt if s else None)
        out = st.step(x.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        rep = _check_mono_step(ours, st, which, 3, x, labels, out, tally)
        check_adam(ours, opt, *before, s + 1)
        print(f"[{which} B={batch} step {s + 1}] {flips_summary(rep)}")
    assert int(ours.state_dict()["encoder.bn1.num_batches_tracked"]) == 3
    print(tally)


def test_fused_mono_step_vs_reference_golden(gpu):
    """3 fused steps from the seed-0 weights on the B=4 batch of the vectors captured from the REAL
    train_monomodal.MonomodalEncoder.train_step (audio and image models): step 1 against the golden
    fp32 reference and the forced fp64 oracle, steps 2-3 against the oracle from our own state."""
    g = dict(np.load(__import__("os").path.join(__import__("os").path.dirname(__file__), "golden",
                                                 "avmnist_mono_b4.npz"), allow_pickle=False))
    labels = torch.from_numpy(g["labels"])
    tally = Tally()
    for which in ("audio", "image"):
        ours = _ours(which, gpu, 0)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        x = torch.from_numpy(g[f"{which}_x"])
        st = FusedMonoStep(ours, opt, None, tuple(x.shape))
        for s in range(3):
            st._pair = pair_from(ours, lambda: mref.build_oracle_monomodal(which, 0))
            before = snapshot(ours, opt if s else None)
            out = st.step(x.to(gpu), labels.to(gpu))
            torch.cuda.synchronize()
            if s == 0:
                ref_logits, ref_loss = torch.from_numpy(g[f"{which}_logits"][0]), torch.tensor([g[f"{which}_losses"][0]])
                _check_mono_step(ours, st, which, 0, x, labels, out, tally, ref_logits, ref_loss)
                gn = np.array([p.grad.double().norm().item() for p in ours.parameters()])
                gn64 = np.array([p.grad.norm().item() for p in st._pair[1].parameters()])
                check_out(f"{which} grad norms", gn, g[f"{which}_grad_norm_step1"], gn64, tally, bound=GRAD_REL)
            else:
                _check_mono_step(ours, st, which, 0, x, labels, out, tally)
            check_adam(ours, opt, *before, s + 1)
    print(tally)


def test_mono_graph_replay_equals_eager(gpu):
    res = []
    for use_graph in (False, True):
        ours = _ours("audio", gpu, 7)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        x, labels = _batch("audio", 64, 5)
        st = FusedMonoStep(ours, opt, None, tuple(x.shape), use_graph=use_graph)
        for _ in range(4):
            st.step(x.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()]).cpu())
    assert torch.equal(res[0], res[1])


def test_mono_eval_step_vs_oracle(gpu):
    ours = _ours("audio", gpu, 4)
    ref = mref.build_oracle_monomodal("audio", 4)
    for m in list(ours.modules()) + list(ref.modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            gg = torch.Generator().manual_seed(m.num_features)
            m.running_mean.copy_(torch.randn(m.num_features, generator=gg) * 0.1)
            m.running_var.copy_(torch.rand(m.num_features, generator=gg) + 0.5)
    x, labels = _batch("audio", 96, 31)
    st = FusedMonoEvalStep(ours, None, tuple(x.shape))
    outs = [st.step(x.to(gpu), labels.to(gpu))["loss"].item() for _ in range(3)]  # eager, capture, replay
    r = mref.validation_step(ref, x, labels)
    assert outs[0] == outs[1] == outs[2]
    assert rel_l2(st.logits, r["logits"]) < 1e-4
    assert abs(outs[0] - r["loss"].item()) <= 1e-4 * abs(r["loss"].item())
    clear = _clear(r["logits"].double())
    assert torch.equal(st.preds.cpu()[clear], r["preds"][clear])


def test_train_and_validation_step_api(gpu):
    """The reference's call signatures and return dicts, fused (FusedAdam) and autograd (torch Adam)
    paths, with the reference's own metric-recorder surface (config.groups / update_group)."""
    from types import SimpleNamespace

    class Rec:
        def __init__(self):
            self.config = SimpleNamespace(groups={"classification": ["accuracy"]})
            self.calls = []

        def update_group(self, group_name, predictions, targets, modality):
            self.calls.append((group_name, modality, predictions.detach().cpu().numpy().copy()))

    x, labels = _batch("audio", 16, 77)
    cfg = SimpleNamespace(experiment=SimpleNamespace(name=NAMES["audio"]))
    batch = {"audio": x, "image": torch.zeros(16, 1, 28, 28), "labels": labels, "pattern_name": ["a"] * 16}
    results = {}
    for kind in ("fused", "autograd"):
        ours = _ours("audio", gpu, 11)
        opt = (tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4) if kind == "fused"
               else torch.optim.Adam(ours.parameters(), lr=5e-4, weight_decay=1e-4))
        loss_fns = None if kind == "fused" else (lambda lg, lb: {"total_loss": torch.nn.functional.cross_entropy(lg, lb)})
        rec = Rec()
        ours.train()
        r = ours.train_step(batch, opt, loss_fns, gpu, rec, cfg)
        assert set(r) == {"loss", "metrics"} and set(r["metrics"]) == {"loss", "accuracy"}
        assert rec.calls[0][:2] == ("classification", "audio")
        assert (kind == "fused") == (ours._fused is not None)
        ours.eval()
        v = ours.validation_step(batch, loss_fns, gpu, rec, cfg)
        assert set(v) == {"loss", "metrics"}
        results[kind] = (r, v, torch.cat([p.detach().reshape(-1) for p in ours.parameters()]).cpu())
    o32 = mref.build_oracle_monomodal("audio", 11)
    r32 = mref.train_step(o32, orc.OracleAdam(list(o32.parameters()), lr=5e-4, weight_decay=1e-4), x, labels)
    for kind, (r, v, _) in results.items():
        assert abs(r["loss"] - r32["loss"].item()) <= 1e-4 * abs(r32["loss"].item()), kind
    # both paths run the same HIP kernels: same loss, parameters within Adam's sign-amplified rounding
    assert abs(results["fused"][0]["loss"] - results["autograd"][0]["loss"]) <= 1e-6
    assert rel_l2(results["fused"][2], results["autograd"][2]) < 1e-4


def test_fit_monomodal_hands_encoder_to_late_fusion(gpu, tmp_path):
    from tspm_amd.data import AVMNIST, synthetic_corpus
    from tspm_amd.monomodal import fit_monomodal
    ours = _ours("audio", gpu, 0)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    tr = AVMNIST(None, "train", "audio", selected_patterns=["a"], corpus=synthetic_corpus(96, 5), device=gpu)
    va = AVMNIST(None, "valid", "audio", selected_patterns=["a"], corpus=synthetic_corpus(40, 6), device=gpu)
    loaders = {"train": tr.device_loader(32, shuffle=True), "validation": va.device_loader(32),
               "test": va.device_loader(32)}
    sched = lambda o: torch.optim.lr_scheduler.ReduceLROnPlateau(o, mode="min", factor=0.5, patience=5)  # noqa: E731
    h = fit_monomodal(ours, opt, None, loaders, 2, experiment_name=NAMES["audio"], model_output_path=tmp_path,
                      scheduler_factory=sched)
    tr0 = h["metrics_history"]["train"][0]
    assert {"loss", "accuracy", "accuracy_AUDIO", "f1_macro_AUDIO"} <= set(tr0)
    assert "accuracy_AUDIO" in h["metrics_history"]["test"]
    assert h["encoder_path"] and (tmp_path / "encoder_audio_best.pth").exists() and (tmp_path / "best.pth").exists()
    enc_sd = torch.load(tmp_path / "encoder_audio_best.pth", weights_only=True)
    # the pretrained late-fusion config loads it into AVMNIST.audio_encoder (train_multimodal.py:186-187)
    torch.manual_seed(1)
    fusion = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5)
    fusion.audio_encoder.load_state_dict(enc_sd)
    assert list(enc_sd) == list(fusion.audio_encoder.state_dict())
