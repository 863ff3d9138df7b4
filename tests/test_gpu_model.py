"""End-to-end parity of the HIP encoders / fused train step against the reference.

Ground truth: the CPU oracle in fp64 with the HIP step's own ReLU masks and max-pool argmax forced
into it (tests/parity.py; flips proven to be near-ties and counted).  Bounds, with no relaxed
branch: logits / loss / embeddings rel-L2 <= 1e-4, every gradient rel-L2 <= 1e-3 and cosine >= 0.9999,
and each also within 4x the error of the fp32 reference on the same decisions.  The fp32 reference is
the golden vectors captured from the real MML_Suite code (B=4) or the oracle in fp32 (bit-identical
to the reference on CPU, pinned by tests/test_oracle_golden.py).

Multi-step: every step is checked from OUR state (parity.anchor — Adam's first updates are
~lr x sign(g), so two correct implementations' free-running trajectories separate); Adam itself is
checked exactly (fp64 Adam applied to our gradients and moments reproduces our update).
"""
import numpy as np
import pytest
import torch

import tspm_amd
from oracle import avmnist_ref as orc
from parity import (GRAD_REL, Tally, anchor, check_adam, check_grad, check_out, engine_decisions, flip_report,
                    flips_summary, head_decisions, pair_from, rel_l2, snapshot, step_decisions)

pytestmark = pytest.mark.gpu


def _build(seed, dropout=0.5):
    return lambda: orc.build_oracle_avmnist(seed, dropout=dropout)


def _forced(o32, o64, audio, image, labels, keep, forced):
    """One oracle step (no optimizer) in fp32 and fp64 with our decisions forced."""
    t32, t64 = orc.MaskTrace(forced), orc.MaskTrace(forced)
    r32 = orc.train_step(o32, None, audio, image, labels, keep, t32)
    r64 = orc.train_step(o64, None, audio.double(), image.double(), labels, keep, t64)
    return r32, r64, t64


def _compare_params(ours, o32, o64, tally):
    p32, p64 = dict(o32.named_parameters()), dict(o64.named_parameters())
    for n, p in ours.named_parameters():
        check_grad(f"grad {n}", p.grad, p32[n].grad, p64[n].grad, tally)
    s32, s64 = o32.state_dict(), o64.state_dict()
    for k, v in ours.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            check_out(k, v, s32[k], s64[k], tally, bound=GRAD_REL)


def _check_step(ours, st, o32, o64, audio, image, labels, keep, out, tally, ref32_logits=None, ref32_loss=None):
    forced = step_decisions(st)
    r32, r64, t64 = _forced(o32, o64, audio, image, labels, keep, forced)
    rep = flip_report(t64, forced, keep)
    check_out("logits", out["logits"], r32["logits"] if ref32_logits is None else ref32_logits, r64["logits"], tally)
    check_out("loss", out["loss"], (r32["loss"] if ref32_loss is None else ref32_loss).reshape(1),
              r64["loss"].reshape(1), tally)
    _compare_params(ours, o32, o64, tally)
    return rep


@pytest.mark.parametrize("batch", [4, 32, 128])
@pytest.mark.parametrize("which", ["audio", "image"])
def test_encoder_forward_backward(gpu, batch, which):
    audio, image, _, _ = orc.synthetic_batch(batch, seed=99)
    x = audio if which == "audio" else image
    ctor, octor, hid = ((tspm_amd.ResNet18, orc.oracle_resnet18, 64) if which == "audio"
                        else (tspm_amd.ResNet34, orc.oracle_resnet34, 128))
    torch.manual_seed(0)
    ours = ctor(1, hid).to(gpu).train()
    torch.manual_seed(0)
    r32 = octor(1, hid)
    import copy
    r64 = copy.deepcopy(r32).double()
    g = torch.randn(batch, hid, generator=torch.Generator().manual_seed(5))
    xg = x.to(gpu)
    emb = ours(xg)
    emb.backward(g.to(gpu))
    torch.cuda.synchronize()
    forced = engine_decisions(ours.engine_for(xg), "enc.")
    t32, t64 = orc.MaskTrace(forced), orc.MaskTrace(forced)
    e32 = orc.encoder_forward(r32, x, True, t32, "enc.")
    e32.backward(g)
    e64 = orc.encoder_forward(r64, x.double(), True, t64, "enc.")
    e64.backward(g.double())
    rep = flip_report(t64, forced)
    tally = Tally()
    check_out("embedding", emb, e32, e64, tally)
    _compare_params(ours, r32, r64, tally)
    for k, v in ours.state_dict().items():
        if k.endswith("num_batches_tracked"):
            assert int(v) == 1, k
    print(f"[{which} B={batch}] {flips_summary(rep)}; {tally}")


def test_fused_step_vs_golden_reference(gpu, golden):
    """3 fused HIP train steps (eager first call, captured graph afterwards) from the seed-0 weights
    on the B=4 batch of the vectors captured from the real MML_Suite AVMNIST.train_step (the
    reference's dropout masks).  Step 1 is held against the golden fp32 reference and the forced fp64
    oracle; steps 2-3 and the final eval forward against the fp64 oracle from our own state."""
    torch.manual_seed(0)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    audio, image = torch.from_numpy(golden["audio"]), torch.from_numpy(golden["image"])
    labels = torch.from_numpy(golden["labels"])
    masks = [torch.from_numpy(m) for m in golden["keep_masks"]]
    step = tspm_amd.FusedTrainStep(ours, opt, None, 4)
    names = list(golden["param_names"])
    params = dict(ours.named_parameters())
    tally = Tally()
    for s in range(3):
        o32, o64 = pair_from(ours, _build(0))
        before = snapshot(ours, opt if s else None)
        step.keep_override = masks[s].to(gpu)
        out = step.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        if s == 0:
            rep = _check_step(ours, step, o32, o64, audio, image, labels, masks[s], out, tally,
                              torch.from_numpy(golden["logits"][0]), torch.tensor([golden["losses"][0]]))
            gn = np.array([params[n].grad.double().norm().item() for n in names])
            gn64 = np.array([dict(o64.named_parameters())[n].grad.norm().item() for n in names])
            check_out("grad norms step 1", gn, golden["grad_norm_step1"], gn64, tally, bound=GRAD_REL)
        else:
            rep = _check_step(ours, step, o32, o64, audio, image, labels, masks[s], out, tally)
        check_adam(ours, opt, *before, s + 1)
        print(f"[golden step {s + 1}] {flips_summary(rep)}")
    o32, o64 = pair_from(ours, _build(0))
    ours.eval()
    with torch.no_grad():
        ev = ours(A=audio.to(gpu), I=image.to(gpu))
        o32.eval()
        o64.eval()
        ev32, _, _ = orc.avmnist_forward(o32, audio, image, False)
        ev64, _, _ = orc.avmnist_forward(o64, audio.double(), image.double(), False)
    check_out("eval logits after 3 steps", ev, ev32, ev64, tally)
    print(tally)


@pytest.mark.parametrize("batch", [32, 128, 1024])
def test_fused_step_vs_oracle(gpu, batch):
    """The benched fused step (two-stream graph, carried Adam, LDS floor at 64-128) against the forced-decision fp64
    oracle; batch 1024 = configs[2]'s other per-rank reading (the batch-1024 tuned table: variant-2 kernels, no
    floor) — flips counted and bounded as at 128 (parity.MAX_FLIP_FRAC)."""
    torch.manual_seed(3)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    audio, image, labels, _ = orc.synthetic_batch(batch, seed=1234)
    step = tspm_amd.FusedTrainStep(ours, opt, None, batch)
    tally = Tally()
    for s in range(3):  # eager, capture + replay, replay
        keep = (torch.rand(batch, 128, generator=torch.Generator().manual_seed(8 + s)) > 0.5).to(torch.uint8)
        o32, o64 = pair_from(ours, _build(3))
        before = snapshot(ours, opt if s else None)
        step.keep_override = keep.to(gpu)
        out = step.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        rep = _check_step(ours, step, o32, o64, audio, image, labels, keep, out, tally)
        check_adam(ours, opt, *before, s + 1)
        print(f"[B={batch} step {s + 1}] {flips_summary(rep)}")
    print(tally)


def test_graph_replay_equals_eager(gpu):
    """Deterministic kernels (no atomics): eager and graph-replayed steps are bitwise identical."""
    results = []
    for use_graph in (False, True):
        torch.manual_seed(7)
        ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        audio, image, labels, _ = orc.synthetic_batch(32, seed=5)
        st = tspm_amd.FusedTrainStep(ours, opt, None, 32, use_graph=use_graph)
        for _ in range(4):
            st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()]).cpu())
    assert torch.equal(results[0], results[1])


def test_adam_split_schedule_equals_plain_step(gpu):
    """The single-GPU Adam schedule (the default) that updates each encoder's parameter ranges on that
    encoder's stream as soon as its backward ends gives bitwise the parameters, Adam moments and BN
    buffers of the one-launch update, eager and replayed, and every flat-buffer element belongs to
    exactly one range."""
    results = []
    for mode in (False, True):
        torch.manual_seed(13)
        ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        st = tspm_amd.FusedTrainStep(ours, opt, None, 32, adam_split=mode)
        if mode:
            rs = st._adam_ranges()
            for gi, fg in enumerate(opt.flat_groups()):
                cover = torch.zeros(fg.numel, dtype=torch.int32)
                for part in rs:
                    for a, b in part[gi]:
                        cover[a:b] += 1
                assert bool((cover == 1).all()), mode
        for i in range(4):
            audio, image, labels, _ = orc.synthetic_batch(32, seed=70 + i)
            st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        assert st.graph is not None
        bufs = [m.running_var.detach().reshape(-1) for m in ours.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        mom = [t for fg in opt.flat_groups() for t in (fg.exp_avg, fg.exp_avg_sq)]
        results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()] + bufs + mom).cpu())
    assert torch.equal(results[0], results[1])


def test_phased_allreduce_step_equals_plain_step(gpu):
    """The DP step path — forward + backward as one graph whose step flags release the phase-1
    gradients to the RCCL all-reduce (and that phase's Adam ranges) while phase 2 runs | RCCL of the rest |
    the rest's Adam ranges — under a 1-rank RCCL group
    (all-reduce = identity) gives bitwise the parameters of the plain fused step, eager and
    graph-replayed, and covers every parameter exactly once."""
    import os
    import socket
    import torch.distributed as dist
    s_ = socket.socket()
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
    s_.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    created = False
    if not dist.is_initialized():
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=gpu)
        created = True
    try:
        results = []
        for phased in (False, True):
            torch.manual_seed(9)
            ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
            opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
            st = tspm_amd.FusedTrainStep(ours, opt, None, 32, use_graph=True)
            if phased:
                st.allreduce = st.phased_allreduce(force=True)
                covered = sum(v.numel() for ph in st.allreduce.phases for v in ph)
                assert covered == sum(fg.numel for fg in opt.flat_groups())
                assert len(st.allreduce.phases[0]) >= 1 and len(st.allreduce.phases[1]) >= 1
            for i in range(4):
                audio, image, labels, _ = orc.synthetic_batch(32, seed=50 + i)
                st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
            torch.cuda.synchronize()
            if phased:  # one fwd+bwd graph; Adam per phase behind its exchange (no Adam graph)
                assert isinstance(st.graph, torch.cuda.CUDAGraph) and st.graph_opt is None
            bufs = [m.running_var.detach().reshape(-1) for m in ours.modules() if isinstance(m, torch.nn.BatchNorm2d)]
            results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()] + bufs).cpu())
            # explicit teardown before the process group goes: streams idle, graph and step
            # flags released in that order; a closed step refuses to run
            st.close()
            st.close()  # idempotent
            with pytest.raises(tspm_amd.TspmError):
                st.run()
        bad = (results[0] != results[1]).nonzero().reshape(-1)
        assert bad.numel() == 0, (bad.numel(), bad[:8].tolist(), (results[0] - results[1]).abs().max().item())
    finally:
        if created:
            dist.destroy_process_group()


def test_train_step_api_autograd_path(gpu):
    """AVMNIST.train_step with the reference's own torch.optim.Adam: autograd through the HIP
    encoder / head Functions (dropout off for a deterministic comparison)."""
    torch.manual_seed(11)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.0).to(gpu)
    opt = torch.optim.Adam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    o32, o64 = pair_from(ours, _build(11, dropout=0.0))
    audio, image, labels, _ = orc.synthetic_batch(16, seed=77)

    class Term:
        loss_fn = torch.nn.CrossEntropyLoss()
        weight = 1.0

        def __call__(self, x, y):
            return {"total_loss": self.loss_fn(x, y) * self.weight}

    class Group(dict):
        def __call__(self, x, y):
            out = {"total_loss": 0.0}
            for t in self.values():
                out["total_loss"] = out["total_loss"] + t(x, y)["total_loss"]
            return out

    saved = []  # tensors autograd saves (the head Function keeps fused, h1, hh and its weights)

    def pack(t):
        saved.append(t)
        return t
    batch = {"audio": audio, "image": image, "labels": labels, "pattern_name": ["ai"] * 16}
    p0, _, _ = snapshot(ours)
    with torch.autograd.graph.saved_tensors_hooks(pack, lambda t: t):
        r_ours = ours.train_step(batch, opt, Group(cross_entropy=Term()), gpu, None)
    torch.cuda.synchronize()
    forced = engine_decisions(ours.audio_encoder.engine_for(audio.to(gpu)), "audio.")
    forced.update(engine_decisions(ours.image_encoder.engine_for(image.to(gpu)), "image."))
    h1 = [t for t in saved if tuple(t.shape) == (16, 128)]
    hh = [t for t in saved if tuple(t.shape) == (16, 64)]
    assert len(h1) == 1 and len(hh) == 1
    forced.update(head_decisions(h1[0], hh[0]))
    r32, r64, t64 = _forced(o32, o64, audio, image, labels, None, forced)
    rep = flip_report(t64, forced)
    tally = Tally()
    check_out("loss", torch.tensor([r_ours["loss"]]), r32["loss"].reshape(1), r64["loss"].reshape(1), tally)
    _compare_params(ours, o32, o64, tally)
    check_adam(ours, opt, p0, None, None, 1)
    print(f"[autograd path] {flips_summary(rep)}; {tally}")


def test_fused_train_step_api_and_state_dict_roundtrip(gpu, tmp_path):
    """AVMNIST.train_step picks the fused path with FusedAdam; checkpoints keep the reference's
    state_dict keys / OIHW shapes and Adam state format and reload into a fresh model."""
    torch.manual_seed(0)
    m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(m.parameters(), lr=5e-4, weight_decay=1e-4)
    audio, image, labels, _ = orc.synthetic_batch(8, seed=3)
    batch = {"audio": audio, "image": image, "labels": labels, "pattern_name": ["ai"] * 8}
    for _ in range(3):
        r = m.train_step(batch, opt, None, gpu, None)
        assert np.isfinite(r["loss"])
    assert m._fused_step is not None and m._fused_step.calls == 3
    ck = tmp_path / "best.pth"
    torch.save({"model_state_dict": m.state_dict(), "optimizer_state_dict": opt.state_dict()}, ck)
    loaded = torch.load(ck, weights_only=True)
    ref = orc.build_oracle_avmnist(0)
    assert list(loaded["model_state_dict"]) == list(ref.state_dict())
    for k, v in ref.state_dict().items():
        assert loaded["model_state_dict"][k].shape == v.shape
    # every BatchNorm of both encoders counted 3 steps (the shared nbt counter, bumped by L.counters_add at the end
    # of each step)
    nbt = {k: int(v) for k, v in loaded["model_state_dict"].items() if k.endswith("num_batches_tracked")}
    assert len(nbt) == sum(isinstance(mm, torch.nn.BatchNorm2d) for mm in m.modules()) and set(nbt.values()) == {3}
    st = loaded["optimizer_state_dict"]["state"][0]
    assert float(st["step"]) == 3.0 and st["exp_avg"].shape == (64, 1, 7, 7)
    torch.manual_seed(1)
    m2 = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    m2.load_state_dict(loaded["model_state_dict"])
    opt2 = tspm_amd.FusedAdam(m2.parameters(), lr=5e-4, weight_decay=1e-4)
    opt2.load_state_dict(loaded["optimizer_state_dict"])
    for p, q in zip(m.parameters(), m2.parameters()):
        assert torch.equal(p.detach(), q.detach())
    m.eval(); m2.eval()
    with torch.no_grad():
        assert torch.equal(m(A=audio.to(gpu), I=image.to(gpu)), m2(A=audio.to(gpu), I=image.to(gpu)))


def test_pretrained_config_param_groups_run_fused_step(gpu, tmp_path):
    """The pretrained late-fusion config (train_avmnist_resnet_pretrained.yaml) builds its optimizer as
    getattr(torch.optim, "Adam")(param_groups) (train_multimodal.py:216-304): with the plugin that is
    FusedAdam over ONE group holding every parameter at the base settings (the recorded resolution,
    tests/golden/plugin_resolution.json).  The encoders' pretrained state_dicts load first
    (:156-204), then train_step must run the fused HIP graph step, and match the same step built with
    the keyword form of the optimizer bitwise."""
    torch.manual_seed(5)
    donor = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.0)
    torch.save(donor.audio_encoder.state_dict(), tmp_path / "encoder_audio_best.pth")
    torch.save(donor.image_encoder.state_dict(), tmp_path / "encoder_image_best.pth")
    audio, image, labels, _ = orc.synthetic_batch(16, seed=21)
    batch = {"audio": audio, "image": image, "labels": labels, "pattern_name": ["ai"] * 16}
    res = []
    for form in ("param_groups", "kwargs"):
        torch.manual_seed(0)
        m = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.0)
        m.audio_encoder.load_state_dict(torch.load(tmp_path / "encoder_audio_best.pth", weights_only=True))
        m.image_encoder.load_state_dict(torch.load(tmp_path / "encoder_image_best.pth", weights_only=True))
        m.to(gpu)
        if form == "param_groups":
            opt = tspm_amd.plugin._OptimProxy(torch.optim).Adam([{"params": list(m.parameters()), "lr": 5e-4,
                                                                   "weight_decay": 1e-4}])
        else:
            opt = tspm_amd.FusedAdam(m.parameters(), lr=5e-4, weight_decay=1e-4)
        assert isinstance(opt, tspm_amd.FusedAdam)
        for _ in range(3):
            m.train_step(batch, opt, None, gpu, None)
        assert m._fused_step is not None and m._fused_step.calls == 3
        torch.cuda.synchronize()
        res.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("knob,values", [("TSPM_SLACK_LDS_FLOOR", ("0", "82000")),
                                         ("TSPM_ADAM_CARRY", ("none", "image")),
                                         ("TSPM_ADAM_CARRY", ("none", "both"))])
def test_step_schedules_leave_the_step_bitwise_unchanged(gpu, monkeypatch, knob, values):
    """Scheduling switches of the single-GPU step change no arithmetic: the audio encoder's LDS floor (only how
    many workgroups share a CU) and the Adam updates carried by later backward launches (tspm_conv_bwd_adam:
    tspm_adam_step's element loop over the finished blocks' ranges) — four replayed steps' parameters, BN buffers
    and Adam moments are bitwise those of the plain schedule."""
    results = []
    for val in values:
        monkeypatch.setenv(knob, val)
        torch.manual_seed(17)
        ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        st = tspm_amd.FusedTrainStep(ours, opt, None, 32)
        for i in range(4):
            audio, image, labels, _ = orc.synthetic_batch(32, seed=40 + i)
            st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        bufs = [t.detach().reshape(-1) for m in ours.modules() if isinstance(m, torch.nn.BatchNorm2d)
                for t in (m.running_mean, m.running_var)]
        mom = [t for fg in opt.flat_groups() for t in (fg.exp_avg, fg.exp_avg_sq)]
        results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()] + bufs + mom).cpu())
        st.close()
    assert torch.equal(results[0], results[1])


def test_floored_and_unfloored_steps_interleaved_are_bitwise_the_plain_step(gpu, monkeypatch):
    """ABI 21: the audio LDS floor is a per-launch tspm_conv_algo field on the step's own audio
    engine, not library state.  Two floored steps and one unfloored step, built and run in interleaved order (each
    builds and captures its graph between the others' replays), all end bitwise equal to the plain step — no floor
    leaks into another step's launches and none is lost."""
    cfg = [("82000", "fa"), ("0", "pl"), ("82000", "fb")]
    steps, models, opts = {}, {}, {}
    for floor, tag in cfg:
        monkeypatch.setenv("TSPM_SLACK_LDS_FLOOR", floor)
        torch.manual_seed(23)
        models[tag] = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opts[tag] = tspm_amd.FusedAdam(models[tag].parameters(), lr=5e-4, weight_decay=1e-4)
        steps[tag] = tspm_amd.FusedTrainStep(models[tag], opts[tag], None, 64)
        assert steps[tag].slack_lds_floor == int(floor)
    monkeypatch.delenv("TSPM_SLACK_LDS_FLOOR")
    batches = [orc.synthetic_batch(64, seed=70 + i) for i in range(4)]
    for i, (audio, image, labels, _) in enumerate(batches):
        order = ("fa", "pl", "fb") if i % 2 == 0 else ("fb", "pl", "fa")
        for tag in order:
            steps[tag].step(audio.to(gpu), image.to(gpu), labels.to(gpu))
            assert steps[tag].eng_a.lds_floor == 0  # the floor is set only while the step enqueues its audio launches
    torch.cuda.synchronize()
    res = {}
    for tag in steps:
        m, opt = models[tag], opts[tag]
        bufs = [t.detach().reshape(-1) for mm in m.modules() if isinstance(mm, torch.nn.BatchNorm2d)
                for t in (mm.running_mean, mm.running_var)]
        mom = [t for fg in opt.flat_groups() for t in (fg.exp_avg, fg.exp_avg_sq)]
        res[tag] = torch.cat([p.detach().reshape(-1) for p in m.parameters()] + bufs + mom).cpu()
        steps[tag].close()
    assert torch.equal(res["fa"], res["pl"]) and torch.equal(res["fb"], res["pl"])
