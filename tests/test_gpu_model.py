"""End-to-end parity of the HIP encoders / fused train step against the reference.

Ground truth is the oracle run in fp64 (same seeded weights, inputs and dropout mask).  The
reference itself computes in fp32 (ATen CPU); at batch 128 its own gradients are ~1e-3 away from
fp64 (the 1e-9…1.5e7 audio input and the tiny late feature maps make the step ill-conditioned), so
a fixed absolute threshold would be meaningless.  Criterion, per tensor:

    rel_l2(ours, fp64) <= FACTOR * rel_l2(reference_fp32, fp64) + FLOOR

with FACTOR = 4 and FLOOR = 2e-6 (outputs) / 2e-5 (gradients).  The fp32 reference is either the
golden vectors captured from the real MML_Suite code (B=4) or the oracle in fp32 (bit-identical to
the reference on CPU, pinned by tests/test_oracle_golden.py).

ReLU-threshold flips: an activation with |bn(y) + residual| below fp32 rounding can land on either
side of zero in ANY fp32 implementation (measured: 1-2 of ~2.6M mask elements per encoder at
B=128, for ours and for the fp32 oracle alike, seed-dependent — scripts/diag_r18.py).  One flip
perturbs every upstream gradient by ~1e-3 relative; max-pool argmax near-ties on the quantised
MNIST images (LUT/255 pixels, 81 % zeros) behave the same way for the stem gradients.  Gradients
therefore pass either the tight criterion above or, when such a flip has occurred, rel_l2 <= 2e-2
with cosine >= 0.9999 (a wrong kernel gives O(1) errors: tests/test_gpu_ops.py bounds every kernel
element-wise).

Adam: its first step is ~lr * sign(g), so parameter trajectories amplify rounding of tiny
gradient elements; the optimizer is therefore checked exactly against fp64 Adam applied to OUR
gradients, and multi-step logits/losses against the fp64 trajectory within max(5 %, 4x the fp32
reference's own deviation) (chaotic regime: B=4 batch statistics over 4 samples at 1x1 maps).
"""
import copy

import numpy as np
import pytest
import torch

import tspm_amd
from oracle import avmnist_ref as orc

pytestmark = pytest.mark.gpu
FACTOR = 4.0
FLOOR_OUT = 2e-6
FLOOR_GRAD = 2e-5


def rel_l2(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def check(name, ours, ref32, ref64, floor):
    e_ours, e_ref = rel_l2(ours, ref64), rel_l2(ref32, ref64)
    assert e_ours <= FACTOR * e_ref + floor, f"{name}: ours {e_ours:.3e} vs fp32-reference {e_ref:.3e} (fp64 truth)"
    return e_ours, e_ref


def cosine(a, b):
    a = torch.as_tensor(a).detach().double().cpu().reshape(-1)
    b = torch.as_tensor(b).detach().double().cpu().reshape(-1)
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-300)).item()


def check_grad(name, ours, ref32, ref64):
    """Tight criterion, or the ReLU-flip-tolerant one (module docstring)."""
    e_ours, e_ref = rel_l2(ours, ref64), rel_l2(ref32, ref64)
    if e_ours <= FACTOR * e_ref + FLOOR_GRAD:
        return "tight"
    assert e_ours <= 2e-2 and cosine(ours, ref64) >= 0.9999, \
        f"{name}: ours {e_ours:.3e} vs fp32-reference {e_ref:.3e} (fp64 truth), cos {cosine(ours, ref64):.6f}"
    return "flip"


def adam_fp64(p0, g, step, lr=5e-4, wd=1e-4, b1=0.9, b2=0.999, eps=1e-8, m=None, v=None):
    p0, g = p0.double(), g.double()
    g = g + wd * p0
    m = (1 - b1) * g if m is None else b1 * m + (1 - b1) * g
    v = (1 - b2) * g * g if v is None else b2 * v + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    return p0 - (lr / bc1) * m / (v.sqrt() / bc2 ** 0.5 + eps), m, v


def oracle_pair(seed, dropout=0.5):
    o32 = orc.build_oracle_avmnist(seed, dropout=dropout)
    o64 = copy.deepcopy(o32).double()
    return o32, o64


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
    r64 = copy.deepcopy(r32).double()
    g = torch.randn(batch, hid, generator=torch.Generator().manual_seed(5))
    emb = ours(x.to(gpu))
    emb.backward(g.to(gpu))
    e32 = orc.encoder_forward(r32, x, True)
    e32.backward(g)
    e64 = orc.encoder_forward(r64, x.double(), True)
    e64.backward(g.double())
    check("embedding", emb, e32, e64, FLOOR_OUT)
    for (n, p), (_, q), (_, d) in zip(ours.named_parameters(), r32.named_parameters(), r64.named_parameters()):
        assert p.grad is not None, n
        check_grad(f"grad {n}", p.grad, q.grad, d.grad)
    sd, s32, s64 = ours.state_dict(), r32.state_dict(), r64.state_dict()
    for k in s64:
        if k.endswith("running_mean") or k.endswith("running_var"):
            check(k, sd[k], s32[k], s64[k], FLOOR_OUT)
        if k.endswith("num_batches_tracked"):
            assert int(sd[k]) == int(s32[k]) == 1, k


def _fp64_steps(o64, audio, image, labels, masks):
    opt = orc.OracleAdam(list(o64.parameters()), lr=5e-4, weight_decay=1e-4)
    out = []
    for m in masks:
        r = orc.train_step(o64, opt, audio.double(), image.double(), labels, m)
        out.append((r["logits"], r["loss"], {n: p.grad.clone() for n, p in o64.named_parameters()},
                    {n: p.detach().clone() for n, p in o64.named_parameters()}))
    return out


def test_fused_step_vs_golden_reference(gpu, golden):
    """3 fused HIP train steps (eager first call, captured graph afterwards) against the vectors
    captured from the real MML_Suite AVMNIST.train_step (B=4, seed-0 weights, reference's dropout
    masks), with the fp64 oracle as the yardstick."""
    torch.manual_seed(0)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    audio, image = torch.from_numpy(golden["audio"]), torch.from_numpy(golden["image"])
    labels = torch.from_numpy(golden["labels"])
    masks = [torch.from_numpy(m) for m in golden["keep_masks"]]
    _, o64 = oracle_pair(0)
    truth = _fp64_steps(o64, audio, image, labels, masks)
    step = tspm_amd.FusedTrainStep(ours, opt, None, 4)
    names = list(golden["param_names"])
    params = dict(ours.named_parameters())
    for s in range(3):
        step.keep_override = masks[s].to(gpu)
        out = step.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        lg64, loss64, g64, _ = truth[s]
        if s == 0:
            check("logits step 0", out["logits"], golden["logits"][s], lg64, FLOOR_OUT)
            check("loss step 0", out["loss"], torch.tensor([golden["losses"][s]]), loss64.reshape(1), FLOOR_OUT)
        else:  # after Adam steps: trajectory criterion (module docstring)
            e_ref = rel_l2(golden["logits"][s], lg64)
            e_ours = rel_l2(out["logits"], lg64)
            assert e_ours < max(5e-2, FACTOR * e_ref), (s, e_ours, e_ref)
            assert rel_l2(out["loss"], loss64.reshape(1)) < max(5e-2, FACTOR * rel_l2(
                torch.tensor([golden["losses"][s]]), loss64.reshape(1))), (s, out["loss"].item(), loss64.item())
        if s == 0:
            gn = np.array([params[n].grad.double().norm().item() for n in names])
            gn64 = np.array([g64[n].norm().item() for n in names])
            check("grad norms step 1", gn, golden["grad_norm_step1"], gn64, FLOOR_GRAD)
    ours.eval()
    with torch.no_grad():
        ev = ours(A=audio.to(gpu), I=image.to(gpu))
    o64.eval()
    with torch.no_grad():
        ev64, _, _ = orc.avmnist_forward(o64, audio.double(), image.double(), False)
    # after 3 Adam steps (trajectory criterion; B=4 running statistics of 4-sample batches)
    e_ref, e_ours = rel_l2(golden["eval_logits"], ev64), rel_l2(ev, ev64)
    assert e_ours < max(0.1, FACTOR * e_ref), (e_ours, e_ref)


@pytest.mark.parametrize("batch", [32, 128])
def test_fused_step_vs_oracle(gpu, batch):
    torch.manual_seed(3)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
    opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    o32, o64 = oracle_pair(3)
    opt32 = orc.OracleAdam(list(o32.parameters()), lr=5e-4, weight_decay=1e-4)
    audio, image, labels, _ = orc.synthetic_batch(batch, seed=1234)
    keep = (torch.rand(batch, 128, generator=torch.Generator().manual_seed(8)) > 0.5).to(torch.uint8)
    truth = _fp64_steps(o64, audio, image, labels, [keep, keep])
    step = tspm_amd.FusedTrainStep(ours, opt, None, batch)
    p0 = {n: p.detach().cpu().double().clone() for n, p in ours.named_parameters()}
    for s in range(2):
        step.keep_override = keep.to(gpu)
        out = step.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        r = orc.train_step(o32, opt32, audio, image, labels, keep)
        torch.cuda.synchronize()
        lg64, loss64, g64, p64 = truth[s]
        if s == 0:
            check("logits step 0", out["logits"], r["logits"], lg64, FLOOR_OUT)
            for (n, p), (_, q) in zip(ours.named_parameters(), o32.named_parameters()):
                check_grad(f"grad {n}", p.grad, q.grad, g64[n])
                # the optimizer, exactly: fp64 Adam applied to OUR gradient reproduces OUR update
                exp, _, _ = adam_fp64(p0[n], p.grad.detach().cpu(), 1)
                got = p.detach().cpu().double()
                assert ((got - exp).abs() <= 1e-6 * exp.abs() + 2e-9).all(), n
        else:  # after one Adam step (trajectory criterion, module docstring)
            e_ref = rel_l2(r["logits"], lg64)
            assert rel_l2(out["logits"], lg64) < max(5e-2, FACTOR * e_ref), (rel_l2(out["logits"], lg64), e_ref)


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


def test_phased_allreduce_step_equals_plain_step(gpu):
    """The DP step path — backward split in two phases, graph 1 | RCCL all-reduce of phase-1
    gradients overlapping graph 2 | RCCL of the rest | Adam graph — under a 1-rank RCCL group
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
            bufs = [m.running_var.detach().reshape(-1) for m in ours.modules() if isinstance(m, torch.nn.BatchNorm2d)]
            results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()] + bufs).cpu())
        assert torch.equal(results[0], results[1])
    finally:
        if created:
            dist.destroy_process_group()


def test_train_step_api_autograd_path(gpu):
    """AVMNIST.train_step with the reference's own torch.optim.Adam: autograd through the HIP
    encoder / head Functions (dropout off for a deterministic comparison)."""
    torch.manual_seed(11)
    ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.0).to(gpu)
    opt = torch.optim.Adam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
    o32, o64 = oracle_pair(11, dropout=0.0)
    opt32 = orc.OracleAdam(list(o32.parameters()), lr=5e-4, weight_decay=1e-4)
    audio, image, labels, _ = orc.synthetic_batch(16, seed=77)
    truth = _fp64_steps(o64, audio, image, labels, [None])

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

    batch = {"audio": audio, "image": image, "labels": labels, "pattern_name": ["ai"] * 16}
    p0 = {n: p.detach().cpu().double().clone() for n, p in ours.named_parameters()}
    r_ours = ours.train_step(batch, opt, Group(cross_entropy=Term()), gpu, None)
    r32 = orc.train_step(o32, opt32, audio, image, labels, None)
    _, loss64, g64, p64 = truth[0]
    check("loss", torch.tensor([r_ours["loss"]]), r32["loss"].reshape(1), loss64.reshape(1), FLOOR_OUT)
    for (n, p), (_, q) in zip(ours.named_parameters(), o32.named_parameters()):
        check_grad(f"grad {n}", p.grad, q.grad, g64[n])
        exp, _, _ = adam_fp64(p0[n], p.grad.detach().cpu(), 1)
        assert ((p.detach().cpu().double() - exp).abs() <= 1e-6 * exp.abs() + 2e-9).all(), n


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
    assert int(loaded["model_state_dict"]["audio_encoder.bn1.num_batches_tracked"]) == 3
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


def test_overlapped_adam_equals_plain_step(gpu):
    """Single-GPU step with the late layers' Adam on a third stream, overlapping the early layers'
    backward (FusedTrainStep.overlap_opt), is bitwise the plain step (Adam is element-wise), eager and
    graph-replayed, parameters and optimizer state alike."""
    results = []
    for overlap in ("0", "stream", "main"):
        torch.manual_seed(13)
        ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        st = tspm_amd.FusedTrainStep(ours, opt, None, 32, use_graph=True)
        st.overlap_opt = overlap
        for i in range(4):
            audio, image, labels, _ = orc.synthetic_batch(32, seed=70 + i)
            st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        fg = opt.flat_groups()[0]
        results.append(torch.cat([fg.param, fg.exp_avg, fg.exp_avg_sq]).cpu())
    assert torch.equal(results[0], results[1]) and torch.equal(results[0], results[2])
