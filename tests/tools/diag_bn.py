"""Diagnostics for BN backward and model-level error vs an fp64 oracle (GPU box)."""
import sys
import os
_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, _REPO)
sys.path.insert(0, os.path.join(_REPO, "tests"))
import torch
import torch.nn.functional as F
import tspm_amd
from tspm_amd import _lib as L
from oracle import avmnist_ref as orc

dev = torch.device("cuda", 0)
lib = L.lib()
sh = L.stream_handle


def rel(a, b):
    a = a.double().cpu().reshape(-1); b = b.double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def bn_case(m, c):
    g = torch.Generator().manual_seed(5)
    y = torch.randn(m, c, generator=g) * 3 + 1
    gamma, beta = torch.randn(c, generator=g), torch.randn(c, generator=g)
    gout = torch.randn(m, c, generator=g)
    yd = y.double().requires_grad_(True)
    ga = gamma.double().requires_grad_(True); be = beta.double().requires_grad_(True)
    z = F.batch_norm(yd.T[None, :, :, None], None, None, ga, be, True, 0.0, 1e-5)[0, :, :, 0].T
    out_ref = torch.relu(z)
    out_ref.backward(gout.double())
    y_, g_, gm, bt = y.to(dev), gout.to(dev), gamma.to(dev), beta.to(dev)
    mean, inv = torch.empty(c, device=dev), torch.empty(c, device=dev)
    wsb = max(lib.tspm_bn_stats_workspace(m, c), lib.tspm_bn_bwd_workspace(m, c))
    ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
    L.check(lib.tspm_bn_stats(m, c, y_.data_ptr(), 1, 0, None, None, None, 0.1, 1e-5, mean.data_ptr(), inv.data_ptr(),
                              ws.data_ptr(), wsb, sh()), "stats")
    out = torch.empty(m, c, device=dev)
    L.check(lib.tspm_bn_apply(m, c, y_.data_ptr(), mean.data_ptr(), inv.data_ptr(), gm.data_ptr(), bt.data_ptr(), 0,
                              None, None, None, None, None, 1, out.data_ptr(), None, 0, sh()), "apply")
    dy = torch.empty(m, c, device=dev)
    gw, gb = torch.empty(c, device=dev), torch.empty(c, device=dev)
    L.check(lib.tspm_bn_bwd(m, c, g_.data_ptr(), out.data_ptr(), y_.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                            gm.data_ptr(), gw.data_ptr(), gb.data_ptr(), dy.data_ptr(), None, None, None, None, None,
                            None, None, None, None, None, 0, ws.data_ptr(), wsb, sh()), "bwd")
    torch.cuda.synchronize()
    G = lib.tspm_bn_stats_workspace(m, c) // (2 * c * 4)
    # torch-on-gpu recomputation of the sums for comparison
    gp = g_ * (out > 0)
    sg = gp.double().sum(0); sx = (gp.double() * (y_.double() - mean.double())).sum(0)
    print(f"m={m} c={c} G={G} out rel {rel(out, out_ref.detach()):.2e} dbeta rel {rel(gb, be.grad):.2e} "
          f"dgamma rel {rel(gw, ga.grad):.2e} dy rel {rel(dy, yd.grad):.2e} | sg-vs-torch {rel(gb, sg):.2e} "
          f"sx*inv-vs-torch {rel(gw, sx * inv.double()):.2e}")


if "--bn" in sys.argv:
    for m, c in [(64, 64), (1024, 64), (4096, 64), (6272, 64), (512, 256), (128, 512), (384, 512), (3008, 64)]:
        bn_case(m, c)


# ---- model-level: errors of ours and of the fp32 oracle against an fp64 oracle --------------------
def model_case(batch, seed=3):
    torch.manual_seed(seed)
    ours = tspm_amd.ResNet18(1, 64).to(dev)
    torch.manual_seed(seed)
    r32 = orc.oracle_resnet18(1, 64)
    torch.manual_seed(seed)
    r64 = orc.oracle_resnet18(1, 64).double()
    audio, _, _, _ = orc.synthetic_batch(batch, seed=99)
    g = torch.randn(batch, 64, generator=torch.Generator().manual_seed(5))
    e = ours(audio.to(dev)); e.backward(g.to(dev))
    e32 = orc.encoder_forward(r32, audio, True); e32.backward(g)
    e64 = orc.encoder_forward(r64, audio.double(), True); e64.backward(g.double())
    print(f"B={batch}: emb ours {rel(e, e64):.2e} oracle32 {rel(e32, e64):.2e}")
    worst = []
    for (n, p), (_, q), (_, d) in zip(ours.named_parameters(), r32.named_parameters(), r64.named_parameters()):
        eo, e3 = rel(p.grad, d.grad), rel(q.grad, d.grad)
        worst.append((eo / max(e3, 1e-7), n, eo, e3))
    for w in worst[::-1]:
        print(f"   {w[1]:40s} ours {w[2]:.2e} oracle32 {w[3]:.2e} ratio {w[0]:.1f}")


for b in (128,):
    model_case(b)
