"""Diagnostic: where does the MMIMDb step's input-BatchNorm1d gamma gradient lose precision at n=4?
Compares intermediate gradients of the fused HIP step with fp32 / fp64 oracle runs (MaxOut choices
forced).  Prints rel-L2 errors per stage."""
import copy
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import tspm_amd  # noqa: E402
from oracle import mmimdb_ref as orc  # noqa: E402
from test_mmimdb_cpu import dropin  # noqa: E402
from tspm_amd import mmimdb as M  # noqa: E402
from parity import rel_l2  # noqa: E402

dev = torch.device("cuda", 0)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ours = dropin(0).to(dev)
opt = tspm_amd.FusedAdam(ours.parameters(), lr=1e-5, weight_decay=1e-3)
st = M.FusedMMIMDbStep(ours, opt, None, n, use_graph=False)
I, T, y = orc.synthetic_batch(n, seed=77)
keep = (torch.rand(2, n, 512, generator=torch.Generator().manual_seed(10)) >= 0.5).to(torch.uint8)
st.keep_override = keep.to(dev)
st.step(I.to(dev), T.to(dev), y.to(dev))
torch.cuda.synchronize()
e = st.eng
forced = {}
for site, A in (("mo1", e.A1), ("mo2", e.A2)):
    a = A.cpu()
    h = a.shape[1] // 2
    forced[site] = torch.where(a[:, h:] > a[:, :h], 1, torch.where(a[:, h:] == a[:, :h], 2, 0)).to(torch.int8)

res = {}
stages = {}
for dt in (torch.float32, torch.float64):
    o = orc.build_oracle_mmimdb(0).to(dt)
    t = {}

    def keep_t(name, v):
        v.retain_grad()
        t[name] = v
        return v
    for p_ in o.parameters():
        p_.grad = None
    o.train()
    Z = keep_t("Z", o.fusion_module(o.image_model(I.to(dt)), o.text_model(T.to(dt))))
    net = o.mm_mlp.net
    tr = orc.MaxOutTrace(forced)
    Zn = keep_t("Zn", net[0](Z))
    A1 = net[1](Zn, tr, "mo1")
    Y1 = keep_t("Y1", A1 * (keep[0].to(dt) * 2.0))
    Y1n = keep_t("Y1n", net[3](Y1))
    A2 = net[4](Y1n, tr, "mo2")
    Y2 = keep_t("Y2", A2 * (keep[1].to(dt) * 2.0))
    Y2n = keep_t("Y2n", net[6](Y2))
    lg = keep_t("logits", net[7](Y2n))
    loss = orc.bce_loss(lg, y.to(dt))
    loss.backward()
    stages[dt] = {k: (v.detach().clone(), v.grad.detach().clone()) for k, v in t.items()}
ourf = {"Z": e.Z, "Zn": e.Zn, "Y1": e.Y1, "Y1n": e.Y1n, "Y2": e.Y2, "Y2n": e.Y2n, "logits": e.logits}
ourg = {"Z": e.dZ, "Zn": e.dZn, "Y1": e.dY1, "Y1n": e.dY1n, "Y2": e.dY2, "Y2n": e.dY2n, "logits": e.dlogits}
for k in ("Z", "Zn", "Y1", "Y1n", "Y2", "Y2n", "logits"):
    f64, g64 = stages[torch.float64][k]
    f32, g32 = stages[torch.float32][k]
    print(f"{k:6s} fwd ours {rel_l2(ourf[k].cpu(), f64):.2e} ref {rel_l2(f32, f64):.2e}   "
          f"grad ours {rel_l2(ourg[k].cpu(), g64):.2e} ref {rel_l2(g32, g64):.2e}")
# BN b2 backward in fp64 on OUR inputs (x = Y2, g = dY2n): isolates the kernel from its inputs
x = e.Y2.cpu().double()
gg = e.dY2n.cpu().double()
gam = ours.mm_mlp.net[6].weight.detach().cpu().double()
mu = x.mean(0)
var = x.var(0, unbiased=False)
inv = 1 / (var + 1e-5).sqrt()
xh = (x - mu) * inv
dx = gam * inv * (gg - gg.mean(0) - xh * (gg * xh).mean(0))
print("b2 kernel vs fp64-on-our-inputs:", f"{rel_l2(e.dY2.cpu(), dx):.2e}",
      " fp64-on-our-inputs vs truth:", f"{rel_l2(dx, stages[torch.float64]['Y2'][1]):.2e}")
x64 = stages[torch.float64]["Y2"][0]
g64 = stages[torch.float64]["Y2n"][1]
for lab, xx, g_ in (("truth x, our g", x64, gg), ("our x, truth g", x, g64)):
    mu = xx.mean(0); inv = 1 / (xx.var(0, unbiased=False) + 1e-5).sqrt(); xh = (xx - mu) * inv
    d_ = gam * inv * (g_ - g_.mean(0) - xh * (g_ * xh).mean(0))
    print(f"  {lab}: {rel_l2(d_, stages[torch.float64]['Y2'][1]):.2e}")
print("ours invstd range", inv.min().item(), inv.max().item())
x32 = stages[torch.float32]["Y2"][0].double()
for lab, xx in (("ref32 x", x32), ("our x", x)):
    mu = xx.mean(0); inv = 1 / (xx.var(0, unbiased=False) + 1e-5).sqrt(); xh = (xx - mu) * inv
    d_ = gam * inv * (g64 - g64.mean(0) - xh * (g64 * xh).mean(0))
    err = (d_ - stages[torch.float64]['Y2'][1]).pow(2).sum(0)
    top = err.argsort(descending=True)[:3]
    print(f"  {lab} truth g: {rel_l2(d_, stages[torch.float64]['Y2'][1]):.2e}; worst channels {top.tolist()}")
    for ch in top.tolist():
        print("     ch", ch, "x64", x64[:, ch].tolist(), "dx", (xx[:, ch] - x64[:, ch]).tolist(), "inv", inv[ch].item())
