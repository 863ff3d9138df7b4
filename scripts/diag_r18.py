"""Compare backward intermediates of the HIP ResNet18 (B=128) with fp64 and fp32 autograd."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import torch.nn.functional as F
import tspm_amd
from oracle import avmnist_ref as orc

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128


def hwnc(t):  # NCHW -> [H*W*N, C]
    n, c, h, w = t.shape
    return t.permute(2, 3, 0, 1).reshape(h * w * n, c)


def rel(a, b):
    a = a.double().cpu().reshape(-1); b = b.double().cpu().reshape(-1)
    return ((a - b).norm() / b.norm().clamp_min(1e-300)).item()


def run_ref(enc, x, g):
    """encoder forward with retained intermediates (per block: g_out, d_y2, d_a1, d_y1)."""
    keep = {}
    if x.dim() == 3:
        x = x.unsqueeze(1)
    h = F.conv2d(x, enc.conv1.weight, None, 2, 3)
    h = F.relu(F.batch_norm(h, None, None, enc.bn1.weight, enc.bn1.bias, True, 0.1, 1e-5))
    h = F.max_pool2d(h, 3, 2, 1)
    i = 0
    for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
        for b in layer:
            y1 = F.conv2d(h, b.conv1.weight, None, b.stride, 1); y1.retain_grad()
            a1 = F.relu(F.batch_norm(y1, None, None, b.bn1.weight, b.bn1.bias, True, 0.1, 1e-5)); a1.retain_grad()
            y2 = F.conv2d(a1, b.conv2.weight, None, 1, 1); y2.retain_grad()
            z = F.batch_norm(y2, None, None, b.bn2.weight, b.bn2.bias, True, 0.1, 1e-5)
            if b.downsample is not None:
                c, bn = b.downsample[0], b.downsample[1]
                idn = F.batch_norm(F.conv2d(h, c.weight, None, c.stride, 0), None, None, bn.weight, bn.bias, True, 0.1, 1e-5)
            else:
                idn = h
            h = F.relu(z + idn); h.retain_grad()
            keep[i] = (h, y2, a1, y1)
            i += 1
    e = F.linear(F.adaptive_avg_pool2d(h, 1).flatten(1), enc.fc.weight, enc.fc.bias)
    e.backward(g)
    out = {}
    for i, (h, y2, a1, y1) in keep.items():
        out[f"block{i}.g_out"] = hwnc(h.grad); out[f"block{i}.d_y2"] = hwnc(y2.grad)
        out[f"block{i}.d_a1"] = hwnc(a1.grad); out[f"block{i}.d_y1"] = hwnc(y1.grad)
    return out


WHICH = sys.argv[2] if len(sys.argv) > 2 else "audio"
ctor, octor, hid = (tspm_amd.ResNet18, orc.oracle_resnet18, 64) if WHICH == "audio" else (tspm_amd.ResNet34, orc.oracle_resnet34, 128)
torch.manual_seed(3); ours = ctor(1, hid).to(dev)
torch.manual_seed(3); r32 = octor(1, hid)
torch.manual_seed(3); r64 = octor(1, hid).double()
audio, image, _, _ = orc.synthetic_batch(B, seed=99)
if WHICH != "audio":
    audio = image
g = torch.randn(B, hid, generator=torch.Generator().manual_seed(5))
got = {}
x = audio.to(dev)
eng = ours.engine_for(x)
eng.debug_hook = lambda name, t: got.__setitem__(name, t.detach().clone().cpu())
e = ours(x); e.backward(g.to(dev)); torch.cuda.synchronize()
ref64 = run_ref(r64, audio.double(), g.double())
ref32 = run_ref(r32, audio, g)
for k in sorted(ref64, key=lambda s: (-int(s.split('.')[0][5:]), s)):
    n = ref64[k].numel()
    a = got[k].reshape(-1)[:n]
    colsum64 = ref64[k].sum(0)
    print(f"{k:16s} ours {rel(a, ref64[k]):.2e} fp32-oracle {rel(ref32[k], ref64[k]):.2e} | colsum ours "
          f"{rel(a.view_as(ref64[k]).double().sum(0), colsum64):.2e} fp32 {rel(ref32[k].double().sum(0), colsum64):.2e}")

print("param grads (ours / fp32 oracle, rel to fp64):")
for (n, p), (_, q), (_, d) in zip(ours.named_parameters(), r32.named_parameters(), r64.named_parameters()):
    eo, e3 = rel(p.grad, d.grad), rel(q.grad, d.grad)
    flag = "  <<<" if eo > 4 * e3 + 2e-5 else ""
    print(f"   {n:40s} {eo:.2e} / {e3:.2e}{flag}")

# ---- relu-mask agreement of block outputs: ours / fp32 oracle vs fp64 -------------------------------
def block_outputs(enc, x):
    outs = []
    if x.dim() == 3:
        x = x.unsqueeze(1)
    with torch.no_grad():
        h = F.conv2d(x, enc.conv1.weight, None, 2, 3)
        h = F.relu(F.batch_norm(h, None, None, enc.bn1.weight, enc.bn1.bias, True, 0.1, 1e-5))
        h = F.max_pool2d(h, 3, 2, 1)
        for layer in (enc.layer1, enc.layer2, enc.layer3, enc.layer4):
            for b in layer:
                y1 = F.conv2d(h, b.conv1.weight, None, b.stride, 1)
                a1 = F.relu(F.batch_norm(y1, None, None, b.bn1.weight, b.bn1.bias, True, 0.1, 1e-5))
                z = F.batch_norm(F.conv2d(a1, b.conv2.weight, None, 1, 1), None, None, b.bn2.weight, b.bn2.bias, True, 0.1, 1e-5)
                if b.downsample is not None:
                    c, bn = b.downsample[0], b.downsample[1]
                    idn = F.batch_norm(F.conv2d(h, c.weight, None, c.stride, 0), None, None, bn.weight, bn.bias, True, 0.1, 1e-5)
                else:
                    idn = h
                h = F.relu(z + idn)
                outs.append((a1, h))
    return outs

# weights were updated by nothing (no optimizer) -> same as at the forward above
o64 = block_outputs(r64, audio.double())
o32 = block_outputs(r32, audio)
print("relu-mask flips vs fp64 (a1 / out): ours | fp32-oracle")
for i, bp in enumerate(eng.blocks):
    a64, h64 = o64[i]
    a32, h32 = o32[i]
    n, c, hh, ww = h64.shape
    ours_out = bp.out.detach().cpu().view(hh, ww, n, c).permute(2, 3, 0, 1)
    ours_a1 = bp.a1.detach().cpu().view(hh, ww, n, c).permute(2, 3, 0, 1)
    f_o = int(((ours_out > 0) != (h64 > 0)).sum()); f_a = int(((ours_a1 > 0) != (a64 > 0)).sum())
    r_o = int(((h32 > 0) != (h64 > 0)).sum()); r_a = int(((a32 > 0) != (a64 > 0)).sum())
    print(f"  block{i:2d}: {f_a:3d} / {f_o:3d}  |  {r_a:3d} / {r_o:3d}   (of {h64.numel()})")
