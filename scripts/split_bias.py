"""Error profile of variant 4 (bf16-piece products) against variant 1 (f32 MFMA) vs fp64: rel-L2, max normalised
error and the signed bias (mean error / mean |ref|) — a biased rounding inside the bf16 MFMA accumulation would show
in the bias, and in long sums downstream (BN weight gradients).   python scripts/split_bias.py"""
import os
import sys

import torch
import torch.nn.functional as F

_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [_R, os.path.join(_R, "tests")]
from abi_helpers import conv_dgrad, conv_fwd, conv_wgrad  # noqa: E402

dev = torch.device("cuda", 0)
for case in [(256, 64, 8, 24, 64, 3, 3, 1, 1), (256, 256, 2, 2, 256, 3, 3, 1, 1), (512, 512, 1, 1, 512, 3, 3, 1, 1)]:
    n, c, h, w, k, r, s, st, pad = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(n, c, h, w, generator=g)
    wt = torch.randn(k, c, r, s, generator=g) * 0.05
    p, q = (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1
    dy = torch.randn(n, k, p, q, generator=g)
    refs = {"fwd": F.conv2d(x.double(), wt.double(), None, st, pad),
            "dgrad": torch.nn.grad.conv2d_input((n, c, h, w), wt.double(), dy.double(), st, pad),
            "wgrad": torch.nn.grad.conv2d_weight(x.double(), (k, c, r, s), dy.double(), st, pad)}
    xg, wg, dyg = x.to(dev), wt.to(dev), dy.to(dev)
    for v in (1, 4):
        a = (1, 1, 2, 1, 1, v)
        outs = {"fwd": conv_fwd(xg, wg, st, pad, a), "dgrad": conv_dgrad(dyg, wg, (h, w), st, pad, a),
                "wgrad": conv_wgrad(xg, dyg, (r, s), st, pad, a)}
        for kind, ref in refs.items():
            o = outs[kind].double().cpu()
            e = o - ref
            print(f"{str(case):36s} v{v} {kind:5s} rel-L2 {e.norm() / ref.norm():.3e}  bias {e.mean() / ref.abs().mean():+.3e}"
                  f"  mean|e|/mean|ref| {e.abs().mean() / ref.abs().mean():.3e}", flush=True)
