"""Parity at per-rank batch 1024 (BASELINE configs[2]'s other per-rank reading, the one the
batch-1024 line in DESIGN §5 is measured on).

Every entry of the batch-1024 tuned table (``tuned/mi355x_b1024.json``: variant-2 LDS-DMA kernels, register-direct
and stem configurations, the fused dgrad + wgrad pairs) runs at its exact layer shape (M up to 786k rows) and is held
element-wise to the fp64 convolution with the conv tolerance of tests/test_gpu_ops.py:
|y - y_ref| <= 64 * 2^-23 * sum|w||x| per element.  The fused backward launch of a pair is additionally bitwise the
two separate launches.  The whole fused train step at batch 1024 is checked against the forced-decision fp64 oracle
in tests/test_gpu_model.py::test_fused_step_vs_oracle[1024]."""
import ctypes
import json
import os

import pytest
import torch
import torch.nn.functional as F

from abi_helpers import conv_bound, conv_dgrad, conv_fwd, conv_wgrad, shape, to_hwnc
from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu
EPS32 = 2.0 ** -23
TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                     "task-specific-pretraining-multimodal_amd", "tuned", "mi355x_b1024.json")
ENTRIES = json.load(open(TABLE))["entries"]


def _check(out, ref, bound, what):
    out = out.double().cpu()
    err = (out - ref).abs()
    tol = 64 * EPS32 * bound + 1e-30
    bad = err > tol
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements out of tolerance; max err {err.max().item():.3e}, " \
                                f"max ratio {(err / tol).max().item():.2f}"


def _operands(n, h, w, c, k, r, s, st, pad, seed):
    g = torch.Generator().manual_seed(seed)
    p, q = (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1
    x = torch.randn(n, c, h, w, generator=g)
    wt = torch.randn(k, c, r, s, generator=g) * (0.05 if c > 1 else 0.1)
    dy = torch.randn(n, k, p, q, generator=g)
    return x, wt, dy, p, q


def _id(e):
    return f"{e['kind']}-{'x'.join(map(str, e['shape']))}-{'.'.join(map(str, e['algo']))}"


@pytest.mark.parametrize("entry", ENTRIES, ids=_id)
def test_tuned_b1024_conv_vs_fp64(gpu, entry):
    kind, (n, h, w, c, k, r, s, st, pad), algo = entry["kind"], entry["shape"], entry["algo"]
    assert n == 1024
    x, wt, dy, p, q = _operands(n, h, w, c, k, r, s, st, pad, seed=sum(entry["shape"]) + len(algo))
    stem = c == 1
    what = f"{kind} {entry['shape']} {algo}"
    if kind == "fwd":
        out = conv_fwd(x.to(gpu), wt.to(gpu), st, pad, tuple(algo), nchw_input=stem)
        _check(out, F.conv2d(x.double(), wt.double(), None, st, pad), conv_bound(x, wt, st, pad), what)
        return
    if kind in ("wgrad", "bwd"):
        aw = tuple(algo[6:12]) if kind == "bwd" else tuple(algo)
        dw = conv_wgrad(x.to(gpu), dy.to(gpu), (r, s), st, pad, aw, nchw_input=stem)
        ref = torch.nn.grad.conv2d_weight(x.double(), (k, c, r, s), dy.double(), st, pad)
        bound = torch.nn.grad.conv2d_weight(x.double().abs(), (k, c, r, s), dy.double().abs(), st, pad)
        _check(dw, ref, bound, what + " (wgrad)")
    if kind in ("dgrad", "bwd"):
        ad = tuple(algo[:6])
        dx = conv_dgrad(dy.to(gpu), wt.to(gpu), (h, w), st, pad, ad)
        ref = torch.nn.grad.conv2d_input((n, c, h, w), wt.double(), dy.double(), st, pad)
        bound = torch.nn.grad.conv2d_input((n, c, h, w), wt.double().abs(), dy.double().abs(), st, pad)
        _check(dx, ref, bound, what + " (dgrad)")
    if kind == "bwd":  # the fused launch: bitwise the two separate launches (dw, dx above)
        lib, shp = L.lib(), shape(n, h, w, c, k, r, s, st, pad)
        ad, aw = L.ConvAlgo(*algo[:6]), L.ConvAlgo(*algo[6:12])
        xs = L.hwnc_strides(n, h, w, c)
        assert lib.tspm_conv_bwd_supported(ctypes.byref(shp), ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(xs))
        xd, dyd = to_hwnc(x).to(gpu), to_hwnc(dy).to(gpu)
        wd = wt.to(gpu).contiguous(memory_format=torch.channels_last)
        dx_f = torch.empty(h * w * n, c, device=gpu)
        dw_f = torch.empty(k, c, r, s, device=gpu).contiguous(memory_format=torch.channels_last)
        nd = lib.tspm_conv_dgrad_workspace(ctypes.byref(shp), ctypes.byref(ad))
        nw = lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(aw))
        wsd = torch.zeros(max(nd, 256), dtype=torch.uint8, device=gpu)
        wsw = torch.zeros(max(nw, 256), dtype=torch.uint8, device=gpu)
        L.check(lib.tspm_conv_bwd(ctypes.byref(shp), ctypes.byref(ad), ctypes.byref(aw), xd.data_ptr(), ctypes.byref(xs),
                                  dyd.data_ptr(), wd.data_ptr(), dx_f.data_ptr(), 0, dw_f.data_ptr(), wsd.data_ptr(),
                                  wsd.numel(), wsw.data_ptr(), wsw.numel(), L.stream_handle()), "conv_bwd")
        torch.cuda.synchronize()
        assert torch.equal(dx_f.view(h, w, n, c).permute(2, 3, 0, 1).cpu(), dx.cpu()), what
        assert torch.equal(dw_f.contiguous().cpu(), dw.cpu()), what
