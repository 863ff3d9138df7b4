"""tspm_conv_bwd_quad (round 6): a downsampling BasicBlock's second-conv backward and its 1x1 downsample's backward
in one launch — conv2's dx / dw (and the bn1 partial sums of dx) and the downsample's dx / dw bitwise those of two
tspm_conv_bwd_ex calls with the same algos, on the ResNet18 / ResNet34 downsampling blocks at batch 128."""
import ctypes

import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu

# (n, h, w, c, k): block input (h, w, c) and planes k; conv2 is k -> k 3x3 s1 on the (h/2, w/2) output
BLOCKS = [(128, 8, 24, 64, 128), (128, 4, 12, 128, 256), (128, 2, 6, 256, 512),
          (128, 7, 7, 64, 128), (128, 4, 4, 128, 256), (128, 2, 2, 256, 512)]
# (dgrad tm, tn, wn, wk), (wgrad tm, tn, wn, wk), conv2 (dgrad, wgrad) splits, downsample (dgrad, wgrad) splits
ALGOS = [((1, 1, 2, 2), (1, 1, 2, 1), (4, 1), (1, 1)), ((1, 1, 4, 1), (1, 1, 2, 1), (2, 3), (1, 3)),
         ((1, 1, 1, 4), (1, 1, 2, 2), (1, 6), (2, 6)), ((2, 1, 4, 1), (1, 1, 2, 1), (4, 1), (1, 2))]


def _shape(n, h, w, c, k, r, st, pad):
    return L.ConvShape(n, h, w, c, k, r, r, st, pad, (h + 2 * pad - r) // st + 1, (w + 2 * pad - r) // st + 1)


@pytest.mark.parametrize("blk", BLOCKS, ids=lambda b: "x".join(map(str, b)))
@pytest.mark.parametrize("alg", ALGOS, ids=str)
@pytest.mark.parametrize("with_bnp", [False, True])
def test_bwd_quad_bitwise_equals_two_launches(gpu, blk, alg, with_bnp):
    n, h, w, c, k = blk
    dcfg, wcfg, (sd1, sw1), (sd2, sw2) = alg
    lib, sh = L.lib(), L.stream_handle()
    ho, wo = (h + 1) // 2, (w + 1) // 2
    s2 = _shape(n, ho, wo, k, k, 3, 1, 1)      # conv2
    sd = _shape(n, h, w, c, k, 1, 2, 0)        # downsample
    ad, aw = L.ConvAlgo(*dcfg, sd1, 1), L.ConvAlgo(*wcfg, sw1, 1)
    qd, qw = L.ConvAlgo(*dcfg, sd2, 1), L.ConvAlgo(*wcfg, sw2, 1)
    xs2, xsd = L.hwnc_strides(n, ho, wo, k), L.hwnc_strides(n, h, w, c)
    if not lib.tspm_conv_bwd_quad_supported(ctypes.byref(s2), ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(xs2),
                                            ctypes.byref(sd), ctypes.byref(qd), ctypes.byref(qw), ctypes.byref(xsd)):
        pytest.skip("tile pair not built / does not fit")
    g = torch.Generator().manual_seed(n + h + c + k)
    M2 = n * ho * wo
    a1 = torch.randn(M2 * k, generator=g).to(gpu)           # conv2 input
    d2 = torch.randn(M2 * k, generator=g).to(gpu)           # conv2 output gradient
    w2 = (torch.randn(k * 9 * k, generator=g) * 0.05).to(gpu)
    xin = torch.randn(n * h * w * c, generator=g).to(gpu)   # block input
    dd = torch.randn(M2 * k, generator=g).to(gpu)           # downsample output gradient
    wd = (torch.randn(k * c, generator=g) * 0.05).to(gpu)
    out = torch.relu(torch.randn(M2 * k, generator=g)).to(gpu)
    y1 = torch.randn(M2 * k, generator=g).to(gpu)
    mean = y1.view(M2, k).mean(0)
    wsb = 1 << 26
    ws = [torch.zeros(wsb, dtype=torch.uint8, device=gpu) for _ in range(4)]
    res = []
    for quad in (False, True):
        da1 = torch.full((M2 * k,), float("nan"), device=gpu)
        gin = torch.full((n * h * w * c,), float("nan"), device=gpu)
        dw2 = torch.full((w2.numel(),), float("nan"), device=gpu)
        dwd = torch.full((wd.numel(),), float("nan"), device=gpu)
        part = torch.full((3 * (M2 // 32) * k,), float("nan"), device=gpu)
        bnp = L.BnBwdPart(out.data_ptr(), y1.data_ptr(), mean.data_ptr(), None, None, part.data_ptr())
        B = ctypes.byref(bnp) if with_bnp else None
        if quad:
            L.check(lib.tspm_conv_bwd_quad(
                ctypes.byref(s2), ctypes.byref(ad), ctypes.byref(aw), a1.data_ptr(), ctypes.byref(xs2), d2.data_ptr(),
                w2.data_ptr(), da1.data_ptr(), 0, dw2.data_ptr(), B, ws[0].data_ptr(), wsb, ws[1].data_ptr(), wsb,
                ctypes.byref(sd), ctypes.byref(qd), ctypes.byref(qw), xin.data_ptr(), ctypes.byref(xsd), dd.data_ptr(),
                wd.data_ptr(), gin.data_ptr(), dwd.data_ptr(), ws[2].data_ptr(), wsb, ws[3].data_ptr(), wsb, None, sh),
                "conv_bwd_quad")
        else:
            L.check(lib.tspm_conv_bwd_ex(ctypes.byref(s2), ctypes.byref(ad), ctypes.byref(aw), a1.data_ptr(),
                                         ctypes.byref(xs2), d2.data_ptr(), w2.data_ptr(), da1.data_ptr(), 0,
                                         dw2.data_ptr(), None, B, ws[0].data_ptr(), wsb, ws[1].data_ptr(), wsb, sh),
                    "conv_bwd_ex")
            L.check(lib.tspm_conv_bwd_ex(ctypes.byref(sd), ctypes.byref(qd), ctypes.byref(qw), xin.data_ptr(),
                                         ctypes.byref(xsd), dd.data_ptr(), wd.data_ptr(), gin.data_ptr(), 0,
                                         dwd.data_ptr(), None, None, ws[2].data_ptr(), wsb, ws[3].data_ptr(), wsb, sh),
                    "conv_bwd_ex")
        torch.cuda.synchronize()
        res.append([t.cpu() for t in (da1, gin, dw2, dwd)] + ([part.cpu()] if with_bnp else []))
    for a, b in zip(*res):  # (the third partial plane is unused without a second BN: NaN on both sides)
        assert bool(((a == b) | (torch.isnan(a) & torch.isnan(b))).all())
