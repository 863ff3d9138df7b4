"""tspm_conv_bwd — the input and weight gradient of one convolution in ONE launch — against the two
separate launches (tspm_conv_dgrad + tspm_conv_wgrad, themselves bounded element-wise against fp64
in tests/test_gpu_ops.py): bitwise equal, for every built (dgrad, wgrad) tile pair, with and without
split-K on either side, beta 0 / 1, on the ResNet18 / ResNet34 backward shapes at batch 128."""
import ctypes
import itertools

import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu

DGRAD = [(1, 1, 2, 2), (1, 1, 4, 1), (1, 1, 1, 4)]          # (tm, tn, wn, wk): wm = 4 / (wn*wk)
WGRAD = [(1, 1, 2, 1), (1, 1, 1, 4), (1, 1, 2, 2), (1, 1, 1, 2)]
# (n, h, w, c, k, r, s, stride, pad): R34 layer1 / layer3 / layer4, R18 layer2 s2, 1x1 downsample
SHAPES = [(128, 7, 7, 64, 64, 3, 3, 1, 1), (128, 2, 2, 256, 256, 3, 3, 1, 1), (128, 1, 1, 512, 512, 3, 3, 1, 1),
          (128, 8, 24, 64, 128, 3, 3, 2, 1), (128, 4, 12, 128, 256, 1, 1, 2, 0)]


def _shape(n, h, w, c, k, r, s, st, pad):
    return L.ConvShape(n, h, w, c, k, r, s, st, pad, (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1)


@pytest.mark.parametrize("shp", SHAPES)
def test_fused_bwd_bitwise_equals_separate_launches(gpu, shp):
    lib = L.lib()
    s = _shape(*shp)
    g = torch.Generator().manual_seed(sum(shp))
    x = torch.randn(s.n * s.h * s.w * s.c, generator=g).to(gpu)
    dy = torch.randn(s.n * s.p * s.q * s.k, generator=g).to(gpu)
    w = (torch.randn(s.k * s.r * s.s * s.c, generator=g) * 0.05).to(gpu)
    dx0 = torch.randn(s.n * s.h * s.w * s.c, generator=g).to(gpu)
    xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
    sh = L.stream_handle()
    ran = 0
    for d, wg, (sd, sw), beta in itertools.product(DGRAD, WGRAD, [(1, 1), (2, 1), (1, 3)], (0, 1)):
        ad, aw = L.ConvAlgo(*d, sd, 1), L.ConvAlgo(*wg, sw, 1)
        if not lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(xs)):
            continue
        nd = lib.tspm_conv_dgrad_workspace(ctypes.byref(s), ctypes.byref(ad))
        nw = lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(aw))
        wsd = torch.zeros(max(nd, 256), dtype=torch.uint8, device=gpu)
        wsw = torch.zeros(max(nw, 256), dtype=torch.uint8, device=gpu)
        dx_a, dw_a = dx0.clone(), torch.full((w.numel(),), float("nan"), device=gpu)
        dx_b, dw_b = dx0.clone(), torch.full((w.numel(),), float("nan"), device=gpu)
        assert lib.tspm_conv_dgrad(ctypes.byref(s), ctypes.byref(ad), dy.data_ptr(), w.data_ptr(), dx_a.data_ptr(), beta,
                                   wsd.data_ptr(), wsd.numel(), sh) == 0
        assert lib.tspm_conv_wgrad(ctypes.byref(s), ctypes.byref(aw), x.data_ptr(), ctypes.byref(xs), dy.data_ptr(),
                                   dw_a.data_ptr(), wsw.data_ptr(), wsw.numel(), sh) == 0
        assert lib.tspm_conv_bwd(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), x.data_ptr(), ctypes.byref(xs),
                                 dy.data_ptr(), w.data_ptr(), dx_b.data_ptr(), beta, dw_b.data_ptr(), wsd.data_ptr(),
                                 wsd.numel(), wsw.data_ptr(), wsw.numel(), sh) == 0
        torch.cuda.synchronize()
        assert torch.equal(dx_a, dx_b), (d, wg, sd, sw, beta)
        assert torch.equal(dw_a, dw_b), (d, wg, sd, sw, beta)
        ran += 1
    assert ran > 0


def test_unbuilt_pair_is_refused(gpu):
    lib = L.lib()
    s = _shape(*SHAPES[0])
    xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
    ad, aw = L.ConvAlgo(2, 2, 1, 1, 1, 1), L.ConvAlgo(1, 1, 2, 1, 1, 1)  # tm = tn = 2 dgrad: not built fused
    assert lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(xs)) == 0
    assert lib.tspm_conv_bwd(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), 16, ctypes.byref(xs), 16, 16, 16, 0,
                             16, None, 0, None, 0, None) == 1
