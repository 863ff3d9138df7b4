"""tspm_conv_fwd_pair (round 6): a downsampling BasicBlock's first 3x3 conv and its 1x1 downsample (resnet.py:41,
50-51) in one launch — outputs, BN save_mean / save_invstd and running statistics bitwise those of two tspm_conv_fwd
calls with the same algos, for the ResNet18 / ResNet34 downsampling blocks at batch 128 (variant 1) and 1024
(variant 2), with and without split-K on either half and with the BN merge in-launch or by tspm_bn_finalize."""
import ctypes

import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu

# (n, h, w, c, k): block input and planes; conv1 3x3 s2 p1, downsample 1x1 s2 p0
BLOCKS = [(128, 8, 24, 64, 128), (128, 4, 12, 128, 256), (128, 2, 6, 256, 512),
          (128, 7, 7, 64, 128), (128, 4, 4, 128, 256), (128, 2, 2, 256, 512), (1024, 2, 2, 256, 512)]
# (tm, tn, wn, wk, variant), split of conv1, split of the downsample
ALGOS = [((1, 1, 2, 2, 1), 1, 1), ((1, 1, 2, 2, 1), 3, 1), ((1, 1, 1, 2, 1), 4, 2), ((2, 1, 2, 2, 1), 1, 1),
         ((1, 1, 1, 4, 1), 1, 1), ((1, 1, 2, 1, 2), 2, 1)]


def _shape(n, h, w, c, k, r, st, pad):
    return L.ConvShape(n, h, w, c, k, r, r, st, pad, (h + 2 * pad - r) // st + 1, (w + 2 * pad - r) // st + 1)


class _Half:
    def __init__(self, s, algo, gen, dev):
        self.s, self.a = s, algo
        self.w = (torch.randn(s.k * s.r * s.s * s.c, generator=gen) * 0.05).to(dev)
        lib = L.lib()
        self.wsb = max(lib.tspm_conv_fwd_workspace(ctypes.byref(s), ctypes.byref(algo)), 256)
        self.ws = torch.zeros(self.wsb, dtype=torch.uint8, device=dev)
        nfl = max(lib.tspm_conv_fwd_bn_partial_floats(ctypes.byref(s), ctypes.byref(algo)), 16)
        ncnt = max(lib.tspm_conv_fwd_bn_counters(ctypes.byref(s), ctypes.byref(algo)), 16)
        self.part = torch.empty(nfl, device=dev)
        self.cnt = torch.zeros(ncnt, dtype=torch.int32, device=dev)
        self.rm, self.rv = torch.zeros(s.k, device=dev), torch.ones(s.k, device=dev)
        self.mean, self.inv = torch.empty(s.k, device=dev), torch.empty(s.k, device=dev)
        self.y = torch.empty(s.p * s.q * s.n * s.k, device=dev)

    def bnf(self):
        return L.BnFuse(self.part.data_ptr(), self.cnt.data_ptr(), self.rm.data_ptr(), self.rv.data_ptr(), 0.1, 1e-5,
                        self.mean.data_ptr(), self.inv.data_ptr(), 0, 0, 0)

    def result(self):
        return torch.cat([self.y, self.mean, self.inv, self.rm, self.rv]).cpu()


@pytest.mark.parametrize("blk", BLOCKS, ids=lambda b: "x".join(map(str, b)))
@pytest.mark.parametrize("alg", ALGOS, ids=lambda a: f"{a[0]}-s{a[1]}-{a[2]}")
def test_fwd_pair_bitwise_equals_two_launches(gpu, blk, alg):
    n, h, w, c, k = blk
    (tm, tn, wn, wk, var), sp1, sp2 = alg
    if n == 1024:
        var = 2  # the batch-1024 tables' LDS-DMA build
    lib, sh = L.lib(), L.stream_handle()
    s1, s2 = _shape(n, h, w, c, k, 3, 2, 1), _shape(n, h, w, c, k, 1, 2, 0)
    a1, a2 = L.ConvAlgo(tm, tn, wn, wk, sp1, var), L.ConvAlgo(tm, tn, wn, wk, sp2, var)
    xs = L.hwnc_strides(n, h, w, c)
    if not lib.tspm_conv_fwd_pair_supported(ctypes.byref(s1), ctypes.byref(a1), ctypes.byref(xs), ctypes.byref(s2),
                                            ctypes.byref(a2), ctypes.byref(xs)):
        pytest.skip("tile does not fit this block")
    g = torch.Generator().manual_seed(n + h + c)
    x = torch.randn(n * h * w * c, generator=g).to(gpu)
    res = []
    for paired in (False, True):
        g2 = torch.Generator().manual_seed(5)
        h1, h2 = _Half(s1, a1, g2, gpu), _Half(s2, a2, g2, gpu)
        b1, b2 = h1.bnf(), h2.bnf()
        for _ in range(2):  # twice on the same buffers: counters left zero, running stats updated twice
            if paired:
                L.check(lib.tspm_conv_fwd_pair(ctypes.byref(s1), ctypes.byref(a1), x.data_ptr(), ctypes.byref(xs),
                                               h1.w.data_ptr(), h1.y.data_ptr(), ctypes.byref(b1), h1.ws.data_ptr(),
                                               h1.wsb, ctypes.byref(s2), ctypes.byref(a2), x.data_ptr(),
                                               ctypes.byref(xs), h2.w.data_ptr(), h2.y.data_ptr(), ctypes.byref(b2),
                                               h2.ws.data_ptr(), h2.wsb, sh), "conv_fwd_pair")
            else:
                for hh, ss, aa, bb in ((h1, s1, a1, b1), (h2, s2, a2, b2)):
                    L.check(lib.tspm_conv_fwd(ctypes.byref(ss), ctypes.byref(aa), x.data_ptr(), ctypes.byref(xs),
                                              hh.w.data_ptr(), hh.y.data_ptr(), ctypes.byref(bb), hh.ws.data_ptr(),
                                              hh.wsb, sh), "conv_fwd")
        torch.cuda.synchronize()
        res.append((h1.result(), h2.result()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])

