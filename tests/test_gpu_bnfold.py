"""tspm_conv_fwd_bnin (ABI 15): BasicBlock's bn1 + ReLU applied by conv2's operand loader.

The fused launch must give BITWISE what tspm_bn_apply (bn1 + ReLU) followed by tspm_conv_fwd (conv2,
with its own BN statistics epilogue) gives: the conv output, the activation it writes for the backward
(every element exactly once — the buffer is pre-filled with NaN), and the statistics of the conv output.
Covers split-K (the centre-tap stages of a row block in one slice), several output-channel blocks (only
the first writes), 1x1 / 2x2 / 4x4 / 8x24 maps (border positions skip taps) and channels that ReLU zeroes.
"""
import ctypes

import pytest
import torch

from abi_helpers import lds_supported, sh
from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu

CASES = [(32, 4, 4, 64, 64), (128, 2, 2, 256, 256), (128, 1, 1, 512, 512), (64, 8, 24, 64, 64), (32, 7, 7, 128, 128)]
ALGOS = [(1, 1, 1, 4, 1, 1), (2, 1, 1, 4, 2, 1), (1, 1, 2, 2, 5, 1), (1, 2, 2, 2, 1, 1), (2, 2, 1, 1, 3, 1),
         (1, 1, 4, 1, 4, 1)]


def _fwd(lib, shp, algo, x, w, bi, dev):
    k = shp.k
    m = shp.p * shp.q * shp.n
    y = torch.empty(m, k, device=dev)
    tiles = lib.tspm_conv_fwd_tiles(ctypes.byref(shp), ctypes.byref(algo))
    part = torch.empty(3 * tiles * k, device=dev)
    cnt = torch.zeros(k // 32 + 1, dtype=torch.int32, device=dev)
    mean, inv = torch.empty(k, device=dev), torch.empty(k, device=dev)
    rm, rv = torch.zeros(k, device=dev), torch.ones(k, device=dev)
    bnf = L.BnFuse(part.data_ptr(), cnt.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5, mean.data_ptr(),
                   inv.data_ptr(), 0, 0, 0)
    wsb = lib.tspm_conv_fwd_workspace(ctypes.byref(shp), ctypes.byref(algo))
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    st = L.hwnc_strides(shp.n, shp.h, shp.w, shp.c)
    if bi is None:
        L.check(lib.tspm_conv_fwd(ctypes.byref(shp), ctypes.byref(algo), x.data_ptr(), ctypes.byref(st), w.data_ptr(),
                                  y.data_ptr(), ctypes.byref(bnf), ws.data_ptr(), wsb, sh()), "conv_fwd")
    else:
        L.check(lib.tspm_conv_fwd_bnin(ctypes.byref(shp), ctypes.byref(algo), x.data_ptr(), ctypes.byref(st),
                                       w.data_ptr(), y.data_ptr(), ctypes.byref(bnf), ctypes.byref(bi), ws.data_ptr(),
                                       wsb, sh()), "conv_fwd_bnin")
    return y, mean, inv, rm, rv


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("algo", ALGOS)
def test_conv_fwd_bnin_equals_apply_then_conv(gpu, case, algo):
    n, h, w, c, k = case
    if not lds_supported("fwd", (n, c, h, w, k, 3, 3, 1, 1), algo):
        pytest.skip("variant-1 tile does not fit this shape")
    lib = L.lib()
    g = torch.Generator().manual_seed(7 + n + c)
    m = h * w * n
    y1 = (torch.randn(m, c, generator=g) * 3 + torch.randn(c, generator=g)).to(gpu)  # conv1 output (pre-BN)
    mean = y1.double().mean(0).float()
    inv = (1.0 / torch.sqrt(y1.double().var(0, unbiased=False) + 1e-5)).float()
    gamma = torch.randn(c, generator=g).to(gpu)
    gamma[::7] = -gamma[::7].abs()  # channels the ReLU mostly zeroes
    beta = (torch.randn(c, generator=g) * 0.5).to(gpu)
    wt = (torch.randn(k, c, 3, 3, generator=g) * 0.05).to(gpu).contiguous(memory_format=torch.channels_last)
    shp = L.ConvShape(n, h, w, c, k, 3, 3, 1, 1, h, w)
    a = L.ConvAlgo(*algo)
    # reference: tspm_bn_apply (bn1 + ReLU) then the plain conv
    a1 = torch.empty(m, c, device=gpu)
    L.check(lib.tspm_bn_apply(m, c, y1.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                              0, None, None, None, None, None, 1, a1.data_ptr(), None, 0, sh()), "bn_apply")
    ref = _fwd(lib, shp, a, a1, wt, None, gpu)
    # fused
    a_out = torch.full((m, c), float("nan"), device=gpu)
    bi = L.BnInput(mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(), beta.data_ptr(), a_out.data_ptr())
    got = _fwd(lib, shp, a, y1, wt, bi, gpu)
    torch.cuda.synchronize()
    assert torch.equal(a_out, a1), (a_out != a1).sum().item()
    for name, r, o in zip(("y", "mean", "invstd", "running_mean", "running_var"), ref, got):
        assert torch.equal(r, o), (name, (r - o).abs().max().item())


def test_conv_fwd_bnin_refuses_unsupported(gpu):
    lib = L.lib()
    shp = L.ConvShape(32, 4, 4, 64, 64, 3, 3, 2, 1, 2, 2)  # stride 2: no centre-tap writer for odd positions
    a = L.ConvAlgo(1, 1, 1, 4, 1, 1)
    t = torch.zeros(16 * 32 * 64, device=gpu)
    bi = L.BnInput(t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr())
    st = L.hwnc_strides(32, 4, 4, 64)
    rc = lib.tspm_conv_fwd_bnin(ctypes.byref(shp), ctypes.byref(a), t.data_ptr(), ctypes.byref(st), t.data_ptr(),
                                t.data_ptr(), None, ctypes.byref(bi), None, 0, sh())
    assert rc != 0
    a0 = L.ConvAlgo(0, 0, 0, 0, 0, 0)  # register-direct variant
    shp1 = L.ConvShape(32, 4, 4, 64, 64, 3, 3, 1, 1, 4, 4)
    rc = lib.tspm_conv_fwd_bnin(ctypes.byref(shp1), ctypes.byref(a0), t.data_ptr(), ctypes.byref(st), t.data_ptr(),
                                t.data_ptr(), None, ctypes.byref(bi), None, 0, sh())
    assert rc != 0
