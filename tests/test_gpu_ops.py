"""Per-kernel parity of libtspm (through the C ABI) against fp64 CPU references of the same op.

Tolerance for the MFMA convolutions (exact fp32 products, fp32 accumulation in a different order
than ATen): |y - y_ref| <= 64 * 2^-23 * sum|w||x| + 1e-30 per element (SURVEY.md §8(c) golden plan).
Memory-bound kernels (BN, pooling, Adam) are compared with rtol 1e-5 / atol scaled to the data.
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from abi_helpers import conv_bound, conv_dgrad, conv_fwd, conv_wgrad, from_hwnc, lds_supported, sh, to_hwnc

pytestmark = pytest.mark.gpu
EPS32 = 2.0 ** -23

CONV_CASES = [
    # n, c, h, w, k, r, s, stride, pad
    (2, 64, 8, 24, 64, 3, 3, 1, 1),      # mixed positions per wave (per-lane padding masks)
    (32, 64, 7, 7, 64, 3, 3, 1, 1),      # position-uniform waves (R34 layer1 shape)
    (64, 64, 8, 24, 128, 3, 3, 2, 1),    # stride 2 (R18 layer2 first conv)
    (32, 128, 4, 4, 256, 3, 3, 2, 1),
    (32, 256, 2, 2, 512, 1, 1, 2, 0),    # 1x1 s2 downsample
    (32, 512, 1, 1, 512, 3, 3, 1, 1),    # 1x1 spatial (R34 layer4): only the centre tap is valid
    (4, 128, 3, 5, 64, 3, 3, 2, 1),      # ragged, odd sizes, tiny batch
    (96, 64, 2, 6, 64, 3, 3, 1, 1),
    # exact ResNet18-audio / ResNet34-image layer shapes at the bench batch (128 per GPU)
    (128, 512, 1, 3, 512, 3, 3, 1, 1),
    (128, 256, 2, 6, 512, 3, 3, 2, 1),
    (128, 256, 2, 6, 512, 1, 1, 2, 0),
    (128, 256, 2, 6, 256, 3, 3, 1, 1),
    (128, 512, 1, 1, 512, 3, 3, 1, 1),
    (128, 256, 2, 2, 256, 3, 3, 1, 1),
    (128, 64, 7, 7, 64, 3, 3, 1, 1),
]
# (tm, tn, wn, wk, splits): tile shape, waves along N per workgroup, in-workgroup split-K, wgrad split
ALGOS = [(0, 0, 0, 0, 0), (1, 1, 1, 1, 1), (2, 2, 2, 2, 1), (1, 2, 1, 8, 1), (1, 1, 4, 2, 1), (1, 2, 2, 4, 1),
         (1, 1, 1, 16, 1), (1, 2, 1, 16, 1)]
# variant 1 (LDS-staged): (tm, tn, wn, wk, splits, 1) with wm = 4 / (wn*wk); every (wm, wn, wk) wave
# arrangement, both tile sizes and split-K over workgroups
# (the 2x2 wave tiles were removed in round 5: no tuned table selected them)
LDS_ALGOS = [(1, 1, 1, 1, 1, 1), (1, 1, 2, 1, 1, 1), (1, 1, 4, 1, 1, 1), (1, 1, 1, 4, 1, 1),
             (1, 2, 1, 2, 3, 1), (2, 1, 1, 4, 2, 1), (1, 1, 2, 2, 5, 1), (2, 1, 2, 1, 2, 1),
             # variant 2: the same kernels with single-role waves and an LDS-DMA ring (the batch-256 / 1024 tables)
             (1, 1, 2, 1, 1, 2), (2, 1, 1, 4, 2, 2), (1, 1, 2, 2, 5, 2), (1, 2, 1, 1, 2, 2),
             # variant 4: variant 1 with each fp32 product formed from exact bf16 pieces on the bf16 MFMA (round 6);
             # every plane layout (64-, 128-, 256- and 512-byte column rows) and both 16-deep step splits
             (1, 1, 1, 1, 1, 4), (1, 1, 2, 1, 1, 4), (1, 1, 4, 1, 1, 4), (1, 2, 1, 2, 3, 4), (1, 1, 2, 2, 5, 4),
             (2, 1, 2, 1, 2, 4), (2, 1, 1, 2, 2, 4), (2, 1, 1, 1, 1, 4)]


def _check(out, ref, bound, what):
    out = out.double().cpu()
    err = (out - ref).abs()
    tol = 64 * EPS32 * bound + 1e-30
    bad = err > tol
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements out of tolerance; max err {err.max().item():.3e}, " \
                                f"max ratio {(err / tol).max().item():.2f}"


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("algo", ALGOS + LDS_ALGOS)
def test_conv_fwd(gpu, case, algo):
    if not lds_supported("fwd", case, algo):
        pytest.skip("variant-1 tile does not fit this shape")
    n, c, h, w, k, r, s, st, pad = case
    g = torch.Generator().manual_seed(hash((case, algo)) % (2 ** 31))
    x = torch.randn(n, c, h, w, generator=g)
    wt = torch.randn(k, c, r, s, generator=g) * 0.05
    ref = F.conv2d(x.double(), wt.double(), None, st, pad)
    out = conv_fwd(x.to(gpu), wt.to(gpu), st, pad, algo)
    _check(out, ref, conv_bound(x, wt, st, pad), f"conv_fwd {case} {algo}")


@pytest.mark.parametrize("case", [(4, 1, 32, 94), (8, 1, 28, 28), (3, 1, 13, 9), (128, 1, 32, 94), (128, 1, 28, 28),
                                  (2, 1, 40, 500)])
@pytest.mark.parametrize("algo", [(0, 0, 0, 0, 0), (2, 2, 1, 1, 1), (1, 2, 2, 4, 1), (0, 0, 0, 0, 0, 3)])
def test_stem_fwd_nchw_input(gpu, case, algo):
    """7x7/2 stem reading the reference's NCHW input in place; spectrogram-like dynamic range."""
    n, c, h, w = case
    g = torch.Generator().manual_seed(7)
    x = 10.0 ** torch.empty(n, c, h, w).uniform_(-8, 7, generator=g)
    wt = torch.randn(64, c, 7, 7, generator=g) * 0.1
    ref = F.conv2d(x.double(), wt.double(), None, 2, 3)
    out = conv_fwd(x.to(gpu), wt.to(gpu), 2, 3, algo, nchw_input=True)
    _check(out, ref, conv_bound(x, wt, 2, 3), f"stem fwd {case} {algo}")


@pytest.mark.parametrize("case", [(128, 1, 32, 94), (128, 1, 28, 28), (5, 1, 13, 9), (1024, 1, 32, 94)])
@pytest.mark.parametrize("offset", [0.0, 3e4])
@pytest.mark.parametrize("fused", [True, False])
def test_stem_band_kernel_bn_statistics(gpu, case, offset, fused):
    """Variant 3 (stem.hip: one image x a band of output rows per workgroup): the per-band BN partials merged
    by tspm_bn_finalize (fused: inside tspm_conv_fwd; else by the caller with the queried tile count / rows)
    give the batch mean / invstd of its output, and the output matches the fp64 convolution."""
    from abi_helpers import conv_fwd_with_stats
    n, c, h, w = case
    g = torch.Generator().manual_seed(37)
    x = torch.randn(n, c, h, w, generator=g) + offset / 100
    wt = torch.randn(64, c, 7, 7, generator=g) * 0.1
    wt[:, :, 3, 3] += offset / 100
    y, mean, inv = conv_fwd_with_stats(x.to(gpu), wt.to(gpu), 2, 3, (0, 0, 0, 0, 0, 3), fused=fused)
    torch.cuda.synchronize()
    yd = y.double().cpu()
    ref = F.conv2d(x.double(), wt.double(), None, 2, 3)
    _check(y, ref, conv_bound(x, wt, 2, 3), f"stem band fwd {case}")
    mean_ref = yd.mean((0, 2, 3))
    var_ref = yd.var((0, 2, 3), unbiased=False)
    scale = yd.abs().amax((0, 2, 3)) + 1
    assert ((mean.double().cpu() - mean_ref).abs() <= 1e-6 * scale).all()
    assert torch.allclose(inv.double().cpu(), 1 / torch.sqrt(var_ref + 1e-5), rtol=1e-4)


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("algo", ALGOS[:4] + ALGOS[6:] + LDS_ALGOS)
@pytest.mark.parametrize("beta", [0, 1])
def test_conv_dgrad(gpu, case, algo, beta):
    if not lds_supported("dgrad", case, algo):
        pytest.skip("variant-1 tile does not fit this shape")
    n, c, h, w, k, r, s, st, pad = case
    g = torch.Generator().manual_seed(11)
    wt = torch.randn(k, c, r, s, generator=g) * 0.05
    p = (h + 2 * pad - r) // st + 1
    q = (w + 2 * pad - s) // st + 1
    dy = torch.randn(n, k, p, q, generator=g)
    init = torch.randn(n, c, h, w, generator=g) if beta else None
    ref = torch.nn.grad.conv2d_input((n, c, h, w), wt.double(), dy.double(), st, pad)
    bound = torch.nn.grad.conv2d_input((n, c, h, w), wt.double().abs(), dy.double().abs(), st, pad)
    if beta:
        ref = ref + init.double()
        bound = bound + init.double().abs()
    out = conv_dgrad(dy.to(gpu), wt.to(gpu), (h, w), st, pad, algo, init.to(gpu) if beta else None)
    _check(out, ref, bound, f"conv_dgrad {case} {algo} beta={beta}")


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("algo", ALGOS[:3] + [(1, 1, 1, 4, 7), (2, 2, 2, 2, 3), (1, 2, 4, 1, 16),
                                             (1, 1, 1, 16, 5), (1, 2, 1, 16, 2)] + LDS_ALGOS + [(1, 1, 1, 1, 16, 1)])
def test_conv_wgrad(gpu, case, algo):
    if not lds_supported("wgrad", case, algo):
        pytest.skip("variant-1 tile does not fit this shape")
    n, c, h, w, k, r, s, st, pad = case
    g = torch.Generator().manual_seed(13)
    x = torch.randn(n, c, h, w, generator=g)
    p = (h + 2 * pad - r) // st + 1
    q = (w + 2 * pad - s) // st + 1
    dy = torch.randn(n, k, p, q, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (k, c, r, s), dy.double(), st, pad)
    bound = torch.nn.grad.conv2d_weight(x.double().abs(), (k, c, r, s), dy.double().abs(), st, pad)
    out = conv_wgrad(x.to(gpu), dy.to(gpu), (r, s), st, pad, algo)
    _check(out, ref, bound, f"conv_wgrad {case} {algo}")


@pytest.mark.parametrize("case", [(4, 1, 32, 94), (8, 1, 28, 28), (16, 1, 28, 28), (128, 1, 32, 94), (128, 1, 28, 28),
                                  (3, 1, 13, 9)])
@pytest.mark.parametrize("algo", [(0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 3)])
def test_stem_wgrad_nchw_input(gpu, case, algo):
    n, c, h, w = case
    g = torch.Generator().manual_seed(17)
    x = 10.0 ** torch.empty(n, c, h, w).uniform_(-8, 7, generator=g)
    p, q = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
    dy = torch.randn(n, 64, p, q, generator=g) * 1e-6
    ref = torch.nn.grad.conv2d_weight(x.double(), (64, c, 7, 7), dy.double(), 2, 3)
    bound = torch.nn.grad.conv2d_weight(x.double().abs(), (64, c, 7, 7), dy.double().abs(), 2, 3)
    out = conv_wgrad(x.to(gpu), dy.to(gpu), (7, 7), 2, 3, algo, nchw_input=True)
    _check(out, ref, bound, f"stem wgrad {case} {algo}")


@pytest.mark.parametrize("case", [CONV_CASES[i] for i in (0, 1, 2, 5, 6, 8, 12)])
@pytest.mark.parametrize("algo", [(0, 0, 0, 0, 0), (2, 2, 2, 2, 1), (1, 1, 1, 8, 1), (1, 1, 1, 1, 1, 1),
                                  (2, 1, 1, 4, 2, 1), (1, 1, 2, 2, 5, 1)])
@pytest.mark.parametrize("offset", [0.0, 3e4])
@pytest.mark.parametrize("fused", [True, False])
def test_conv_fwd_epilogue_bn_statistics(gpu, case, algo, offset, fused):
    """BatchNorm batch statistics of the conv output from the conv epilogue's per-tile partials,
    merged in-launch (fused) or by tspm_bn_finalize."""
    from abi_helpers import conv_fwd_with_stats
    if not lds_supported("fwd", case, algo):
        pytest.skip("variant-1 tile does not fit this shape")
    n, c, h, w, k, r, s, st, pad = case
    g = torch.Generator().manual_seed(31)
    x = torch.randn(n, c, h, w, generator=g) + offset / 100
    wt = torch.randn(k, c, r, s, generator=g) * 0.05
    wt[:, :, r // 2, s // 2] += offset / (c * 100)  # push channel means far from zero
    y, mean, inv = conv_fwd_with_stats(x.to(gpu), wt.to(gpu), st, pad, algo, fused=fused)
    torch.cuda.synchronize()
    yd = y.double().cpu()
    mean_ref = yd.mean((0, 2, 3))
    var_ref = yd.var((0, 2, 3), unbiased=False)
    scale = yd.abs().amax((0, 2, 3)) + 1
    assert ((mean.double().cpu() - mean_ref).abs() <= 1e-6 * scale).all()
    assert torch.allclose(inv.double().cpu(), 1 / torch.sqrt(var_ref + 1e-5), rtol=1e-4)


# ------------------------------------------------------------------------------------------------
# BatchNorm
# ------------------------------------------------------------------------------------------------
def _bn_ws(lib, m, c, dev, bwd=False):
    b = (lib.tspm_bn_bwd_workspace if bwd else lib.tspm_bn_stats_workspace)(m, c)
    return torch.zeros(max(b, 16), dtype=torch.uint8, device=dev), b  # counter header starts zero


@pytest.mark.parametrize("m,c,offset", [(6272, 64, 0.0), (128, 512, 3.0), (96256, 64, 1e7), (4, 512, 0.5), (600, 128, -2e3)])
@pytest.mark.parametrize("nslab", [1, 3])
def test_bn_stats_and_apply(gpu, m, c, offset, nslab):
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(3)
    y = torch.randn(m, c, generator=g) * torch.rand(c, generator=g) * 5 + offset * torch.rand(c, generator=g)
    slabs = torch.stack([y / nslab] * nslab) if nslab > 1 else y[None]
    if nslab > 1:
        slabs[0] = y - (nslab - 1) * (y / nslab)
    ysum = slabs.double().sum(0)
    rm = torch.randn(c, generator=g)
    rv = torch.rand(c, generator=g) + 0.5
    gamma = torch.randn(c, generator=g)
    beta = torch.randn(c, generator=g)
    rm_ref, rv_ref = rm.double().clone(), rv.double().clone()
    ref = F.batch_norm(ysum, rm_ref, rv_ref, gamma.double(), beta.double(), True, 0.1, 1e-5)
    d_slabs = slabs.to(gpu).contiguous()
    y_out = torch.empty(m, c, device=gpu)
    d_rm, d_rv = rm.to(gpu), rv.to(gpu)
    mean = torch.empty(c, device=gpu)
    inv = torch.empty(c, device=gpu)
    ws, wsb = _bn_ws(lib, m, c, gpu)
    L.check(lib.tspm_bn_stats(m, c, d_slabs.data_ptr(), nslab, m * c, y_out.data_ptr(), d_rm.data_ptr(), d_rv.data_ptr(),
                              0.1, 1e-5, mean.data_ptr(), inv.data_ptr(), ws.data_ptr(), wsb, sh()), "bn_stats")
    src = y_out if nslab > 1 else d_slabs[0]
    out = torch.empty(m, c, device=gpu)
    d_gamma, d_beta = gamma.to(gpu), beta.to(gpu)  # keep alive: a freed temporary's block is reused at once
    L.check(lib.tspm_bn_apply(m, c, src.data_ptr(), mean.data_ptr(), inv.data_ptr(), d_gamma.data_ptr(),
                              d_beta.data_ptr(), 0, None, None, None, None, None, 0, out.data_ptr(), None, 0, sh()),
            "bn_apply")
    torch.cuda.synchronize()
    scale = ysum.abs().max(0).values + 1.0
    if nslab > 1:
        # the slab sum is fp32 (one rounding per add); statistics are checked on the summed tensor
        assert torch.allclose(y_out.double().cpu(), ysum, rtol=1e-6, atol=1e-6 * scale.max().item())
        ysum = y_out.double().cpu()
        rm_ref, rv_ref = rm.double().clone(), rv.double().clone()
        ref = F.batch_norm(ysum, rm_ref, rv_ref, gamma.double(), beta.double(), True, 0.1, 1e-5)
    mean_ref = ysum.mean(0)
    var_ref = ysum.var(0, unbiased=False)
    assert ((mean.double().cpu() - mean_ref).abs() <= 1e-6 + 4e-7 * scale).all()
    assert torch.allclose(inv.double().cpu(), 1 / torch.sqrt(var_ref + 1e-5), rtol=2e-5)
    assert ((d_rm.double().cpu() - rm_ref).abs() <= 1e-6 + 1e-7 * scale).all()
    assert torch.allclose(d_rv.double().cpu(), rv_ref, rtol=5e-5)
    # normalised output: error dominated by |y| * eps * invstd
    tol = 1e-4 + 4 * 2.0 ** -23 * scale * (1 / torch.sqrt(var_ref + 1e-5)) * gamma.double().abs()
    assert ((out.double().cpu() - ref).abs() <= tol).all()


def _bn_ref_block(y, y2, gamma, beta, gamma2, beta2, res, mode, relu):
    """fp64 autograd reference of out = act(bn(y) + residual) (batch statistics)."""
    y = y.double().requires_grad_(True)
    ga = gamma.double().requires_grad_(True)
    be = beta.double().requires_grad_(True)
    # NB: 2-D input.  ATen's CPU batch_norm backward returns wrong grads for the strided 4-D view
    # y.T[None, :, :, None] (channels-last-like strides) — found while building this test.
    z = F.batch_norm(y, None, None, ga, be, True, 0.0, 1e-5)
    extra = []
    if mode == 1:
        r = res.double().requires_grad_(True)
        z = z + r
        extra = [r]
    elif mode == 2:
        y2d = y2.double().requires_grad_(True)
        g2 = gamma2.double().requires_grad_(True)
        b2 = beta2.double().requires_grad_(True)
        z = z + F.batch_norm(y2d, None, None, g2, b2, True, 0.0, 1e-5)
        extra = [y2d, g2, b2]
    out = torch.relu(z) if relu else z
    return out, [y, ga, be] + extra


@pytest.mark.parametrize("m,c", [(6272, 64), (512, 256), (128, 512), (384, 512), (24576, 64), (1536, 256), (100, 8),
                                 (96256, 64)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_bn_block_fwd_bwd(gpu, m, c, mode):
    """BN apply + backward (the two-launch partial / apply pair) against float64 autograd."""
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(5)
    y = torch.randn(m, c, generator=g) * 3 + 1
    y2 = torch.randn(m, c, generator=g) * 2 - 1
    res = torch.randn(m, c, generator=g)
    gamma, beta = torch.randn(c, generator=g), torch.randn(c, generator=g)
    gamma2, beta2 = torch.randn(c, generator=g), torch.randn(c, generator=g)
    gout = torch.randn(m, c, generator=g)
    out_ref, leaves = _bn_ref_block(y, y2, gamma, beta, gamma2, beta2, res, mode, True)
    out_ref.backward(gout.double())

    def dev(t):
        return t.to(gpu).contiguous()

    dy_, dy2_, dres_ = dev(y), dev(y2), dev(res)
    means, invs = [], []
    for yy in (dy_, dy2_):
        mean, inv = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
        ws, wsb = _bn_ws(lib, m, c, gpu)
        L.check(lib.tspm_bn_stats(m, c, yy.data_ptr(), 1, 0, None, None, None, 0.1, 1e-5, mean.data_ptr(), inv.data_ptr(),
                                  ws.data_ptr(), wsb, sh()), "stats")
        means.append(mean); invs.append(inv)
    dg, db, dg2, db2 = dev(gamma), dev(beta), dev(gamma2), dev(beta2)
    out = torch.empty(m, c, device=gpu)
    r = dres_ if mode == 1 else (dy2_ if mode == 2 else None)
    L.check(lib.tspm_bn_apply(m, c, dy_.data_ptr(), means[0].data_ptr(), invs[0].data_ptr(), dg.data_ptr(), db.data_ptr(),
                              mode, L.ptr(r), means[1].data_ptr() if mode == 2 else None,
                              invs[1].data_ptr() if mode == 2 else None, dg2.data_ptr() if mode == 2 else None,
                              db2.data_ptr() if mode == 2 else None, 1, out.data_ptr(), None, 0, sh()), "apply")
    torch.cuda.synchronize()
    assert torch.allclose(out.double().cpu(), out_ref.detach(), rtol=1e-4, atol=1e-4)
    # backward
    gg = dev(gout)
    dyo = torch.empty(m, c, device=gpu)
    dy2o = torch.empty(m, c, device=gpu) if mode == 2 else None
    dreso = torch.empty(m, c, device=gpu) if mode == 1 else None
    gw, gb = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    gw2, gb2 = torch.empty(c, device=gpu), torch.empty(c, device=gpu)
    ws, wsb = _bn_ws(lib, m, c, gpu, bwd=True)
    two = mode == 2
    L.check(lib.tspm_bn_bwd(m, c, gg.data_ptr(), out.data_ptr(), dy_.data_ptr(), means[0].data_ptr(), invs[0].data_ptr(),
                            dg.data_ptr(), gw.data_ptr(), gb.data_ptr(), dyo.data_ptr(),
                            dy2_.data_ptr() if two else None, means[1].data_ptr() if two else None,
                            invs[1].data_ptr() if two else None, dg2.data_ptr() if two else None,
                            gw2.data_ptr() if two else None, gb2.data_ptr() if two else None,
                            L.ptr(dy2o), L.ptr(dreso), None, None, 0, ws.data_ptr(), wsb, sh()), "bn_bwd")
    torch.cuda.synchronize()
    yl, gal, bel = leaves[:3]
    assert torch.allclose(dyo.double().cpu(), yl.grad, rtol=1e-3, atol=2e-5)
    assert torch.allclose(gw.double().cpu(), gal.grad, rtol=1e-4, atol=1e-3)
    assert torch.allclose(gb.double().cpu(), bel.grad, rtol=1e-4, atol=1e-3)
    if mode == 1:
        assert torch.allclose(dreso.double().cpu(), leaves[3].grad, rtol=1e-6, atol=1e-6)
    if mode == 2:
        assert torch.allclose(dy2o.double().cpu(), leaves[3].grad, rtol=1e-3, atol=2e-5)
        assert torch.allclose(gw2.double().cpu(), leaves[4].grad, rtol=1e-4, atol=1e-3)
        assert torch.allclose(gb2.double().cpu(), leaves[5].grad, rtol=1e-4, atol=1e-3)


def test_bn_bwd_concurrent_streams(gpu):
    """Two BN backwards (partial-sum launch + apply launch each) in flight at once on two streams (as the
    two encoders' backward passes run), many times: workspaces do not alias, and the results equal the same
    launches run one after the other."""
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(11)
    shapes = [(24576, 64), (6272, 64)]  # the largest fused grids of the two encoders (192 + 196 rows blocks)
    bufs = []
    for m, c in shapes:
        y = (torch.randn(m, c, generator=g) * 2).to(gpu)
        out = torch.randn(m, c, generator=g).relu().to(gpu)
        gg = torch.randn(m, c, generator=g).to(gpu)
        mean, inv = y.mean(0).contiguous(), (1 / (y.var(0, unbiased=False) + 1e-5).sqrt()).contiguous()
        gamma = torch.randn(c, generator=g).to(gpu)
        ws, wsb = _bn_ws(lib, m, c, gpu, bwd=True)
        bufs.append(dict(m=m, c=c, y=y, out=out, g=gg, mean=mean, inv=inv, gamma=gamma, ws=ws, wsb=wsb,
                         dy=torch.empty(m, c, device=gpu), gw=torch.empty(c, device=gpu), gb=torch.empty(c, device=gpu)))

    def launch(b, stream):
        L.check(lib.tspm_bn_bwd(b["m"], b["c"], b["g"].data_ptr(), b["out"].data_ptr(), b["y"].data_ptr(),
                                b["mean"].data_ptr(), b["inv"].data_ptr(), b["gamma"].data_ptr(), b["gw"].data_ptr(),
                                b["gb"].data_ptr(), b["dy"].data_ptr(), None, None, None, None, None, None, None, None,
                                None, None, 0, b["ws"].data_ptr(), b["wsb"], stream.cuda_stream), "bn_bwd")
    s0 = torch.cuda.current_stream()
    for b in bufs:
        launch(b, s0)
    torch.cuda.synchronize()
    want = [(b["dy"].clone(), b["gw"].clone(), b["gb"].clone()) for b in bufs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(50):
        launch(bufs[0], s1)
        launch(bufs[1], s2)
    torch.cuda.synchronize()
    for b, (dy, gw, gb) in zip(bufs, want):
        assert torch.equal(b["dy"], dy) and torch.equal(b["gw"], gw) and torch.equal(b["gb"], gb)


# ------------------------------------------------------------------------------------------------
# pooling
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,c,h,w", [(4, 64, 16, 47), (32, 64, 14, 14), (3, 64, 5, 6)])
def test_maxpool(gpu, n, c, h, w):
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(9)
    x = torch.randn(n, c, h, w, generator=g)
    x = torch.relu(x)  # ties at 0 like post-ReLU activations
    xr = x.double().requires_grad_(True)
    ref = F.max_pool2d(xr, 3, 2, 1)
    gout = torch.randn(ref.shape, generator=g)
    ref.backward(gout.double())
    p, q = ref.shape[2], ref.shape[3]
    xd = to_hwnc(x.to(gpu))
    y = torch.empty(p * q * n, c, device=gpu)
    idx = torch.empty(p * q * n, c, dtype=torch.uint8, device=gpu)
    L.check(lib.tspm_maxpool_fwd(n, h, w, c, 3, 2, 1, p, q, xd.data_ptr(), y.data_ptr(), idx.data_ptr(), None, 0, sh()),
            "mp fwd")
    if (p * q * n) % 4 == 0:  # tiled variant with the transposed copy: same y / idx bitwise, y_t = y^T
        ld_t = p * q * n + 4
        y2, idx2 = torch.empty_like(y), torch.empty_like(idx)
        yt = torch.full((c, ld_t), 7.0, device=gpu)
        L.check(lib.tspm_maxpool_fwd(n, h, w, c, 3, 2, 1, p, q, xd.data_ptr(), y2.data_ptr(), idx2.data_ptr(),
                                     yt.data_ptr(), ld_t, sh()), "mp fwd_t")
        torch.cuda.synchronize()
        assert torch.equal(y2, y) and torch.equal(idx2, idx)
        assert torch.equal(yt[:, :p * q * n], y.view(p * q * n, c).t())
        assert bool((yt[:, p * q * n:] == 7.0).all())
    dx = torch.empty(h * w * n, c, device=gpu)
    gd = to_hwnc(gout.to(gpu))
    L.check(lib.tspm_maxpool_bwd(n, h, w, c, 3, 2, 1, p, q, gd.data_ptr(), idx.data_ptr(), dx.data_ptr(), sh()), "mp bwd")
    torch.cuda.synchronize()
    assert torch.equal(from_hwnc(y, n, p, q, c).cpu(), ref.detach().float())
    assert torch.allclose(from_hwnc(dx, n, h, w, c).double().cpu(), xr.grad, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("npos,n,c", [(3, 8, 512), (1, 16, 512), (4, 2, 64)])
def test_avgpool(gpu, npos, n, c):
    from tspm_amd import _lib as L
    lib = L.lib()
    x = torch.randn(npos * n, c)
    xd = x.to(gpu)
    y = torch.empty(n, c, device=gpu)
    L.check(lib.tspm_avgpool_fwd(npos, n, c, xd.data_ptr(), y.data_ptr(), sh()), "avg fwd")
    gy = torch.randn(n, c)
    gyd = gy.to(gpu)
    dx = torch.empty(npos * n, c, device=gpu)
    L.check(lib.tspm_avgpool_bwd(npos, n, c, gyd.data_ptr(), c, dx.data_ptr(), sh()), "avg bwd")
    torch.cuda.synchronize()
    assert torch.allclose(y.cpu(), x.view(npos, n, c).mean(0), rtol=1e-6, atol=1e-6)
    assert torch.allclose(dx.cpu(), (gy / npos).repeat(npos, 1), rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------------------------------------------
# linear / CE / Adam
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n,i,o", [(128, 512, 64), (4, 192, 128), (33, 64, 10), (128, 512, 128), (1000, 7, 3)])
def test_linear(gpu, n, i, o):
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(21)
    x, w, b = torch.randn(n, i, generator=g), torch.randn(o, i, generator=g) * 0.1, torch.randn(o, generator=g)
    keep = (torch.rand(n, o, generator=g) > 0.5).to(torch.uint8)
    xd, wd, bd, kd = x.to(gpu), w.to(gpu), b.to(gpu), keep.to(gpu)
    y = torch.empty(n, o, device=gpu)
    L.check(lib.tspm_linear_fwd(n, i, o, xd.data_ptr(), i, wd.data_ptr(), bd.data_ptr(), 1, kd.data_ptr(), 2.0,
                                y.data_ptr(), o, sh()), "lin fwd")
    ref = torch.relu(x.double() @ w.double().T + b.double()) * keep.double() * 2
    gy = torch.randn(n, o, generator=g)
    gyd = gy.to(gpu)
    dx = torch.empty(n, i, device=gpu)
    dw = torch.empty(o, i, device=gpu)
    db = torch.empty(o, device=gpu)
    L.check(lib.tspm_linear_bwd_data(n, i, o, gyd.data_ptr(), o, wd.data_ptr(), dx.data_ptr(), i, sh()), "lin dgrad")
    L.check(lib.tspm_linear_bwd_weight(n, i, o, xd.data_ptr(), i, gyd.data_ptr(), o, dw.data_ptr(), db.data_ptr(), sh()),
            "lin wgrad")
    g2 = gyd.clone()
    L.check(lib.tspm_act_bwd(n, o, g2.data_ptr(), o, y.data_ptr(), o, 2.0, sh()), "act bwd")
    torch.cuda.synchronize()
    assert torch.allclose(y.double().cpu(), ref, rtol=1e-5, atol=1e-4)
    assert torch.allclose(dx.double().cpu(), gy.double() @ w.double(), rtol=1e-5, atol=1e-4)
    assert torch.allclose(dw.double().cpu(), gy.double().T @ x.double(), rtol=1e-5, atol=1e-4)
    assert torch.allclose(db.double().cpu(), gy.double().sum(0), rtol=1e-5, atol=1e-4)
    assert torch.allclose(g2.double().cpu(), gy.double() * (ref > 0) * 2, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n", [4, 128, 1000])
def test_cross_entropy(gpu, n):
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(23)
    z = torch.randn(n, 10, generator=g) * 3
    lab = torch.randint(0, 10, (n,), generator=g)
    zr = z.double().requires_grad_(True)
    loss_ref = F.cross_entropy(zr, lab)
    loss_ref.backward()
    zd, ld = z.to(gpu), lab.to(gpu)
    loss = torch.zeros(1, device=gpu)
    dz = torch.empty(n, 10, device=gpu)
    stats = torch.zeros(4, device=gpu)
    L.check(lib.tspm_cross_entropy(n, 10, zd.data_ptr(), ld.data_ptr(), loss.data_ptr(), dz.data_ptr(), 1.0,
                                   stats.data_ptr(), sh()), "ce")
    torch.cuda.synchronize()
    assert abs(loss.item() - loss_ref.item()) < 1e-5 * max(1, abs(loss_ref.item()))
    assert torch.allclose(dz.double().cpu(), zr.grad, rtol=1e-5, atol=1e-7)
    assert stats[1].item() == float((z.argmax(1) == lab).sum())
    assert stats[2].item() == float(n)


def test_adam_matches_torch_adam(gpu):
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(29)
    n = 100003  # not a multiple of 4: exercises the tail
    p0 = torch.randn(n, generator=g)
    p_ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=5e-4, weight_decay=1e-4)
    pd = p0.to(gpu)
    gbuf = torch.empty(n, device=gpu)
    m = torch.zeros(n, device=gpu)
    v = torch.zeros(n, device=gpu)
    hyper = torch.tensor([5e-4, 0.9, 0.999, 1e-8, 1e-4, 1.0, 0.0, 0.0], dtype=torch.float64)
    hyper.view(torch.int64)[6] = 0
    hd = hyper.to(gpu)
    for step in range(5):
        grad = torch.randn(n, generator=g)
        p_ref.grad = grad.clone()
        opt.step()
        gbuf.copy_(grad)
        L.check(lib.tspm_adam_begin(hd.data_ptr(), sh()), "adam_begin")
        L.check(lib.tspm_adam_step(n, pd.data_ptr(), gbuf.data_ptr(), m.data_ptr(), v.data_ptr(), hd.data_ptr(), sh()),
                "adam")
    torch.cuda.synchronize()
    assert hd.view(torch.int64)[6].item() == 5
    assert torch.allclose(pd.cpu(), p_ref.detach(), rtol=1e-6, atol=1e-6)
    st = opt.state[p_ref]
    # a few ulp: torch's CPU lerp/addcmul vectorisation contracts differently
    assert torch.allclose(m.cpu(), st["exp_avg"], rtol=1e-6, atol=1e-8)
    assert torch.allclose(v.cpu(), st["exp_avg_sq"], rtol=1e-6, atol=1e-12)


def test_image_lut_and_dropout(gpu, lut):
    from tspm_amd import _lib as L
    lib = L.lib()
    u8 = torch.randint(0, 256, (7, 28, 28), dtype=torch.uint8)
    out = torch.empty(7, 28, 28, device=gpu)
    u8d, lutd = u8.to(gpu), lut.to(gpu)
    L.check(lib.tspm_image_lut(u8.numel(), u8d.data_ptr(), lutd.data_ptr(), out.data_ptr(), sh()), "lut")
    ref = lut[u8.long()].float() * (1.0 / 255.0)
    keep = torch.empty(1 << 20, dtype=torch.uint8, device=gpu)
    ctr = torch.tensor([3], dtype=torch.int64, device=gpu)
    L.check(lib.tspm_dropout_mask(keep.numel(), 0.5, 1234, ctr.data_ptr(), keep.data_ptr(), sh()), "mask")
    keep2 = torch.empty_like(keep)
    ctr2 = torch.tensor([4], dtype=torch.int64, device=gpu)
    L.check(lib.tspm_dropout_mask(keep.numel(), 0.5, 1234, ctr2.data_ptr(), keep2.data_ptr(), sh()), "mask2")
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref)
    frac = keep.float().mean().item()
    assert 0.49 < frac < 0.51
    assert (keep != keep2).float().mean().item() > 0.4


def test_linear_strided_rows(gpu):
    """The head reads/writes column slices of the [N,192] concat buffer: ldx/ldy > width."""
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(5)
    n, i, o, ldx, ldy = 96, 64, 40, 192, 200
    xb = torch.randn(n, ldx, generator=g)
    w = torch.randn(o, i, generator=g) * 0.1
    xd, wd = xb.to(gpu), w.to(gpu)
    y = torch.full((n, ldy), 7.0, device=gpu)
    L.check(lib.tspm_linear_fwd(n, i, o, xd[:, 64:].data_ptr(), ldx, wd.data_ptr(), None, 0, None, 1.0,
                                y.data_ptr(), ldy, sh()), "lin fwd")
    gy = torch.randn(n, ldy, generator=g)
    gyd = gy.to(gpu)
    dw = torch.empty(o, i, device=gpu)
    L.check(lib.tspm_linear_bwd_weight(n, i, o, xd[:, 64:].data_ptr(), ldx, gyd.data_ptr(), ldy, dw.data_ptr(), None,
                                       sh()), "lin wgrad")
    torch.cuda.synchronize()
    x = xb[:, 64:64 + i].double()
    assert torch.allclose(y[:, :o].double().cpu(), x @ w.double().T, rtol=1e-5, atol=1e-4)
    assert torch.equal(y[:, o:].cpu(), torch.full((n, ldy - o), 7.0))
    assert torch.allclose(dw.double().cpu(), gy[:, :o].double().T @ x, rtol=1e-5, atol=1e-4)


def test_fused_bn_counters_rearm_and_running_stats(gpu):
    """The in-launch merge leaves its counters zero (so one buffer serves every launch), repeated
    launches give identical statistics, and the running statistics follow nn.BatchNorm2d."""
    from abi_helpers import conv_fwd_with_stats, zeroed_counters
    g = torch.Generator().manual_seed(77)
    x = torch.randn(128, 64, 7, 7, generator=g).to(gpu)
    wt = (torch.randn(128, 64, 3, 3, generator=g) * 0.05).to(gpu)
    cnt = zeroed_counters(128, gpu)
    rm = torch.zeros(128, device=gpu)
    rv = torch.ones(128, device=gpu)
    outs = []
    for algo in [(1, 2, 1, 4, 1), (1, 2, 1, 4, 1), (2, 2, 2, 2, 1), (1, 1, 4, 1, 1)]:
        outs.append(conv_fwd_with_stats(x, wt, 2, 1, algo, fused=True, counters=cnt, running=(rm, rv)))
        torch.cuda.synchronize()
        assert int(cnt.abs().sum()) == 0
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])
    y = outs[0][0].double().cpu()
    mean_ref = y.mean((0, 2, 3))
    var_unb = y.var((0, 2, 3), unbiased=True)
    rm_ref, rv_ref = torch.zeros(128, dtype=torch.float64), torch.ones(128, dtype=torch.float64)
    for _ in range(4):
        rm_ref = 0.9 * rm_ref + 0.1 * mean_ref
        rv_ref = 0.9 * rv_ref + 0.1 * var_unb
    assert torch.allclose(rm.double().cpu(), rm_ref, rtol=1e-5, atol=1e-6)
    assert torch.allclose(rv.double().cpu(), rv_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("case,algo", [
    ((128, 64, 8, 24, 64, 3, 3, 1, 1), (2, 1, 1, 4, 1, 1)),    # 384 tiles, 64-channel blocks
    ((128, 64, 7, 7, 64, 3, 3, 1, 1), (1, 1, 2, 2, 1, 1)),     # 196 tiles: last group short
    ((128, 128, 4, 4, 128, 3, 3, 1, 1), (1, 1, 4, 1, 4, 1)),   # 128-channel blocks, split-K
    ((128, 32, 9, 11, 32, 3, 3, 1, 1), (1, 1, 1, 4, 1, 1)),    # 396 tiles: last group short, 32-channel blocks
])
@pytest.mark.parametrize("offset", [0.0, 3e4])
def test_conv_fwd_two_level_bn_merge(gpu, case, algo, offset):
    """Layers with too many row tiles for one merging workgroup: the two-level in-launch merge (no
    tspm_bn_finalize launch) gives the statistics of the finalize path to within float rounding of
    a double result, is deterministic, re-arms its counters and updates the running statistics."""
    from abi_helpers import conv_fwd_with_stats
    from tspm_amd import _lib as L
    n, c, h, w, k, r, s_, st, pad = case
    lib = L.lib()
    shp = L.ConvShape(n, h, w, c, k, r, s_, st, pad, (h + 2 * pad - r) // st + 1, (w + 2 * pad - s_) // st + 1)
    a = L.ConvAlgo(*algo)
    assert lib.tspm_conv_fwd_bn_counters(ctypes.byref(shp), ctypes.byref(a)) > (k + 31) // 32, "not a two-level case"
    g = torch.Generator().manual_seed(41)
    x = (torch.randn(n, c, h, w, generator=g) + offset / 100).to(gpu)
    wt = torch.randn(k, c, r, s_, generator=g) * 0.05
    wt[:, :, r // 2, s_ // 2] += offset / (c * 100)
    wt = wt.to(gpu)
    runs = []
    for two in (True, True, False):
        rm, rv = torch.zeros(k, device=gpu), torch.ones(k, device=gpu)
        y, mean, inv = conv_fwd_with_stats(x, wt, st, pad, algo, fused=True, running=(rm, rv), two_level=two)
        torch.cuda.synchronize()
        runs.append((y, mean, inv, rm, rv))
    for t1, t2 in zip(runs[0], runs[1]):
        assert torch.equal(t1, t2)
    yd = runs[0][0].double().cpu()
    mean_ref = yd.mean((0, 2, 3))
    var_ref = yd.var((0, 2, 3), unbiased=False)
    scale = yd.abs().amax((0, 2, 3)) + 1
    for y, mean, inv, rm, rv in (runs[0], runs[2]):
        assert ((mean.double().cpu() - mean_ref).abs() <= 1e-6 * scale).all()
        assert torch.allclose(inv.double().cpu(), 1 / torch.sqrt(var_ref + 1e-5), rtol=1e-4)
        assert torch.allclose(rv.double().cpu(), 0.9 + 0.1 * yd.var((0, 2, 3), unbiased=True), rtol=1e-5)
    # two-level vs finalize: both merge in double, so they agree to float rounding
    assert torch.allclose(runs[0][1], runs[2][1], rtol=2e-7, atol=1e-6 * float(scale.max()))
    assert torch.allclose(runs[0][2], runs[2][2], rtol=1e-6)


def test_wgrad_split_counters_rearm(gpu):
    """Split-K weight gradient with the in-launch slab reduction: repeated calls of different split
    counts through ONE zeroed workspace stay within the fp32 bound of the fp64 result (the last
    arriver of each tile re-arms its counter), and the counter header is zero afterwards."""
    import ctypes
    from abi_helpers import shape, sh, to_hwnc
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(128, 64, 7, 7, generator=g)
    dy = torch.randn(128, 64, 7, 7, generator=g)
    ref = torch.nn.grad.conv2d_weight(x.double(), (64, 64, 3, 3), dy.double(), 1, 1)
    bound = torch.nn.grad.conv2d_weight(x.double().abs(), (64, 64, 3, 3), dy.double().abs(), 1, 1)
    shp = shape(128, 7, 7, 64, 64, 3, 3, 1, 1)
    xd, dyd = to_hwnc(x.to(gpu)), to_hwnc(dy.to(gpu))
    st = L.hwnc_strides(128, 7, 7, 64)
    need = max(lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(L.ConvAlgo(1, 1, 1, 4, sp)))
               for sp in (2, 5, 16))
    ws = torch.zeros(need, dtype=torch.uint8, device=gpu)
    for sp in (2, 5, 16, 5, 2):
        dw = torch.empty(64, 64, 3, 3, device=gpu).contiguous(memory_format=torch.channels_last)
        a = L.ConvAlgo(1, 1, 1, 4, sp)
        L.check(lib.tspm_conv_wgrad(ctypes.byref(shp), ctypes.byref(a), xd.data_ptr(), ctypes.byref(st),
                                    dyd.data_ptr(), dw.data_ptr(), ws.data_ptr(), need, sh()), "wgrad")
        torch.cuda.synchronize()
        _check(dw.contiguous(), ref, bound, f"split {sp}")
        assert int(ws[:L.COUNTER_BYTES].int().sum()) == 0


@pytest.mark.parametrize("m,c", [(6272, 64), (512, 256), (128, 512), (96, 128)])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_bn_transposed_copies(gpu, m, c, mode):
    """The tiled kernels that also write transposed copies ([c][rows], per channel)
    give the same HWNC outputs as the plain kernels (forward bitwise; backward within 1e-6: the
    plain path merges its <= 64 partial tiles inside the apply kernel, the transposed path keeps the
    separate final pass over more tiles, so the per-channel sums are added in a different fixed
    order), and the copies are exact transposes."""
    from tspm_amd import _lib as L
    lib = L.lib()
    g = torch.Generator().manual_seed(8)
    t = lambda *sh_, s=1.0: (torch.randn(*sh_, generator=g) * s).to(gpu)  # noqa: E731
    y, y2, res, gout = t(m, c, s=3), t(m, c, s=2), t(m, c), t(m, c)
    mean, inv, gamma, beta = t(c), t(c).abs() + 0.5, t(c), t(c)
    mean2, inv2, gamma2, beta2 = t(c), t(c).abs() + 0.5, t(c), t(c)
    two = mode == 2
    r = res if mode == 1 else (y2 if two else None)
    ld_t = m + 8

    def apply(out, out_t):
        L.check(lib.tspm_bn_apply(m, c, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
                                  mode, L.ptr(r), mean2.data_ptr() if two else None, inv2.data_ptr() if two else None,
                                  gamma2.data_ptr() if two else None, beta2.data_ptr() if two else None, 1,
                                  out.data_ptr(), L.ptr(out_t), ld_t if out_t is not None else 0, sh()), "apply")

    o1, o2 = torch.empty(m, c, device=gpu), torch.empty(m, c, device=gpu)
    ot = torch.zeros(c, ld_t, device=gpu)
    apply(o1, None)
    apply(o2, ot)

    def bwd(dy, dy2, dres, dy_t, dy2_t):
        ws, wsb = _bn_ws(lib, m, c, gpu, bwd=True)
        gw, gb, gw2, gb2 = (torch.empty(c, device=gpu) for _ in range(4))
        L.check(lib.tspm_bn_bwd(m, c, gout.data_ptr(), o1.data_ptr(), y.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                gamma.data_ptr(), gw.data_ptr(), gb.data_ptr(), dy.data_ptr(),
                                y2.data_ptr() if two else None, mean2.data_ptr() if two else None,
                                inv2.data_ptr() if two else None, gamma2.data_ptr() if two else None,
                                gw2.data_ptr() if two else None, gb2.data_ptr() if two else None, L.ptr(dy2),
                                L.ptr(dres), L.ptr(dy_t), L.ptr(dy2_t), ld_t if dy_t is not None else 0, ws.data_ptr(),
                                wsb, sh()), "bn_bwd")

    mk = lambda: torch.empty(m, c, device=gpu)  # noqa: E731
    a = [mk(), mk() if two else None, mk() if mode == 1 else None]
    b = [mk(), mk() if two else None, mk() if mode == 1 else None]
    dyt = torch.zeros(c, ld_t, device=gpu)
    dy2t = torch.zeros(c, ld_t, device=gpu) if two else None
    bwd(*a, None, None)
    bwd(*b, dyt, dy2t)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.equal(ot[:, :m], o1.t())
    for u, v in zip(a, b):
        if u is not None:
            assert torch.allclose(u, v, rtol=1e-6, atol=1e-6 * float(v.abs().max()))
    assert torch.equal(dyt[:, :m], b[0].t())
    if two:
        assert torch.equal(dy2t[:, :m], b[1].t())


