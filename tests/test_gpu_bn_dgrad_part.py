"""The BatchNorm backward's partial sums formed in the dgrad epilogue (round 6: tspm_conv_bwd_ex with a
tspm_bn_bwd_part, consumed by tspm_bn_bwd_apply_part) against the two-launch BN backward.

* dx and dw of tspm_conv_bwd_ex are bitwise those of tspm_conv_bwd (the epilogue only adds the partial sums);
* the partial sums per 32-row tile and channel equal the fp64 sums of g' = dx * [out > 0] times 1 / (y - mean) /
  (y2 - mean2) within the fp32 rounding of a 32-term sum (8 * 2^-23 * sum |terms|);
* tspm_bn_bwd_apply_part over those partials gives tspm_bn_bwd's dy / dy2 / dres / dgamma / dbeta up to the
  reordered summation (dres bitwise: it is g' itself).
Shapes: the batch-128 ResNet34 / ResNet18 block convolutions (consuming BNs of 4 to 768 row tiles), with the
tuned fused-backward configurations, beta 0 (conv2 -> bn1) and 1 (conv1 onto the residual -> previous bn2)."""
import ctypes

import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu

# (n, h, w, c, k, r, s, stride, pad), (dgrad algo), (wgrad algo), beta, two
CASES = [
    ((128, 2, 2, 256, 256, 3, 3, 1, 1), (1, 1, 2, 2, 4, 1), (1, 1, 1, 2, 1, 1), 0, False),  # R34 layer3 conv2 -> bn1
    ((128, 2, 2, 256, 256, 3, 3, 1, 1), (1, 1, 2, 2, 4, 1), (1, 1, 1, 2, 1, 1), 1, False),  # ... conv1 -> bn2
    ((128, 1, 1, 512, 512, 3, 3, 1, 1), (1, 1, 1, 4, 1, 1), (1, 1, 2, 1, 1, 1), 1, False),  # R34 layer4
    ((128, 4, 4, 128, 256, 3, 3, 2, 1), (1, 1, 4, 1, 4, 1), (1, 1, 2, 1, 3, 1), 1, True),   # layer3 conv1 -> layer2 bn2+ds
    ((128, 4, 4, 128, 128, 3, 3, 1, 1), (1, 1, 4, 1, 2, 1), (1, 1, 2, 1, 3, 1), 0, False),  # R34 layer2 conv2 (64 tiles)
    ((128, 2, 6, 256, 256, 3, 3, 1, 1), (1, 1, 2, 2, 2, 1), (2, 1, 2, 1, 3, 1), 1, False),  # R18 layer3 conv1
    # more than 128 row tiles: the apply's merge prologue in several batches of 128
    ((128, 7, 7, 64, 64, 3, 3, 1, 1), (1, 1, 2, 2, 1, 1), (1, 1, 1, 2, 12, 1), 1, False),   # R34 layer1: 196 tiles
    ((128, 8, 24, 64, 64, 3, 3, 1, 1), (2, 1, 2, 1, 1, 1), (1, 1, 2, 1, 24, 1), 0, False),  # R18 layer1: 768 tiles
]


def _shape(n, h, w, c, k, r, s, st, pad):
    return L.ConvShape(n, h, w, c, k, r, s, st, pad, (h + 2 * pad - r) // st + 1, (w + 2 * pad - s) // st + 1)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-b{c[3]}-two{int(c[4])}")
def test_dgrad_epilogue_partials_and_apply(gpu, case):
    shp, dga, wga, beta, two = case
    lib, sh = L.lib(), L.stream_handle()
    s = _shape(*shp)
    M, C = s.n * s.h * s.w, s.c
    G = M // 32
    g = torch.Generator().manual_seed(sum(shp) + beta)
    x = torch.randn(M * C, generator=g).to(gpu)
    dy = torch.randn(s.n * s.p * s.q * s.k, generator=g).to(gpu)
    w = (torch.randn(s.k * s.r * s.s * C, generator=g) * 0.05).to(gpu)
    dx0 = torch.randn(M * C, generator=g).to(gpu)
    out = torch.relu(torch.randn(M, C, generator=g)).to(gpu)           # ReLU output: ~half the mask is zero
    y = (torch.randn(M, C, generator=g) * 2 + 0.5).to(gpu)
    y2 = (torch.randn(M, C, generator=g) * 3 - 1).to(gpu) if two else None
    mean = y.mean(0)
    mean2 = y2.mean(0) if two else None
    ad, aw = L.ConvAlgo(*dga), L.ConvAlgo(*wga)
    xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
    assert lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), ctypes.byref(xs))
    nd = lib.tspm_conv_dgrad_workspace(ctypes.byref(s), ctypes.byref(ad))
    nw = lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(aw))
    wsd = torch.zeros(max(nd, 256), dtype=torch.uint8, device=gpu)
    wsw = torch.zeros(max(nw, 256), dtype=torch.uint8, device=gpu)

    def run(bnp):
        dx = dx0.clone()
        dw = torch.full((w.numel(),), float("nan"), device=gpu)
        args = (ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), x.data_ptr(), ctypes.byref(xs), dy.data_ptr(),
                w.data_ptr(), dx.data_ptr(), beta, dw.data_ptr())
        if bnp is None:
            L.check(lib.tspm_conv_bwd(*args, wsd.data_ptr(), wsd.numel(), wsw.data_ptr(), wsw.numel(), sh), "conv_bwd")
        else:
            L.check(lib.tspm_conv_bwd_ex(*args, None, ctypes.byref(bnp), wsd.data_ptr(), wsd.numel(), wsw.data_ptr(),
                                         wsw.numel(), sh), "conv_bwd_ex")
        return dx, dw

    part = torch.full((3 * G * C,), float("nan"), device=gpu)
    bnp = L.BnBwdPart(out.data_ptr(), y.data_ptr(), mean.data_ptr(), L.ptr(y2), L.ptr(mean2), part.data_ptr())
    dx_ref, dw_ref = run(None)
    dx, dw = run(bnp)
    torch.cuda.synchronize()
    assert torch.equal(dx, dx_ref) and torch.equal(dw, dw_ref)

    # partial sums vs fp64
    gm = (dx.view(M, C).double() * (out > 0).double()).cpu()
    terms = [gm, gm * (y.double().cpu() - mean.double().cpu())]
    if two:
        terms.append(gm * (y2.double().cpu() - mean2.double().cpu()))
    pc = part.view(3, G, C).double().cpu()
    for k, t in enumerate(terms):
        ref = t.view(G, 32, C).sum(1)
        tol = 8 * 2.0 ** -23 * t.abs().view(G, 32, C).sum(1) + 1e-30
        assert bool(((pc[k] - ref).abs() <= tol).all()), f"plane {k}: max err {(pc[k] - ref).abs().max().item():.3e}"

    # the apply over those partials vs the two-launch BN backward on the same gradient
    gamma = (torch.rand(C, generator=g) + 0.5).to(gpu)
    inv = (1 / (y.var(0, unbiased=False) + 1e-5).sqrt()).contiguous()
    gamma2 = (torch.rand(C, generator=g) + 0.5).to(gpu) if two else None
    inv2 = (1 / (y2.var(0, unbiased=False) + 1e-5).sqrt()).contiguous() if two else None
    outs = []
    for mode in ("ref", "part"):
        o = dict(dy=torch.empty(M * C, device=gpu), dgamma=torch.empty(C, device=gpu), dbeta=torch.empty(C, device=gpu),
                 dy2=torch.empty(M * C, device=gpu) if two else None, dgamma2=torch.empty(C, device=gpu) if two else None,
                 dbeta2=torch.empty(C, device=gpu) if two else None,
                 dres=None if two else torch.empty(M * C, device=gpu))
        common = (y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(), o["dgamma"].data_ptr(),
                  o["dbeta"].data_ptr(), o["dy"].data_ptr(), L.ptr(y2), L.ptr(mean2), L.ptr(inv2), L.ptr(gamma2),
                  L.ptr(o["dgamma2"]), L.ptr(o["dbeta2"]), L.ptr(o["dy2"]), L.ptr(o["dres"]))
        if mode == "ref":
            ws_b = lib.tspm_bn_bwd_workspace(M, C)
            ws = torch.empty(ws_b, dtype=torch.uint8, device=gpu)
            L.check(lib.tspm_bn_bwd(M, C, dx.data_ptr(), out.data_ptr(), *common, None, None, 0, ws.data_ptr(), ws_b,
                                    sh), "bn_bwd")
        else:
            L.check(lib.tspm_bn_bwd_apply_part(M, C, G, part.data_ptr(), dx.data_ptr(), out.data_ptr(), *common, sh),
                    "bn_bwd_apply_part")
        outs.append(o)
    torch.cuda.synchronize()
    ref, got = outs
    for k in ("dy", "dgamma", "dbeta", "dy2", "dgamma2", "dbeta2"):
        if ref[k] is None:
            continue
        scale = ref[k].abs().max().item() + 1e-30
        err = (got[k] - ref[k]).abs().max().item()
        assert err <= 2e-5 * scale, f"{k}: max err {err:.3e} (scale {scale:.3e})"
    if ref["dres"] is not None:
        assert torch.equal(got["dres"], ref["dres"])



@pytest.mark.parametrize("stem_hw,algos", [((14, 14), ((1, 1, 2, 2, 1, 1), (1, 1, 1, 2, 12, 1))),    # ResNet34 image
                                           ((16, 47), ((2, 1, 2, 1, 1, 1), (1, 1, 2, 1, 24, 1)))])  # ResNet18 audio
def test_stem_partials_gathered_through_the_max_pool(gpu, stem_hw, algos):
    """Max-pool gather mode (tspm_bn_bwd_part.idx): layer1's first conv1 data gradient (the pool's output gradient,
    beta 1 onto the residual) forms the stem BN's partial sums at each pooled element's argmax; the stem BN backward
    from them (tspm_bn_bwd_apply_part_src) matches the two-launch tspm_bn_bwd_src (partial pass over the gathered
    gradient) up to the reordered sums, and dx is bitwise the plain launch's."""
    lib, sh = L.lib(), L.stream_handle()
    n, C = 128, 64
    H, W = stem_hw
    P, Q = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    s = _shape(n, P, Q, C, C, 3, 3, 1, 1)
    g = torch.Generator().manual_seed(H * W)
    y0 = (torch.randn(H * W * n, C, generator=g) * 2 + 0.3).to(gpu)
    mean = y0.mean(0).contiguous()
    inv = (1 / (y0.var(0, unbiased=False) + 1e-5).sqrt()).contiguous()
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(gpu), torch.randn(C, generator=g).to(gpu)
    a0 = torch.empty_like(y0)
    pooled = torch.empty(P * Q * n, C, device=gpu)
    idx = torch.empty(P * Q * n, C, dtype=torch.uint8, device=gpu)
    L.check(lib.tspm_bn_apply_maxpool(n, H, W, C, y0.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                      beta.data_ptr(), 0, 1e-5, a0.data_ptr(), pooled.data_ptr(), idx.data_ptr(), P, Q,
                                      sh), "bn_apply_maxpool")
    x = torch.randn(P * Q * n * C, generator=g).to(gpu)
    dy = torch.randn(P * Q * n * C, generator=g).to(gpu)
    w = (torch.randn(C * 9 * C, generator=g) * 0.05).to(gpu)
    dx0 = torch.randn(P * Q * n * C, generator=g).to(gpu)
    ad, aw = L.ConvAlgo(*algos[0]), L.ConvAlgo(*algos[1])
    xs = L.hwnc_strides(n, P, Q, C)
    ws = [torch.zeros(1 << 26, dtype=torch.uint8, device=gpu) for _ in range(2)]
    G = P * Q * n // 32
    part = torch.full((3 * G * C,), float("nan"), device=gpu)
    bnp = L.BnBwdPart(a0.data_ptr(), y0.data_ptr(), mean.data_ptr(), None, None, part.data_ptr(), idx.data_ptr(), H, W)
    dxs = []
    for B in (None, ctypes.byref(bnp)):
        dx = dx0.clone()
        dw = torch.empty(w.numel(), device=gpu)
        L.check(lib.tspm_conv_bwd_ex(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), x.data_ptr(), ctypes.byref(xs),
                                     dy.data_ptr(), w.data_ptr(), dx.data_ptr(), 1, dw.data_ptr(), None, B,
                                     ws[0].data_ptr(), ws[0].numel(), ws[1].data_ptr(), ws[1].numel(), sh), "conv_bwd_ex")
        dxs.append(dx)
    torch.cuda.synchronize()
    assert torch.equal(dxs[0], dxs[1])
    G_ = dxs[1]
    src = L.BnGSrc(kind=L.GSRC_MAXPOOL, n=n, h=H, w=W, p=P, q=Q, npos=0, ldg=0, gp=G_.data_ptr(), idx=idx.data_ptr())
    M = H * W * n
    res = []
    for mode in ("ref", "part"):
        dyo, dg, db = torch.empty(M * C, device=gpu), torch.empty(C, device=gpu), torch.empty(C, device=gpu)
        if mode == "ref":
            wsb = lib.tspm_bn_bwd_workspace(M, C)
            wsn = torch.empty(wsb, dtype=torch.uint8, device=gpu)
            L.check(lib.tspm_bn_bwd_src(M, C, ctypes.byref(src), a0.data_ptr(), y0.data_ptr(), mean.data_ptr(),
                                        inv.data_ptr(), gamma.data_ptr(), dg.data_ptr(), db.data_ptr(), dyo.data_ptr(),
                                        None, None, None, None, None, None, None, None, wsn.data_ptr(), wsb, sh), "bn_bwd_src")
        else:
            L.check(lib.tspm_bn_bwd_apply_part_src(M, C, G, part.data_ptr(), ctypes.byref(src), a0.data_ptr(),
                                                   y0.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                                   dg.data_ptr(), db.data_ptr(), dyo.data_ptr(), sh), "apply_part_src")
        res.append((dyo, dg, db))
    torch.cuda.synchronize()
    for a, b, k in zip(res[0], res[1], ("dy", "dgamma", "dbeta")):
        scale = a.abs().max().item() + 1e-30
        err = (b - a).abs().max().item()
        assert err <= 2e-5 * scale, f"{k}: max err {err:.3e} (scale {scale:.3e})"


# (block conv shape, dgrad algo, wgrad algo, beta, two, dres): layers of at most 512 rows (the whole-BN-backward mode)
WHOLE = [
    ((128, 2, 2, 256, 256, 3, 3, 1, 1), (1, 1, 2, 2, 4, 1), (1, 1, 1, 2, 1, 1), 0, False, False),  # R34 l3 conv2 -> bn1
    ((128, 2, 2, 256, 256, 3, 3, 1, 1), (1, 1, 2, 2, 4, 1), (1, 1, 1, 2, 1, 1), 1, False, True),   # l3 conv1 -> bn2 + dres
    ((128, 1, 1, 512, 512, 3, 3, 1, 1), (1, 1, 1, 4, 1, 1), (1, 1, 2, 1, 1, 1), 1, False, True),   # l4
    ((128, 2, 2, 256, 512, 3, 3, 2, 1), (1, 1, 1, 4, 1, 1), (1, 1, 2, 1, 1, 1), 1, True, False),   # l4 conv1 -> l3 bn2 + ds
    ((128, 1, 3, 512, 512, 3, 3, 1, 1), (1, 1, 2, 2, 4, 1), (1, 1, 2, 2, 1, 1), 0, False, False),  # R18 l4 (384 rows)
]


@pytest.mark.parametrize("case", WHOLE, ids=lambda c: f"{c[0]}-b{c[3]}-two{int(c[4])}-res{int(c[5])}")
def test_whole_bn_backward_in_the_dgrad_epilogue(gpu, case):
    """tspm_bn_bwd_part.dy (round 6): the last tile of each dgrad column block merges the partial tiles and applies
    the BN backward itself — dy / dy2 / dres / dgamma / dbeta equal tspm_bn_bwd_apply_part over the same partial sums
    (same merge order and expressions: bitwise), dx bitwise the plain launch's, the tickets left zero, over three
    back-to-back launches on the same buffers."""
    shp, dga, wga, beta, two, with_dres = case
    lib, sh = L.lib(), L.stream_handle()
    s = _shape(*shp)
    M, C = s.n * s.h * s.w, s.c
    G = M // 32
    g = torch.Generator().manual_seed(sum(shp) * 3 + beta)
    x = torch.randn(M * C, generator=g).to(gpu)
    dyin = torch.randn(s.n * s.p * s.q * s.k, generator=g).to(gpu)
    w = (torch.randn(s.k * s.r * s.s * C, generator=g) * 0.05).to(gpu)
    dx0 = torch.randn(M * C, generator=g).to(gpu)
    out = torch.relu(torch.randn(M, C, generator=g)).to(gpu)
    y = (torch.randn(M, C, generator=g) * 2 + 0.5).to(gpu)
    y2 = (torch.randn(M, C, generator=g) * 3 - 1).to(gpu) if two else None
    mean, mean2 = y.mean(0), (y2.mean(0) if two else None)
    inv = (1 / (y.var(0, unbiased=False) + 1e-5).sqrt()).contiguous()
    inv2 = (1 / (y2.var(0, unbiased=False) + 1e-5).sqrt()).contiguous() if two else None
    gamma = (torch.rand(C, generator=g) + 0.5).to(gpu)
    gamma2 = (torch.rand(C, generator=g) + 0.5).to(gpu) if two else None
    ad, aw = L.ConvAlgo(*dga), L.ConvAlgo(*wga)
    xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
    ws = [torch.zeros(1 << 26, dtype=torch.uint8, device=gpu) for _ in range(2)]
    cnt = torch.zeros(C // 32 + 1, dtype=torch.int32, device=gpu)

    def outs():
        return dict(dy=torch.full((M * C,), float("nan"), device=gpu), dg=torch.empty(C, device=gpu),
                    db=torch.empty(C, device=gpu), dy2=torch.full((M * C,), float("nan"), device=gpu) if two else None,
                    dg2=torch.empty(C, device=gpu) if two else None, db2=torch.empty(C, device=gpu) if two else None,
                    dres=torch.full((M * C,), float("nan"), device=gpu) if with_dres else None)

    res = []
    for whole in (False, True):
        for rep in range(3):
            o = outs()
            part = torch.full((3 * G * C,), float("nan"), device=gpu)
            bnp = L.BnBwdPart(out.data_ptr(), y.data_ptr(), mean.data_ptr(), L.ptr(y2), L.ptr(mean2), part.data_ptr())
            if whole:
                bnp.invstd, bnp.gamma, bnp.dgamma, bnp.dbeta = inv.data_ptr(), gamma.data_ptr(), o["dg"].data_ptr(), \
                    o["db"].data_ptr()
                bnp.dy, bnp.counters = o["dy"].data_ptr(), cnt.data_ptr()
                if two:
                    bnp.invstd2, bnp.gamma2, bnp.dgamma2, bnp.dbeta2, bnp.dy2 = (
                        inv2.data_ptr(), gamma2.data_ptr(), o["dg2"].data_ptr(), o["db2"].data_ptr(), o["dy2"].data_ptr())
                if with_dres:
                    bnp.dres = o["dres"].data_ptr()
            dx = dx0.clone()
            dw = torch.empty(w.numel(), device=gpu)
            L.check(lib.tspm_conv_bwd_ex(ctypes.byref(s), ctypes.byref(ad), ctypes.byref(aw), x.data_ptr(),
                                         ctypes.byref(xs), dyin.data_ptr(), w.data_ptr(), dx.data_ptr(), beta,
                                         dw.data_ptr(), None, ctypes.byref(bnp), ws[0].data_ptr(), ws[0].numel(),
                                         ws[1].data_ptr(), ws[1].numel(), sh), "conv_bwd_ex")
            if not whole:
                L.check(lib.tspm_bn_bwd_apply_part(
                    M, C, G, part.data_ptr(), dx.data_ptr(), out.data_ptr(), y.data_ptr(), mean.data_ptr(),
                    inv.data_ptr(), gamma.data_ptr(), o["dg"].data_ptr(), o["db"].data_ptr(), o["dy"].data_ptr(),
                    L.ptr(y2), L.ptr(mean2), L.ptr(inv2), L.ptr(gamma2), L.ptr(o["dg2"]), L.ptr(o["db2"]),
                    L.ptr(o["dy2"]), L.ptr(o["dres"]), sh), "bn_bwd_apply_part")
            torch.cuda.synchronize()
            res.append([dx.cpu(), dw.cpu()] + [v.cpu() for v in o.values() if v is not None])
    assert int(cnt.abs().sum()) == 0
    for r in res[1:]:
        for a, b in zip(res[0], r):
            assert torch.equal(a, b)
