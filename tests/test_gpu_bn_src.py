"""tspm_bn_bwd_src (ABI 19): the BN backward with its incoming gradient formed on the fly from a pooling layer's
output gradient.  Bitwise equal to the pooling backward (tspm_avgpool_bwd / tspm_maxpool_bwd) followed by
tspm_bn_bwd — the same values in the same summation order — for the shapes the encoders use (the audio stem's
16 x 47 map into 8 x 24, the image stem's 14 x 14 into 7 x 7, the last blocks' 1 x 3 / 1 x 1 average pools),
with and without the ReLU mask, the identity-residual gradient and the downsample branch's second BN, plus
ragged batches; and argument checks."""
import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu


def _bufs(gpu, m, c, seed, two):
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = lambda *s: torch.randn(*s, generator=g).to(gpu)  # noqa: E731
    y, y2 = r(m, c) * 3, r(m, c)
    out = torch.relu(r(m, c))
    mean, inv, gamma = r(c), r(c).abs() + 0.5, r(c)
    mean2, inv2, gamma2 = r(c), r(c).abs() + 0.5, r(c)
    return dict(y=y, y2=y2 if two else None, out=out, mean=mean, inv=inv, gamma=gamma, mean2=mean2, inv2=inv2,
                gamma2=gamma2)


def _run(lib, gpu, m, c, b, two, relu, dres, g=None, src=None):
    p = L.ptr
    ws_b = lib.tspm_bn_bwd_workspace(m, c)
    ws = torch.zeros(ws_b, dtype=torch.uint8, device=gpu)
    outs = {k: torch.full((m, c), float("nan"), device=gpu) for k in ("dy", "dy2", "dres")}
    gr = {k: torch.full((c,), float("nan"), device=gpu) for k in ("gw", "gb", "gw2", "gb2")}
    args = [p(b["out"]) if relu else None, p(b["y"]), p(b["mean"]), p(b["inv"]), p(b["gamma"]), p(gr["gw"]),
            p(gr["gb"]), p(outs["dy"]), p(b["y2"]) if two else None, p(b["mean2"]) if two else None,
            p(b["inv2"]) if two else None, p(b["gamma2"]) if two else None, p(gr["gw2"]) if two else None,
            p(gr["gb2"]) if two else None, p(outs["dy2"]) if two else None, p(outs["dres"]) if dres else None]
    s = L.stream_handle()
    if src is None:
        L.check(lib.tspm_bn_bwd(m, c, p(g), *args, None, None, 0, ws.data_ptr(), ws_b, s), "bn_bwd")
    else:
        import ctypes
        L.check(lib.tspm_bn_bwd_src(m, c, ctypes.byref(src), *args, ws.data_ptr(), ws_b, s), "bn_bwd_src")
    torch.cuda.synchronize()
    res = {"dy": outs["dy"], "gw": gr["gw"], "gb": gr["gb"]}
    if two:
        res.update(dy2=outs["dy2"], gw2=gr["gw2"], gb2=gr["gb2"])
    if dres:
        res["dres"] = outs["dres"]
    return res


@pytest.mark.parametrize("n,h,w,c", [(128, 16, 47, 64), (128, 14, 14, 64), (5, 7, 9, 8), (3, 2, 3, 4)])
@pytest.mark.parametrize("relu", [True, False])
def test_maxpool_source_equals_maxpool_bwd_then_bn_bwd(gpu, n, h, w, c, relu):
    lib = L.lib()
    m = h * w * n
    p2, q2 = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    b = _bufs(gpu, m, c, n + h + w + c, False)
    # a real max-pool forward of the activation gives the argmax taps (ties and NaN rules included)
    x = torch.relu(torch.randn(m, c, generator=torch.Generator().manual_seed(3)).to(gpu)).round(decimals=1)
    pooled = torch.empty(p2 * q2 * n, c, device=gpu)
    idx = torch.empty(p2 * q2 * n, c, dtype=torch.uint8, device=gpu)
    s = L.stream_handle()
    L.check(lib.tspm_maxpool_fwd(n, h, w, c, 3, 2, 1, p2, q2, x.data_ptr(), pooled.data_ptr(), idx.data_ptr(), None,
                                 0, s), "maxpool_fwd")
    gp = torch.randn(p2 * q2 * n, c, generator=torch.Generator().manual_seed(4)).to(gpu)
    g = torch.empty(m, c, device=gpu)
    L.check(lib.tspm_maxpool_bwd(n, h, w, c, 3, 2, 1, p2, q2, gp.data_ptr(), idx.data_ptr(), g.data_ptr(), s),
            "maxpool_bwd")
    ref = _run(lib, gpu, m, c, b, False, relu, False, g=g)
    src = L.BnGSrc(kind=L.GSRC_MAXPOOL, n=n, h=h, w=w, p=p2, q=q2, npos=0, ldg=0, gp=gp.data_ptr(), idx=idx.data_ptr())
    got = _run(lib, gpu, m, c, b, False, relu, False, src=src)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k


@pytest.mark.parametrize("npos,n,c", [(3, 128, 512), (1, 128, 512), (2, 6, 68), (1, 1, 4)])
@pytest.mark.parametrize("two,dres", [(False, True), (True, False), (False, False)])
def test_avgpool_source_equals_avgpool_bwd_then_bn_bwd(gpu, npos, n, c, two, dres):
    lib = L.lib()
    m = npos * n
    b = _bufs(gpu, m, c, npos * 100 + n + c, two)
    ldg = c + 4
    gp = torch.randn(n, ldg, generator=torch.Generator().manual_seed(5)).to(gpu)
    g = torch.empty(m, c, device=gpu)
    L.check(lib.tspm_avgpool_bwd(npos, n, c, gp.data_ptr(), ldg, g.data_ptr(), L.stream_handle()), "avgpool_bwd")
    ref = _run(lib, gpu, m, c, b, two, True, dres, g=g)
    src = L.BnGSrc(kind=L.GSRC_AVGPOOL, n=n, h=1, w=npos, p=0, q=0, npos=npos, ldg=ldg, gp=gp.data_ptr(), idx=None)
    got = _run(lib, gpu, m, c, b, two, True, dres, src=src)
    for k in ref:
        assert torch.equal(got[k], ref[k]), k


def test_bn_bwd_src_rejects_bad_sources(gpu):
    import ctypes
    lib = L.lib()
    t = torch.zeros(1 << 16, device=gpu)
    p = t.data_ptr()
    ws = lib.tspm_bn_bwd_workspace(48, 4)
    w = torch.zeros(ws, dtype=torch.uint8, device=gpu)
    args = [None, p, p, p, p, p, p, p] + [None] * 8 + [w.data_ptr(), ws, L.stream_handle()]
    bad = [L.BnGSrc(kind=9, n=4, h=3, w=4, gp=p),                                    # unknown kind
           L.BnGSrc(kind=L.GSRC_AVGPOOL, n=4, h=3, w=3, npos=9, ldg=4, gp=p),        # rows != h * w * n
           L.BnGSrc(kind=L.GSRC_AVGPOOL, n=4, h=3, w=4, npos=5, ldg=4, gp=p),        # npos != h * w
           L.BnGSrc(kind=L.GSRC_MAXPOOL, n=4, h=3, w=4, p=1, q=2, gp=p, idx=p),      # wrong pooled map
           L.BnGSrc(kind=L.GSRC_MAXPOOL, n=4, h=3, w=4, p=2, q=2, gp=p, idx=None)]   # no argmax taps
    for src in bad:
        assert lib.tspm_bn_bwd_src(48, 4, ctypes.byref(src), *args) == 1


@pytest.mark.parametrize("n,h,w,c", [(128, 16, 47, 64), (128, 14, 14, 64), (5, 7, 9, 8), (3, 2, 3, 4), (2, 1, 1, 4)])
@pytest.mark.parametrize("ev", [0, 1])
def test_bn_apply_maxpool_equals_apply_then_maxpool(gpu, n, h, w, c, ev):
    """tspm_bn_apply_maxpool (ABI 19) == tspm_bn_apply[_eval] + tspm_maxpool_fwd, bitwise, NaN and ties included."""
    lib = L.lib()
    m = h * w * n
    p2, q2 = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    g = torch.Generator().manual_seed(n + h + w + c + ev)
    y = (torch.randn(m, c, generator=g) * 2).round(decimals=1)
    y[torch.rand(m, c, generator=g) < 0.01] = float("nan")
    y = y.to(gpu)
    mean = torch.randn(c, generator=g).to(gpu)
    inv = (torch.rand(c, generator=g) + 0.5).to(gpu)
    gamma, beta = torch.randn(c, generator=g).to(gpu), torch.randn(c, generator=g).to(gpu)
    s = L.stream_handle()
    a_ref = torch.empty(m, c, device=gpu)
    if ev:
        L.check(lib.tspm_bn_apply_eval(m, c, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), 1e-5, gamma.data_ptr(),
                                       beta.data_ptr(), 0, None, None, None, None, None, 1, a_ref.data_ptr(), s), "ev")
    else:
        L.check(lib.tspm_bn_apply(m, c, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                  beta.data_ptr(), 0, None, None, None, None, None, 1, a_ref.data_ptr(), None, 0, s), "ap")
    pr = torch.empty(p2 * q2 * n, c, device=gpu)
    ir = torch.empty(p2 * q2 * n, c, dtype=torch.uint8, device=gpu)
    L.check(lib.tspm_maxpool_fwd(n, h, w, c, 3, 2, 1, p2, q2, a_ref.data_ptr(), pr.data_ptr(), ir.data_ptr(), None, 0,
                                 s), "mp")
    a = torch.full((m, c), 7.0, device=gpu)
    pg = torch.full_like(pr, 7.0)
    ig = torch.full_like(ir, 99)
    L.check(lib.tspm_bn_apply_maxpool(n, h, w, c, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                      beta.data_ptr(), ev, 1e-5, a.data_ptr(), pg.data_ptr(), ig.data_ptr(), p2, q2, s),
            "fused")
    torch.cuda.synchronize()
    for got, ref in ((a, a_ref), (pg, pr)):
        assert torch.equal(got.view(torch.int32), ref.view(torch.int32))
    assert torch.equal(ig, ir)
    assert lib.tspm_bn_apply_maxpool(n, h, w, c, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                     beta.data_ptr(), ev, 1e-5, a.data_ptr(), pg.data_ptr(), ig.data_ptr(), p2 + 1, q2,
                                     s) == 1


def test_pool_fusions_leave_the_step_bitwise_unchanged(gpu, monkeypatch):
    """Four graph-replayed AVMNIST steps with the pooling fusions (TSPM_BN_POOL_SRC / TSPM_STEM_FUSE, the
    defaults) give bitwise the parameters, BN buffers and Adam moments of the step with the separate pooling
    launches.  The stem BN's partial sums formed in layer1's first dgrad epilogue (round 6, TSPM_BN_DGRAD_PART_STEM:
    a different summation order, held to fp64 per tile in tests/test_gpu_bn_dgrad_part.py) exist only with the pooling
    fold, so they are switched off in both runs: the comparison is of the pooling fusions alone.  (At batch 32 they
    became reachable once the batch-32 table put LDS-staged kernels on that dgrad, round 6.)"""
    import tspm_amd
    from oracle import avmnist_ref as orc
    results = []
    monkeypatch.setenv("TSPM_BN_DGRAD_PART_STEM", "0")
    for on in ("1", "0"):
        monkeypatch.setenv("TSPM_BN_POOL_SRC", on)
        monkeypatch.setenv("TSPM_STEM_FUSE", on)
        torch.manual_seed(11)
        ours = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(gpu)
        opt = tspm_amd.FusedAdam(ours.parameters(), lr=5e-4, weight_decay=1e-4)
        st = tspm_amd.FusedTrainStep(ours, opt, None, 32)
        for i in range(4):
            audio, image, labels, _ = orc.synthetic_batch(32, seed=90 + i)
            st.step(audio.to(gpu), image.to(gpu), labels.to(gpu))
        torch.cuda.synchronize()
        assert all(e.pool_src == (on == "1") and e.stem_fuse == (on == "1") for e in (st.eng_a, st.eng_i))
        bufs = [t.detach().reshape(-1) for m in ours.modules() if isinstance(m, torch.nn.BatchNorm2d)
                for t in (m.running_mean, m.running_var)]
        mom = [t for fg in opt.flat_groups() for t in (fg.exp_avg, fg.exp_avg_sq)]
        results.append(torch.cat([p.detach().reshape(-1) for p in ours.parameters()] + bufs + mom).cpu())
        st.close()
    assert torch.equal(results[0], results[1])
