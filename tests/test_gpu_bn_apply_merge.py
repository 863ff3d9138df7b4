"""tspm_bn_apply_merge (round 6): the forward BatchNorm apply with the per-tile statistics merge in its prologue
against tspm_bn_finalize + tspm_bn_apply on the same partial tiles.  The merge is the same double-precision
{K, mean - K, M2} combination in another fixed order, so save_mean / save_invstd / running statistics agree to
float rounding (rtol 2e-6) and the applied output to a few ulp of its scale; the partial tiles are built from
fp64 in the conv epilogue's format.  Shapes: the layers whose conv forward leaves its statistics to a merge launch
at batch 128 (ResNet34 layer1: 6,272 rows, 196 tiles; ResNet18 layer2: 6,144 rows, 192 tiles), odd tile counts,
and each residual mode."""
import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu


def _partials(y, rpt):
    M, C = y.shape
    G = -(-M // rpt)
    part = torch.empty(3, G, C, dtype=torch.float64)
    for g in range(G):
        t = y[g * rpt:(g + 1) * rpt].double()
        K = t[0]
        mu = t.mean(0)
        part[0, g], part[1, g], part[2, g] = K, mu - K, ((t - mu) ** 2).sum(0)
    return part.float().reshape(-1), G


@pytest.mark.parametrize("M,C,rpt", [(6272, 64, 32), (6144, 128, 32), (2048, 128, 64), (4000, 256, 32), (96, 16, 32)])
@pytest.mark.parametrize("res_mode", [0, 1, 2])
def test_apply_merge_equals_finalize_then_apply(gpu, M, C, rpt, res_mode):
    lib, sh = L.lib(), L.stream_handle()
    g = torch.Generator().manual_seed(M + C + res_mode)
    y = (torch.randn(M, C, generator=g) * 3 + torch.randn(1, C, generator=g) * 5)
    part, G = _partials(y, rpt)
    y, part = y.to(gpu), part.to(gpu)
    gamma, beta = (torch.rand(C, generator=g) + 0.5).to(gpu), torch.randn(C, generator=g).to(gpu)
    res = torch.randn(M, C, generator=g).to(gpu) if res_mode else None
    m2, i2 = torch.randn(C, generator=g).to(gpu), (torch.rand(C, generator=g) + 0.5).to(gpu)
    g2, b2 = (torch.rand(C, generator=g) + 0.5).to(gpu), torch.randn(C, generator=g).to(gpu)
    r2 = (m2, i2, g2, b2) if res_mode == 2 else (None, None, None, None)
    outs = []
    for merged in (False, True):
        rm, rv = torch.zeros(C, device=gpu) + 0.3, torch.ones(C, device=gpu) * 2
        mean, inv, out = torch.empty(C, device=gpu), torch.empty(C, device=gpu), torch.empty(M, C, device=gpu)
        if merged:
            L.check(lib.tspm_bn_apply_merge(M, C, G, rpt, part.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5,
                                            mean.data_ptr(), inv.data_ptr(), y.data_ptr(), gamma.data_ptr(),
                                            beta.data_ptr(), res_mode, L.ptr(res), *[L.ptr(t) for t in r2], 1,
                                            out.data_ptr(), sh), "bn_apply_merge")
        else:
            L.check(lib.tspm_bn_finalize(M, C, G, rpt, part.data_ptr(), rm.data_ptr(), rv.data_ptr(), 0.1, 1e-5,
                                         mean.data_ptr(), inv.data_ptr(), sh), "bn_finalize")
            L.check(lib.tspm_bn_apply(M, C, y.data_ptr(), mean.data_ptr(), inv.data_ptr(), gamma.data_ptr(),
                                      beta.data_ptr(), res_mode, L.ptr(res), *[L.ptr(t) for t in r2], 1, out.data_ptr(),
                                      None, 0, sh), "bn_apply")
        torch.cuda.synchronize()
        outs.append((mean.cpu(), inv.cpu(), rm.cpu(), rv.cpu(), out.cpu()))
    (ma, ia, rma, rva, oa), (mb, ib, rmb, rvb, ob) = outs
    scale = y.abs().max().item()
    assert torch.allclose(mb, ma, rtol=2e-6, atol=2e-7 * scale)
    assert torch.allclose(ib, ia, rtol=2e-6, atol=0)
    assert torch.allclose(rmb, rma, rtol=2e-6, atol=2e-7 * scale) and torch.allclose(rvb, rva, rtol=2e-6, atol=0)
    assert (ob - oa).abs().max().item() <= 1e-5 * (oa.abs().max().item() + 1)
    # and both against the fp64 statistics of y
    yd = y.double().cpu()
    assert torch.allclose(mb.double(), yd.mean(0), rtol=1e-6, atol=1e-6 * scale)
    assert torch.allclose(ib.double(), 1 / (yd.var(0, unbiased=False) + 1e-5).sqrt(), rtol=1e-5)
