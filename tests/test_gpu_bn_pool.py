"""tspm_bn_apply_pool (ABI 17): the encoder's last block apply with the adaptive average pool folded in.
Bitwise equal to tspm_bn_apply (or tspm_bn_apply_eval) followed by tspm_avgpool_fwd — the same arithmetic in
the same order — for every residual mode, with and without ReLU, train and eval statistics, 1-4 positions
(ResNet18 audio 1x3, ResNet34 image 1x1) and ragged channel / batch counts."""
import pytest
import torch

from tspm_amd import _lib as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("npos,n,c", [(3, 128, 512), (1, 128, 512), (4, 6, 68), (2, 1, 4)])
@pytest.mark.parametrize("res_mode", [0, 1, 2])
@pytest.mark.parametrize("relu", [0, 1])
@pytest.mark.parametrize("ev", [0, 1])
def test_bn_apply_pool_equals_apply_then_pool(gpu, npos, n, c, res_mode, relu, ev):
    lib = L.lib()
    g = torch.Generator(device="cpu").manual_seed(npos * 1000 + n + c + 7 * res_mode + relu)
    m = npos * n

    def r(*s, lo=None):
        t = torch.randn(*s, generator=g)
        return (t.abs() + 0.5 if lo else t).to(gpu)

    y, res = r(m, c), r(m, c)
    mean, var = r(c), r(c, lo=True)
    inv = var if ev else 1.0 / torch.sqrt(var + 1e-5)
    gamma, beta = r(c), r(c)
    mean2, var2, gamma2, beta2 = r(c), r(c, lo=True), r(c), r(c)
    inv2 = var2 if ev else 1.0 / torch.sqrt(var2 + 1e-5)
    p = lambda t: t.data_ptr()  # noqa: E731
    rs = p(res) if res_mode else None
    b2 = (p(mean2), p(inv2), p(gamma2), p(beta2)) if res_mode == 2 else (None, None, None, None)
    out_ref = torch.empty(m, c, device=gpu)
    pooled_ref = torch.empty(n, c, device=gpu)
    s = L.stream_handle()
    if ev:
        L.check(lib.tspm_bn_apply_eval(m, c, p(y), p(mean), p(inv), 1e-5, p(gamma), p(beta), res_mode, rs, *b2, relu,
                                       p(out_ref), s), "bn_apply_eval")
    else:
        L.check(lib.tspm_bn_apply(m, c, p(y), p(mean), p(inv), p(gamma), p(beta), res_mode, rs, *b2, relu,
                                  p(out_ref), None, 0, s), "bn_apply")
    L.check(lib.tspm_avgpool_fwd(npos, n, c, p(out_ref), p(pooled_ref), s), "avgpool_fwd")
    out = torch.full((m, c), float("nan"), device=gpu)
    pooled = torch.full((n, c), float("nan"), device=gpu)
    L.check(lib.tspm_bn_apply_pool(npos, n, c, p(y), p(mean), p(inv), p(gamma), p(beta), res_mode, rs, *b2, relu, ev,
                                   1e-5, p(out), p(pooled), s), "bn_apply_pool")
    torch.cuda.synchronize()
    assert torch.equal(out, out_ref)
    assert torch.equal(pooled, pooled_ref)


def test_bn_apply_pool_rejects_bad_arguments(gpu):
    lib = L.lib()
    x = torch.zeros(64, device=gpu)
    p = x.data_ptr()
    s = L.stream_handle()
    assert lib.tspm_bn_apply_pool(0, 4, 4, p, p, p, p, p, 0, None, None, None, None, None, 1, 0, 1e-5, p, p, s) != 0
    assert lib.tspm_bn_apply_pool(1, 4, 6, p, p, p, p, p, 0, None, None, None, None, None, 1, 0, 1e-5, p, p, s) != 0
    assert lib.tspm_bn_apply_pool(1, 4, 4, p, p, p, p, p, 1, None, None, None, None, None, 1, 0, 1e-5, p, p, s) != 0
    assert lib.tspm_bn_apply_pool(1, 4, 4, p, p, p, p, p, 0, None, None, None, None, None, 1, 0, 1e-5, p, None, s) != 0
