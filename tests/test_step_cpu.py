"""Host-side routing of the fused train step (no GPU): the Python mirror of tspm_head_train_step's shape
limits sends a head the kernel would refuse to the autograd path instead of failing on the first
fused step."""
import torch

import tspm_amd
from tspm_amd.step import head_supported


def _model(hidden, ea=64, ei=128):
    return tspm_amd.AVMNIST(tspm_amd.ResNet18(1, ea), tspm_amd.ResNet34(1, ei), hidden, dropout=0.5)


def test_default_head_is_supported():
    assert head_supported(_model(128))  # the reference's 192 -> 128 -> 64 -> 10 head


def test_heads_outside_the_kernel_limits_are_not_routed_to_the_fused_step():
    assert not head_supported(_model(512))          # hidden > 256
    assert not head_supported(_model(130))          # hidden % 4 != 0 (and hidden // 2 = 65)
    assert not head_supported(_model(128, 200, 128))  # input 328 > 256


def test_fused_step_refuses_unsupported_head():
    class Opt(tspm_amd.FusedAdam):  # never constructed: fused_step_supported checks the type first
        pass
    m = _model(512)
    a, i = torch.zeros(2, 32, 94), torch.zeros(2, 1, 28, 28)
    from tspm_amd.step import fused_step_supported
    assert not fused_step_supported(m, object.__new__(Opt), None, a, i)
