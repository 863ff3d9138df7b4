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


class _FakeGroup:
    """A FusedAdam flat group's layout (offsets aligned to 4 floats) over CPU tensors: AdamCarry only reads
    offsets, numels and data pointers."""
    def __init__(self, params):
        self.params, self.offsets, off = params, [], 0
        for p in params:
            self.offsets.append(off)
            off += (p.numel() + 3) // 4 * 4
        self.numel = off
        self.param, self.grad, self.exp_avg, self.exp_avg_sq = (torch.zeros(off) for _ in range(4))
        self.hyper = torch.zeros(8, dtype=torch.float64)


class _FakeOpt:
    def __init__(self, params):
        self.g = _FakeGroup(params)

    def flat_groups(self):
        return [self.g]


def test_adam_carry_ranges_partition_the_encoder():
    """AdamCarry (step.py): blocks become ready in descending flat order; the carried jobs and rest_of() partition
    the encoder's range exactly once, every job starts 16-byte aligned, and a non-adjacent ready set is left to
    the optimizer's own launches."""
    from tspm_amd.step import AdamCarry
    torch.manual_seed(0)
    params = [torch.zeros(int(n)) for n in torch.randint(1, 3000, (13,))]  # stem .. fc, in flat order
    opt = _FakeOpt(params)
    c = AdamCarry(opt, max_blocks=7, elems_per_block=1000)
    blocks = [params[0:2], params[2:5], params[5:8], params[8:11], params[11:13]]  # last = "fc"
    base = opt.g.param.data_ptr()
    jobs = []
    c.ready(blocks[-1])
    for b in reversed(blocks[:-1]):
        for share in (0.5, 1.0):
            j = c.take(share)
            if j is not None:
                jobs.append(j)
                assert (j.param - base) % 16 == 0 and 1 <= j.blocks <= 7 and j.count > 0
        c.ready(b)
    c.ready([params[12]])  # already carried: not adjacent to what is pending -> ignored
    cover = torch.zeros(opt.g.numel, dtype=torch.int32)
    for a, b in c.carried:
        cover[a:b] += 1
    for a, b in c.rest_of([[(0, opt.g.numel)]])[0]:
        cover[a:b] += 1
    assert bool((cover == 1).all())
    assert sum(j.count for j in jobs) == sum(b - a for a, b in c.carried)
    # the first block (stem side) is never carried: nothing runs after it
    assert c.carried and min(a for a, _ in c.carried) >= opt.g.offsets[2]


def test_adam_carry_refuses_blocks_whose_spans_do_not_tile_their_range():
    """with a parameter order that interleaves another block's parameters into a block's
    [min, max) flat range, the block is not carried (the foreign elements' gradients may still be in flight); the
    contiguous blocks still are, and carried + rest still cover every element exactly once."""
    from tspm_amd.step import AdamCarry
    params = [torch.zeros(n) for n in (40, 24, 36, 52, 8, 16)]
    opt = _FakeOpt(params)
    c = AdamCarry(opt, max_blocks=4, elems_per_block=16)
    c.ready([params[0], params[2]])  # params[1] (another block's) sits between them
    assert c.lo is None and c.take(1.0) is None
    c.ready([params[4], params[5]])  # contiguous tail block
    assert (c.lo, c.hi) == (opt.g.offsets[4], opt.g.numel)
    c.ready([params[3], params[1]])  # not adjacent to each other: refused, pending range unchanged
    assert (c.lo, c.hi) == (opt.g.offsets[4], opt.g.numel)
    c.ready([params[3]])  # adjacent to the pending range: extends it
    assert c.lo == opt.g.offsets[3]
    j = c.take(1.0)
    assert j.count == opt.g.numel - opt.g.offsets[3]
    cover = torch.zeros(opt.g.numel, dtype=torch.int32)
    for a, b in c.carried:
        cover[a:b] += 1
    for a, b in c.rest_of([[(0, opt.g.numel)]])[0]:
        cover[a:b] += 1
    assert bool((cover == 1).all())
