"""FusedTrainStep — the whole AVMNIST late-fusion train step as one HIP-graph replay.

Replaces the per-batch body of MML_Suite/models/avmnist.py:269-310 (zero_grad → forward →
LossFunctionGroup(CE) → backward → Adam.step) and the backward/optimizer loop of
train_multimodal.py:469-488:

    s0: audio ResNet18 fwd ─┐            ┌─ audio ResNet18 bwd ─┐
    s1: image ResNet34 fwd ─┴─ head fwd ─ CE ─ head bwd ─┴─ image ResNet34 bwd ─┴─ [RCCL] ─ Adam

The two encoders are independent until the fusion concat, so they run as parallel graph branches
on two HIP streams.  Every buffer is allocated once; the first call runs eagerly, the second call
captures the graph, later calls only copy the batch into the static input buffers and replay.
Weight gradients are written straight into FusedAdam's flat gradient buffer (overwrite — no
zero_grad pass); with world_size > 1 the flat buffer is all-reduced between backward and Adam
(``ddp.GradAllReduce``) and 1/world is folded into Adam's gradient scale.
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib as L
from .engine import EncoderEngine, prepare_encoder_layout
from .ddp import PhasedGradAllReduce
from .optim import FusedAdam

NUM_CLASSES = 10


def _ce_weight(loss_functions) -> Optional[float]:
    """Weight of the single cross-entropy term of a LossFunctionGroup (experiment_utils/loss.py:83-148),
    or None when the group is anything else (then the step follows the generic autograd path)."""
    if loss_functions is None:
        return 1.0
    try:
        items = list(loss_functions.items())
    except AttributeError:
        return None
    if len(items) != 1:
        return None
    term = items[0][1]
    fn = getattr(term, "loss_fn", None)
    w = getattr(term, "weight", 1.0)
    if not isinstance(fn, torch.nn.CrossEntropyLoss):
        return None
    if fn.weight is not None or fn.reduction != "mean" or fn.label_smoothing != 0.0:
        return None
    return float(w)


def shared_batches_tracked(model: torch.nn.Module, dev: torch.device,
                           types=(torch.nn.BatchNorm2d,)) -> torch.Tensor:
    """The ``num_batches_tracked`` counters of every BatchNorm2d of ``model`` re-pointed as views of ONE
    int64 device buffer (one add per step instead of one per BN), shared by every fused step of the
    model (e.g. a second one for a partial last batch)."""
    bns = [m for m in model.modules() if isinstance(m, types) and m.num_batches_tracked is not None]
    nbt = getattr(model, "_tspm_nbt", None)
    if not (nbt is not None and nbt.numel() == len(bns) and nbt.device == dev and all(
            m.num_batches_tracked.data_ptr() == nbt[i].data_ptr() for i, m in enumerate(bns))):
        nbt = torch.zeros(len(bns), dtype=torch.int64, device=dev)
        for i, m in enumerate(bns):
            nbt[i] = m.num_batches_tracked.to(dev)
            m.num_batches_tracked = nbt[i]
        model._tspm_nbt = nbt
    return nbt


# tspm_head_train_step's shape limits (csrc/misc.hip: HEAD_MAXIN / HEAD_MAXH / HEAD_MAXH2 / HEAD_MAXC, sizes % 4,
# weights + the 4-row block in at most 160 KiB of LDS — head_lds_floats)
HEAD_MAX_IN, HEAD_MAX_HIDDEN, HEAD_MAX_HIDDEN2, HEAD_MAX_CLASSES = 256, 256, 128, 16


def head_supported(model) -> bool:
    """Python mirror of tspm_head_train_step's argument checks for this model's fusion head: a
    head the kernel would refuse routes AVMNIST.train_step to the autograd path (linear kernels + CE) instead
    of raising on the first fused step."""
    try:
        F = int(model.embd_size_A) + int(model.embd_size_I)
        H = int(model.hidden_dim)
        H2 = H // 2
    except (AttributeError, TypeError):
        return False
    C = NUM_CLASSES
    if not (0 < F <= HEAD_MAX_IN and 0 < H <= HEAD_MAX_HIDDEN and 0 < H2 <= HEAD_MAX_HIDDEN2 and 0 < C <= HEAD_MAX_CLASSES):
        return False
    if F % 4 or H % 4 or H2 % 4:
        return False
    rb = 4  # the larger of the kernel's row blocks (tspm_head_desc.rows_per_block = 4; the default is 1 up to 256 rows)
    ldc = ((C + 3) & ~3) + 4
    floats = H * (F + 4) + H2 * (H + 4) + C * (H2 + 4) + rb * ((F + 4) + (H + 4) + (H2 + 4) + ldc) + (H + H2 + C + rb)
    return floats * 4 <= 160 * 1024


def fused_step_supported(model, optimizer, loss_functions, A: torch.Tensor, I: torch.Tensor) -> bool:
    if os.environ.get("TSPM_DISABLE_FUSED_STEP"):
        return False
    if not isinstance(optimizer, FusedAdam):
        return False
    if _ce_weight(loss_functions) is None:
        return False
    if not (A.is_cuda and I.is_cuda):
        return False
    if not head_supported(model):
        return False
    return A.shape[0] == I.shape[0]


class AdamCarry:
    """Adam updates carried by an encoder's later backward launches (tspm_conv_bwd_adam, ABI 20).

    The backward visits the blocks from the last to the first.  When a block is done its parameters (and, first,
    the fc's) are final and no later launch reads them (``ready``); the next fused dgrad + wgrad launches then carry
    their Adam update as extra workgroups of the same grid (``take``: conv2's launch half of what is pending,
    conv1's the rest), overlapping the latency-bound GEMM tiles instead of following the backward.  Parameters
    are visited in descending flat-buffer order, so what is pending is one contiguous element range of the
    (single) flat group; ``carried`` lists the issued ranges — the caller updates the rest with launch_ranges.
    Bitwise the one-launch update (Adam is element-wise; the carried loop is tspm_adam_step's)."""

    def __init__(self, opt, max_blocks: int = 512, elems_per_block: int = 8192):
        fgs = opt.flat_groups()
        self.fg = fgs[0] if len(fgs) == 1 else None
        self.where = {}
        if self.fg is not None:
            from .optim import _ALIGN
            for p, o in zip(self.fg.params, self.fg.offsets):
                self.where[id(p)] = (o, o + (p.numel() + _ALIGN - 1) // _ALIGN * _ALIGN)
        self.lo = self.hi = None  # pending [lo, hi)
        self.carried: List[Tuple[int, int]] = []
        self.max_blocks = max_blocks
        self.elems_per_block = elems_per_block

    def ready(self, params) -> None:
        spans = [self.where.get(id(p)) for p in params]
        if not spans or any(sp is None for sp in spans):
            return
        # the block's spans must tile [a, b) exactly: with a parameter order that interleaves another block's (or
        # the other encoder's) parameters into this range, [min, max) would cover elements whose gradients may
        # still be in flight — such a block stays with the optimizer's own launches
        spans = sorted(spans)
        if any(spans[i][1] != spans[i + 1][0] for i in range(len(spans) - 1)):
            return
        a, b = spans[0][0], spans[-1][1]
        if self.lo is None:
            self.lo, self.hi = a, b
        elif b == self.lo:
            self.lo = a
        # anything else (not adjacent) stays with the caller's own launches

    def take(self, share: float):
        if self.lo is None or share <= 0:
            return None
        n = self.hi - self.lo
        k = n if share >= 1 else min(n, (int(n * share) + 3) // 4 * 4)
        if k <= 0:
            return None
        a, b = self.hi - k, self.hi
        self.hi = a
        if self.hi <= self.lo:
            self.lo = self.hi = None
        self.carried.append((a, b))
        fg = self.fg
        blocks = max(1, min(self.max_blocks, -(-k // self.elems_per_block)))
        return L.AdamJob(fg.param[a:].data_ptr(), fg.grad[a:].data_ptr(), fg.exp_avg[a:].data_ptr(),
                         fg.exp_avg_sq[a:].data_ptr(), k, fg.hyper.data_ptr(), blocks, 0)

    def rest_of(self, ranges):
        """``ranges`` (per group, list of [a, b)) minus the carried ranges."""
        if self.fg is None or not self.carried:
            return ranges
        out = []
        cut = sorted(self.carried)
        for a, b in ranges[0]:
            cur = a
            for c, d in cut:
                if d <= cur or c >= b:
                    continue
                if c > cur:
                    out.append((cur, c))
                cur = max(cur, d)
            if cur < b:
                out.append((cur, b))
        return [out] + list(ranges[1:])


class FusedTrainStep:
    def __init__(self, model, optimizer: FusedAdam, loss_functions, batch: int, audio_hw=(32, 94), image_hw=(28, 28),
                 use_graph: bool = True, allreduce=None, adam_split=True):
        self.model = model
        self.opt = optimizer
        self.loss_functions = loss_functions
        self.ce_weight = _ce_weight(loss_functions)
        if not head_supported(model):
            raise L.TspmError("FusedTrainStep: the fusion head's shape is outside tspm_head_train_step's limits "
                              "(use AVMNIST.train_step, which routes such heads to the autograd path)")
        self.N = batch
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        self.allreduce = allreduce
        p0 = next(model.parameters())
        dev = p0.device
        self.device = dev
        model.train()
        prepare_encoder_layout(model.audio_encoder)
        prepare_encoder_layout(model.image_encoder)
        # flat grads must exist for every parameter (FusedAdam set them as views)
        for p in model.parameters():
            if p.requires_grad and p.grad is None:
                raise L.TspmError("FusedTrainStep: parameter without a FusedAdam gradient view")
        self.eng_a = EncoderEngine(model.audio_encoder, batch, audio_hw[0], audio_hw[1], dev)
        self.eng_i = EncoderEngine(model.image_encoder, batch, image_hw[0], image_hw[1], dev)
        f32 = dict(device=dev, dtype=torch.float32)
        ea, ei = model.embd_size_A, model.embd_size_I
        self.F = ea + ei
        hd = model.hidden_dim
        self.hd, self.h2 = hd, hd // 2
        self.A = torch.empty(batch, audio_hw[0], audio_hw[1], **f32)
        self.I = torch.empty(batch, 1, image_hw[0], image_hw[1], **f32)
        self.labels = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.groups = torch.zeros(batch, dtype=torch.int32, device=dev)  # pattern id per row (metrics)
        # metrics.ClassificationLog: when set, the step also records predictions / confusion counts /
        # the batch loss on the device (train metrics of the epoch, train_multimodal.py:478-491,607-612)
        self.log = None
        self._graph_log = None
        self.fused = torch.empty(batch, self.F, **f32)
        self.h1 = torch.empty(batch, hd, **f32)
        self.hh = torch.empty(batch, self.h2, **f32)
        self.logits = torch.empty(batch, NUM_CLASSES, **f32)
        self.dlogits = torch.empty(batch, NUM_CLASSES, **f32)
        self.dh = torch.empty(batch, self.h2, **f32)     # fc3 pre-activation gradient
        self.dh1 = torch.empty(batch, hd, **f32)         # fc0 pre-activation gradient
        self.dfused = torch.empty(batch, self.F, **f32)
        self.row_ws = torch.empty(2 * batch, **f32)       # per-row CE / correct flags (tspm_head_train_step)
        self.keep = torch.ones(batch, hd, dtype=torch.uint8, device=dev)
        self.loss = torch.zeros(1, **f32)
        self.stats = torch.zeros(4, **f32)  # loss*n, correct, n (accumulated on device)
        self.keep_override: Optional[torch.Tensor] = None
        self.nbt = shared_batches_tracked(model, dev)
        # the image encoder's branch runs on a side stream; the DP exchange on a third (one set per process,
        # shared by every step build: L.shared_streams)
        self.side, self.comm = L.shared_streams(dev, 2)
        self.serial = os.environ.get("TSPM_SERIAL", "0") == "1"  # True: one stream (per-kernel timing)
        # the audio encoder's LDS-staged convs with an 82,000-byte LDS floor: one workgroup per CU, leaving room
        # for the image chain, the replayed step's critical path (scripts/overlap_probe.py --dump: image forward +
        # head + image backward + image Adam).  A/B, alternating processes: 2.5907 vs 2.6280 ms (56,000 bytes:
        # 2.613 vs 2.630), profiles/r5/r5i_floor*.json.  TSPM_SLACK_LDS_FLOOR=0 restores the unconstrained launches
        # At batch 1024 the floor costs 1.05 ms per step (10.84 vs 9.79 ms, profiles/r5/r5t_floor_b1024.json: the
        # audio chain's large convs need their occupancy there) and at batch 32 it is neutral (2.6497 vs 2.6459 ms,
        # r5u_floor_b32.json), so the default applies at batches 64-128 only
        self.slack_lds_floor = int(os.environ.get("TSPM_SLACK_LDS_FLOOR", "82000" if 64 <= batch <= 128 else "0"))
        self.slack_parts = os.environ.get("TSPM_SLACK_PARTS", "fb")  # the audio forward (f) and / or backward (b)
        # Adam updates of finished blocks carried by the later backward launches of "image" / "audio" / "both"
        # encoders (AdamCarry; single-GPU split schedule only); "none" = the optimizer's own launches.  A/B,
        # alternating processes (profiles/r5/r5n-r5p): both 2.5526 vs 2.5931 ms with 512 carrying workgroups of
        # 8,192 elements (256 x 16,384: 2.5571 vs 2.5933; image only: 2.5692 vs 2.5965); batch 1024: 9.807 vs
        # 9.866 ms (r5u_carry_b1024.json)
        self.adam_carry = os.environ.get("TSPM_ADAM_CARRY", "both")
        # the head's samples per workgroup (tspm_head_desc.rows_per_block, ABI 21): 0 = the library's default (1 up
        # to 256 rows, else 4); TSPM_HEAD_RB=1 / 4 forces one for A/B (read here, not inside the library)
        self.head_rows_per_block = int(os.environ.get("TSPM_HEAD_RB", "0"))
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.graph_opt: Optional[torch.cuda.CUDAGraph] = None
        # single-GPU step (adam_split): each encoder's parameters updated by Adam on that encoder's stream right
        # after its own backward (the image encoder's beside the audio chain's tail), the head's with the audio
        # encoder's; bitwise the one-launch update (Adam is element-wise).  A cross-stream edge in the middle of
        # the two chains (e.g. the audio layer3/4 update moved to the image stream) serialised the replayed
        # graph: 3.55 ms vs 2.64 (profiles/r4/r4f_ab_adam_schedules.json)
        self.adam_split = adam_split
        # bench.py's exchange block: when a list, the phased DP step appends per step the host's waits for
        # the two step flags and a pair of events (graph end, step end) bracketing the exposed exchange tail
        self.exchange_probe: Optional[list] = None
        self._split_ranges = None
        self._graph_gen_keep = True
        self._head_bumps_step = False
        self.calls = 0
        self._sig = (id(optimizer), id(loss_functions), batch)
        # dropout RNG counter = FusedAdam's device step counter (distinct per step, graph-safe)
        fgs = optimizer.flat_groups()
        self._rng_ctr_ptr = fgs[0].hyper.data_ptr() + L.HYPER_STEP_OFFSET if fgs else None

    def matches(self, A, I, optimizer, loss_functions) -> bool:
        return self._sig == (id(optimizer), id(loss_functions), A.shape[0]) and tuple(A.shape[1:]) in (
            tuple(self.A.shape[1:]),) and tuple(I.shape[-2:]) == tuple(self.I.shape[-2:])

    # ------------------------------------------------------------------------------------------
    def _head(self, sh: int) -> None:
        """The fusion head's forward, the loss group's cross-entropy and the head's backward in two launches
        (tspm_head_train_step, ABI 16; MML_Suite/models/avmnist.py:219-230,267, experiment_utils/loss.py:98-148):
        h1 / hh / logits / loss, the dropout keep mask (drawn on the device from the step counter unless
        keep_override was copied in), the net.{0,3,5} weight and bias gradients into FusedAdam's flat
        buffer, and dfused = the gradient into both encoders' embeddings."""
        net = self.model.net
        p = float(self.model.dropout_p)
        g = lambda t: t.data_ptr()  # noqa: E731
        d = L.HeadDesc(n=self.N, in_=self.F, hidden=self.hd, hidden2=self.h2, classes=NUM_CLASSES, ldx=self.F,
                       lddx=self.F, gen_keep=1 if (p > 0 and self.keep_override is None) else 0,
                       x=g(self.fused), w0=g(net[0].weight), b0=g(net[0].bias), w3=g(net[3].weight), b3=g(net[3].bias),
                       w5=g(net[5].weight), b5=g(net[5].bias), p=p, loss_weight=self.ce_weight,
                       seed=int(self.model._rng_seed) if p > 0 else 0, counter=self._rng_ctr_ptr if p > 0 else None,
                       keep=g(self.keep), labels=g(self.labels), h1=g(self.h1), hh=g(self.hh), logits=g(self.logits),
                       dlogits=g(self.dlogits), dz3=g(self.dh), dz0=g(self.dh1), dx=g(self.dfused), row_ws=g(self.row_ws),
                       gw0=g(net[0].weight.grad), gb0=g(net[0].bias.grad), gw3=g(net[3].weight.grad),
                       gb3=g(net[3].bias.grad), gw5=g(net[5].weight.grad), gb5=g(net[5].bias.grad),
                       loss=g(self.loss), stats=g(self.stats),
                       adam_step=self._rng_ctr_ptr if self._head_bumps_step else None,
                       rows_per_block=self.head_rows_per_block)
        L.check(L.lib().tspm_head_train_step(d, sh), "head_train_step")

    def _fwd_bwd(self, marks=None) -> None:
        """Enqueue forward + loss + backward on the current stream (+ the side stream for the image encoder).
        ``marks``: two ``_lib.DeviceFlag``s bumped after the audio / image encoder's backward phase 1 (fc,
        layer4, layer3: the same launches, split at the phase boundary), which the DP exchange waits on outside
        the graph (_run_phased)."""
        main = torch.cuda.current_stream()
        ea = self.model.embd_size_A
        side = main if self.serial else self.side
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.eng_i.forward(self.I, self.fused[:, ea:], self.F, train=True, bump_batches_tracked=False)
        with self._slack_floor("f"):
            self.eng_a.forward(self.A, self.fused, self.F, train=True, bump_batches_tracked=False)
        main.wait_stream(side)
        sh = main.cuda_stream
        # the single-GPU split schedule with one flat group: the head's second launch advances the Adam step
        # counter (tspm_head_desc.adam_step) instead of a tspm_adam_begin launch before the fork
        self._head_bumps_step = (marks is None and self._split_opt() and len(self.opt.flat_groups()) == 1
                                 and os.environ.get("TSPM_HEAD_BUMPS_STEP", "1") != "0")
        # (the head's weight-gradient launch on the image stream, beside the audio backward, was measured slower:
        # 2.604 vs 2.589 ms, profiles/r4/r4m2_ab_head.json)
        self._head(sh)
        self._classify(sh)
        side.wait_stream(main)
        if marks is not None:
            mark_a, mark_i = marks
            with self._slack_floor():
                self.eng_a.backward(self.dfused, self.F, phase=1)
            mark_a.bump(main)
            with torch.cuda.stream(side):
                self.eng_i.backward(self.dfused[:, ea:], self.F, phase=1)
                mark_i.bump(side)
            with self._slack_floor():
                self.eng_a.backward(None, self.F, phase=2)
            with torch.cuda.stream(side):
                self.eng_i.backward(None, self.F, phase=2)
        elif self._split_opt():
            img, rest = self._adam_ranges()
            if not self._head_bumps_step:
                self.opt.launch_begin(main.cuda_stream)  # one step-count increment, before every range
            side.wait_stream(main)
            # each encoder's parameters on its own stream at its chain's end, the head's with the audio encoder's
            # (the increment on the image stream and main joining it before the audio + head ranges, with
            # num_batches_tracked moved to the image stream's start: 2.614 vs 2.595 ms, profiles/r4/r4q_ab_lean.json)
            kw = dict(max_blocks=int(os.environ.get("TSPM_ADAM_CARRY_BLOCKS", "512")),
                      elems_per_block=int(os.environ.get("TSPM_ADAM_CARRY_ELEMS", "8192")))
            ci = AdamCarry(self.opt, **kw) if self.adam_carry in ("image", "both") else None
            ca = AdamCarry(self.opt, **kw) if self.adam_carry in ("audio", "both") else None
            with torch.cuda.stream(side):
                self.eng_i.adam_carry = ci
                try:
                    self.eng_i.backward(self.dfused[:, ea:], self.F)
                finally:
                    self.eng_i.adam_carry = None
                self.opt.launch_ranges(side.cuda_stream, ci.rest_of(img) if ci else img)
            with self._slack_floor():
                self.eng_a.adam_carry = ca
                try:
                    self.eng_a.backward(self.dfused, self.F)
                finally:
                    self.eng_a.adam_carry = None
            self.opt.launch_ranges(main.cuda_stream, ca.rest_of(rest) if ca else rest)
        else:
            with torch.cuda.stream(side):
                self.eng_i.backward(self.dfused[:, ea:], self.F)
            with self._slack_floor():
                self.eng_a.backward(self.dfused, self.F)
        main.wait_stream(side)
        L.counters_add(self.nbt)

    @contextlib.contextmanager
    def _slack_floor(self, part: str = "b"):
        """The audio encoder's LDS-staged conv launches with a minimum LDS allocation (TSPM_SLACK_LDS_FLOOR bytes,
        passed per launch as tspm_conv_algo.lds_floor — ABI 21, no library state), so fewer of its workgroups share
        a CU with the image chain (the replayed step's critical path, scripts/overlap_probe.py --dump).  The floor
        lives on this step's own audio engine and only while its launches are enqueued."""
        floor = self.slack_lds_floor if part in self.slack_parts else 0
        if floor and not self.serial:
            self.eng_a.lds_floor = floor
        try:
            yield
        finally:
            self.eng_a.lds_floor = 0

    def _split_opt(self) -> bool:
        """Adam launched per encoder inside the fwd/bwd enqueue (single GPU, no gradient clipping: the
        range launches have no clip-coefficient form)."""
        return bool(self.adam_split) and self.allreduce is None and getattr(self.opt, "clip_coef", None) is None

    def _adam_ranges(self):
        """FusedAdam flat-buffer ranges per group of (image encoder, audio encoder + head)."""
        if self._split_ranges is None:
            from .ddp import flat_ranges
            img = {id(p) for p in self.model.image_encoder.parameters()}
            out = ([], [])
            for fg in self.opt.flat_groups():
                numels = [p.numel() for p in fg.params]
                sel = [id(p) in img for p in fg.params]
                out[0].append(flat_ranges(fg.offsets, numels, fg.numel, sel))
                out[1].append(flat_ranges(fg.offsets, numels, fg.numel, [not x for x in sel]))
            self._split_ranges = out
        return self._split_ranges

    def phased_allreduce(self, force: bool = False, bucket_mb: float = 64.0, group=None):
        """The overlapped DP exchange for this step: gradient ranges of FusedAdam's flat buffers in
        three phases — (0) head + audio fc/layer4/layer3, (1) image fc/layer4/layer3, (2) both
        encoders' layer2/layer1/stem — each launched as soon as the backward part that writes it
        has run (see _run_phased)."""
        from .ddp import PhasedGradAllReduce, flat_ranges
        sets = [{id(p) for p in self.eng_a.phase_params(1)} | {id(p) for p in self.model.net.parameters()},
                {id(p) for p in self.eng_i.phase_params(1)},
                {id(p) for p in self.eng_a.phase_params(2) + self.eng_i.phase_params(2)}]
        views = [[], [], []]
        ranges = ([], [], [])  # per phase, per flat group: the element ranges (Adam after that phase's exchange)
        for fg in self.opt.flat_groups():
            for p in fg.params:
                if sum(id(p) in st for st in sets) != 1:
                    raise L.TspmError("phased all-reduce: parameter not owned by exactly one backward phase")
            numels = [p.numel() for p in fg.params]
            for k, st in enumerate(sets):
                rk = flat_ranges(fg.offsets, numels, fg.numel, [id(p) in st for p in fg.params])
                ranges[k].append(rk)
                views[k] += [fg.grad[a:b] for a, b in rk]
        self._phase_ranges = ranges
        return PhasedGradAllReduce(views, bucket_mb=bucket_mb, group=group, force=force)

    def _run_phased(self) -> None:
        """DP step with the RCCL exchange overlapped with backward, the whole forward + backward as ONE
        HIP graph (the plain step's two-stream schedule), and each phase's Adam update right behind that
        phase's exchange:
             main (graph): [fwd both + head + audio bwd late ─●─ audio bwd early] ─ RCCL(both early) ─ Adam(early)
             side (graph):                   [image bwd late ─●─ image bwd early] ─┘
             comm:          RCCL(head+audio late) ─ Adam(head+audio late) · RCCL(image late) ─ Adam(image late)
        ● = a step flag (``_lib.DeviceFlag``: a one-thread kernel in the graph publishes a per-step count to
        pinned host memory; the host waits for it before launching the collective — ROCm 7 refuses
        graph-external event records); the collectives run on RCCL's stream, each after the flag of the
        backward part that writes its gradients, and the comm / main streams wait for them before the Adam
        ranges of the same parameters (phase 2's backward reads none of the phase-0/1 parameters).  Adam is
        element-wise, so the per-phase ranges give bitwise the one-launch update."""
        ar = self.allreduce
        if getattr(self.opt, "clip_coef", None) is not None:
            # the per-phase Adam ranges have no clip-coefficient form: refuse instead of ignoring it
            raise L.TspmError("phased DP step: FusedAdam.clip_coef is set, but the per-phase Adam ranges cannot "
                              "apply a clip coefficient; use the plain DP step (allreduce=GradAllReduce)")
        eager = not self.use_graph or self.calls == 0
        if getattr(self, "_marks", None) is None:
            self._marks = (L.DeviceFlag(), L.DeviceFlag())
        if getattr(self, "_phase_ranges", None) is None:
            raise L.TspmError("phased step: build the exchange with FusedTrainStep.phased_allreduce()")
        if eager:
            self._fwd_bwd(marks=self._marks)
        else:
            if self.graph is None:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with L.graph_capture(g):
                    self._fwd_bwd(marks=self._marks)
                self.graph, self.graph_opt = g, None
                self._graph_gen_keep = self.keep_override is None
            self.graph.replay()
        # each flag is bumped once per step, after (in graph order) everything main ran before this step
        # (batch upload, the previous step's Adam reading the gradients): once the host has seen it, the
        # gradients it covers are complete, so the exchange launched then needs no device-side wait
        for f in self._marks:
            f.count += 1
        main, comm, r = torch.cuda.current_stream(), self.comm, self._phase_ranges
        probe = self.exchange_probe
        if probe is not None:  # the graph's end on main (the side stream joined it inside the graph)
            ev_graph = torch.cuda.Event(enable_timing=True)
            ev_graph.record(main)
            t0 = time.perf_counter()
        self._marks[0].host_wait(self._marks[0].count)
        if probe is not None:
            t1 = time.perf_counter()
        with torch.cuda.stream(comm):
            ar.wait(ar.launch(0))
            self.opt.launch_begin(comm.cuda_stream)  # one step-count increment, before every range
            self.opt.launch_ranges(comm.cuda_stream, r[0])
        if probe is not None:
            t2 = time.perf_counter()
        self._marks[1].host_wait(self._marks[1].count)
        if probe is not None:
            t3 = time.perf_counter()
        with torch.cuda.stream(comm):
            ar.wait(ar.launch(1))
            self.opt.launch_ranges(comm.cuda_stream, r[1])
        ar.wait(ar.launch(2))  # on main, behind the graph: no stream hop before the last exchange
        main.wait_stream(comm)  # the step-count increment and the phase-0/1 updates before the step ends
        self.opt.launch_ranges(main.cuda_stream, r[2])
        if probe is not None:
            ev_end = torch.cuda.Event(enable_timing=True)
            ev_end.record(main)
            # the window each late phase's exchange has to hide in: from the host seeing that phase's flag to the
            # end of the fwd+bwd graph (the rest of the backward), host clock, the graph's end polled (probe only)
            while not ev_graph.query():
                pass
            t4 = time.perf_counter()
            probe.append({"host_wait_ms": ((t1 - t0) * 1e3, (t3 - t2) * 1e3), "events": (ev_graph, ev_end),
                          "window_ms": ((t4 - t1) * 1e3, (t4 - t3) * 1e3)})

    def close(self) -> None:
        """Release the step's device-side resources in a safe order, before the process group goes away
        (bench.py, the DP tests): wait for every stream (the graph's two, the exchange stream, RCCL's via the
        device), drop the captured graphs (they bump the step flags), then free the flags.  Idempotent; the
        step is unusable afterwards."""
        if getattr(self, "_closed", False):
            return
        self._closed = True
        torch.cuda.synchronize(self.device)
        self.graph, self.graph_opt = None, None
        marks, self._marks = getattr(self, "_marks", None), None
        if marks is not None:
            for f in marks:
                f.close()
        self.allreduce = None
        self.exchange_probe = None

    def _classify(self, sh: int) -> None:
        log = self.log
        if log is None:
            return
        L.check(L.lib().tspm_classify_update(
            self.N, NUM_CLASSES, self.logits.data_ptr(), self.labels.data_ptr(), self.groups.data_ptr(),
            len(log.groups), log.conf.data_ptr(), None, self.loss.data_ptr(), log.loss_log.data_ptr(),
            log.counters.data_ptr(), log.capacity, sh), "classify_update")

    def _opt(self) -> None:
        self.opt.launch(torch.cuda.current_stream().cuda_stream)

    def _enqueue_all(self) -> None:
        self._fwd_bwd()
        if self.allreduce is None and not self._split_opt():
            self._opt()

    # ------------------------------------------------------------------------------------------
    def load_batch(self, A: torch.Tensor, I: torch.Tensor, labels: torch.Tensor,
                   groups: Optional[torch.Tensor] = None) -> None:
        if groups is not None and groups.data_ptr() != self.groups.data_ptr():
            self.groups.copy_(groups.reshape(-1).to(torch.int32), non_blocking=True)
        if A.data_ptr() != self.A.data_ptr():
            self.A.copy_(A.reshape(self.A.shape), non_blocking=True)
        if I.data_ptr() != self.I.data_ptr():
            self.I.copy_(I.reshape(self.I.shape), non_blocking=True)
        if labels.data_ptr() != self.labels.data_ptr():
            self.labels.copy_(labels, non_blocking=True)

    def step(self, A: torch.Tensor, I: torch.Tensor, labels: torch.Tensor,
             groups: Optional[torch.Tensor] = None) -> Dict[str, torch.Tensor]:
        self.load_batch(A, I, labels, groups)
        self.run()
        return {"loss": self.loss, "logits": self.logits}

    def run(self) -> None:
        """One training step on the batch currently in the static input buffers."""
        if getattr(self, "_closed", False):
            raise L.TspmError("FusedTrainStep.run after close()")
        self.model.train()
        self.opt.sync_hyper()
        if self._graph_log is not self.log:  # the metrics log is baked into the captured graphs
            self.graph, self.graph_opt = None, None
            self._graph_log = self.log
        if self.keep_override is not None:
            self.keep.copy_(self.keep_override.reshape(self.keep.shape).to(torch.uint8), non_blocking=True)
        # the captured head either draws its keep mask or reads the copied-in one: re-capture on a change
        if self.graph is not None and self._graph_gen_keep != (self.keep_override is None):
            self.graph, self.graph_opt = None, None
        if isinstance(self.allreduce, PhasedGradAllReduce):
            self._run_phased()
            self.opt.note_steps(1)
            self.calls += 1
            return
        if not self.use_graph or self.calls == 0:
            self._enqueue_all()
        else:
            if self.graph is None:
                self._capture()
            self.graph.replay()
        if self.allreduce is not None:
            self.allreduce()
            if self.use_graph and self.graph_opt is not None:
                self.graph_opt.replay()
            else:
                self._opt()
        self.opt.note_steps(1)
        self.calls += 1

    def _capture(self) -> None:
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with L.graph_capture(g):
            if self.allreduce is None:
                self._enqueue_all()
            else:
                self._fwd_bwd()
        self.graph = g
        self._graph_gen_keep = self.keep_override is None
        if self.allreduce is not None:
            go = torch.cuda.CUDAGraph()
            with L.graph_capture(go):
                self._opt()
            self.graph_opt = go


class FusedEvalStep:
    """AVMNIST.validation_step (MML_Suite/models/avmnist.py:312-360) as one HIP graph: both encoders in
    eval mode (BatchNorm running statistics) on two streams, the fusion head without dropout, the loss
    (LossFunctionGroup total = weight × CE) and ``tspm_classify_update`` — predictions, per-pattern
    confusion counts and the per-batch loss go to a :class:`metrics.ClassificationLog` on the device,
    so an evaluation epoch has no host round trip per batch.  Shares the encoders' cached HIP plans
    (``ResNetEncoder.engine_for``) with the module forward."""

    def __init__(self, model, loss_functions, batch: int, log=None, audio_hw=(32, 94), image_hw=(28, 28),
                 use_graph: bool = True):
        self.model, self.N, self.log = model, batch, log
        self.ce_weight = _ce_weight(loss_functions)
        if self.ce_weight is None:
            raise L.TspmError("FusedEvalStep: the loss group must be a single cross-entropy term")
        self.use_graph = use_graph and not os.environ.get("TSPM_NO_GRAPH")
        dev = next(model.parameters()).device
        self.device = dev
        f32 = dict(device=dev, dtype=torch.float32)
        self.A = torch.zeros(batch, audio_hw[0], audio_hw[1], **f32)
        self.I = torch.zeros(batch, 1, image_hw[0], image_hw[1], **f32)
        self.labels = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.groups = torch.zeros(batch, dtype=torch.int32, device=dev)
        self.eng_a = model.audio_encoder.engine_for(self.A)
        self.eng_i = model.image_encoder.engine_for(self.I)
        ea, ei = model.embd_size_A, model.embd_size_I
        self.F, self.hd = ea + ei, model.hidden_dim
        self.fused = torch.empty(batch, self.F, **f32)
        self.h1 = torch.empty(batch, self.hd, **f32)
        self.hh = torch.empty(batch, self.hd // 2, **f32)
        self.logits = torch.empty(batch, NUM_CLASSES, **f32)
        self.loss = torch.zeros(1, **f32)
        self.preds = torch.zeros(batch, dtype=torch.int64, device=dev)
        self.side = L.shared_streams(dev, 1)[0]
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._graph_log = None
        self.calls = 0

    def load_batch(self, A: torch.Tensor, I: torch.Tensor, labels: torch.Tensor,
                   groups: Optional[torch.Tensor] = None) -> None:
        for dst, src in ((self.A, A), (self.I, I), (self.labels, labels)):
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src.reshape(dst.shape), non_blocking=True)
        if groups is not None and groups.data_ptr() != self.groups.data_ptr():
            self.groups.copy_(groups.reshape(-1).to(torch.int32), non_blocking=True)

    def _enqueue(self) -> None:
        lib = L.lib()
        main = torch.cuda.current_stream()
        ea = self.model.embd_size_A
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            self.eng_i.forward(self.I, self.fused[:, ea:], self.F, train=False)
        self.eng_a.forward(self.A, self.fused, self.F, train=False)
        main.wait_stream(self.side)
        sh = main.cuda_stream
        n, F, hd, h2 = self.N, self.F, self.hd, self.hd // 2
        net = self.model.net
        L.check(lib.tspm_linear_fwd(n, F, hd, self.fused.data_ptr(), F, net[0].weight.data_ptr(),
                                    net[0].bias.data_ptr(), 1, None, 1.0, self.h1.data_ptr(), hd, sh), "eval fc0")
        L.check(lib.tspm_linear_fwd(n, hd, h2, self.h1.data_ptr(), hd, net[3].weight.data_ptr(),
                                    net[3].bias.data_ptr(), 1, None, 1.0, self.hh.data_ptr(), h2, sh), "eval fc3")
        L.check(lib.tspm_linear_fwd(n, h2, NUM_CLASSES, self.hh.data_ptr(), h2, net[5].weight.data_ptr(),
                                    net[5].bias.data_ptr(), 0, None, 1.0, self.logits.data_ptr(), NUM_CLASSES, sh),
                "eval fc5")
        L.check(lib.tspm_cross_entropy(n, NUM_CLASSES, self.logits.data_ptr(), self.labels.data_ptr(),
                                       self.loss.data_ptr(), None, self.ce_weight, None, sh), "eval cross_entropy")
        log = self.log
        L.check(lib.tspm_classify_update(
            n, NUM_CLASSES, self.logits.data_ptr(), self.labels.data_ptr(), self.groups.data_ptr(),
            len(log.groups) if log is not None else 1, log.conf.data_ptr() if log is not None else None,
            self.preds.data_ptr(), self.loss.data_ptr(), log.loss_log.data_ptr() if log is not None else None,
            log.counters.data_ptr() if log is not None else None, log.capacity if log is not None else 0, sh),
            "eval classify_update")

    def run(self) -> None:
        """Evaluate the batch in the static input buffers (logits, loss, preds; log updated)."""
        self.model.eval()
        if not self.use_graph or self.calls == 0:
            self._enqueue()
        else:
            if self.graph is None or self._graph_log is not self.log:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with L.graph_capture(g):
                    self._enqueue()
                self.graph, self._graph_log = g, self.log
            self.graph.replay()
        self.calls += 1

    def step(self, A, I, labels, groups=None) -> Dict[str, torch.Tensor]:
        self.load_batch(A, I, labels, groups)
        self.run()
        return {"loss": self.loss, "logits": self.logits, "preds": self.preds}
