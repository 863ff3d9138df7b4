"""Per-encoder execution plan: the ResNet18/34 encoder forward/backward as a fixed schedule of
libtspm kernels over pre-allocated HWNC buffers.

Mirrors ``ResNetEncoder.forward`` (MML_Suite/models/msa/networks/resnet.py:199-219) and
``BasicBlock.forward`` (:37-54) and their autograd backward.  All launches go to the caller's
current stream through the C ABI; nothing allocates inside ``forward_train``/``backward``, so the
whole step can be captured into a HIP graph.
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import torch

from . import _lib as L
from ._lib import linear_bwd

BN_EPS = 1e-5
BN_MOMENTUM = 0.1


_TUNED_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned")
_tuned_cache: Optional[Dict[Tuple, Tuple[int, int, int, int, int]]] = None


def tuned_table() -> Dict[Tuple, Tuple[int, int, int, int, int]]:
    """Measured tile configurations (scripts/tune_convs.py output under ``tuned/``), keyed
    (kind, n, h, w, c, k, r, s, stride).  ``TSPM_TUNED=0`` disables them (library heuristic)."""
    global _tuned_cache
    if os.environ.get("TSPM_TUNED", "1") == "0":
        return {}
    if _tuned_cache is None:
        _tuned_cache = {}
        only = os.environ.get("TSPM_TUNED_FILE")  # one table instead of tuned/*.json (A/B experiments)
        for path in ([only] if only else sorted(glob.glob(os.path.join(_TUNED_DIR, "*.json")))):
            with open(path) as fh:
                doc = json.load(fh)
            for e in doc.get("entries", []):
                _tuned_cache[(e["kind"],) + tuple(e["shape"][:8])] = tuple(e["algo"])
    return _tuned_cache


def _out_hw(h: int, w: int, k: int, s: int, p: int) -> Tuple[int, int]:
    return (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1


@dataclass
class ConvOp:
    module: torch.nn.Conv2d
    shape: L.ConvShape
    algo_fwd: L.ConvAlgo = field(default_factory=L.ConvAlgo)
    algo_dgrad: L.ConvAlgo = field(default_factory=L.ConvAlgo)
    algo_wgrad: L.ConvAlgo = field(default_factory=L.ConvAlgo)
    bwd_fused: Optional[bool] = None  # tspm_conv_bwd_supported for (algo_dgrad, algo_wgrad); None = not asked
    bn_inlaunch: Optional[bool] = None  # tspm_conv_fwd_bn_inlaunch for algo_fwd; None = not asked

    @property
    def rows_out(self) -> int:
        s = self.shape
        return s.p * s.q * s.n

    @property
    def rows_in(self) -> int:
        s = self.shape
        return s.h * s.w * s.n

    def ws_bytes(self, need_dgrad: bool) -> int:
        lib = L.lib()
        b = lib.tspm_conv_wgrad_workspace(ctypes.byref(self.shape), ctypes.byref(self.algo_wgrad))
        b = max(b, lib.tspm_conv_fwd_workspace(ctypes.byref(self.shape), ctypes.byref(self.algo_fwd)))
        if need_dgrad:
            b = max(b, lib.tspm_conv_dgrad_workspace(ctypes.byref(self.shape), ctypes.byref(self.algo_dgrad)))
        return b

    def bn_counters(self) -> int:
        return L.lib().tspm_conv_fwd_bn_counters(ctypes.byref(self.shape), ctypes.byref(self.algo_fwd))

    def bn_partial_floats(self) -> int:
        return L.lib().tspm_conv_fwd_bn_partial_floats(ctypes.byref(self.shape), ctypes.byref(self.algo_fwd))

    def stat_tiles(self) -> Tuple[int, int]:
        """(tiles, rows per tile) of the BN partial statistics the forward epilogue emits."""
        lib = L.lib()
        return (lib.tspm_conv_fwd_tiles(ctypes.byref(self.shape), ctypes.byref(self.algo_fwd)),
                lib.tspm_conv_fwd_tile_rows(ctypes.byref(self.shape), ctypes.byref(self.algo_fwd)))


@dataclass
class BNOp:
    module: torch.nn.BatchNorm2d
    rows: int
    channels: int
    mean: Optional[torch.Tensor] = None      # save_mean  [C]
    invstd: Optional[torch.Tensor] = None    # save_invstd [C]
    # round 6: (tiles, rows per tile) of partials the conv forward left for the apply to merge (tspm_bn_apply_merge)
    pending: Optional[Tuple[int, int]] = None
    # round 6: the backward's partial sums written by the dgrad epilogue that produces this BN's incoming gradient
    # (tspm_conv_bwd_ex), [3][rows/32][C]; None when the BN is not eligible (tiles > 128, pooled gradient source)
    part: Optional[torch.Tensor] = None
    cnt: Optional[torch.Tensor] = None       # round 6: column-block tickets of the whole-BN-backward epilogue mode


@dataclass
class BlockPlan:
    conv1: ConvOp
    bn1: BNOp
    conv2: ConvOp
    bn2: BNOp
    ds_conv: Optional[ConvOp]
    ds_bn: Optional[BNOp]
    # buffers (HWNC)
    y1: torch.Tensor = None
    a1: torch.Tensor = None
    y2: torch.Tensor = None
    yd: Optional[torch.Tensor] = None
    out: torch.Tensor = None
    # backward: per-block gradients of the conv outputs
    g_y1: torch.Tensor = None
    g_y2: torch.Tensor = None
    g_yd: Optional[torch.Tensor] = None


class EncoderEngine:
    """Execution plan of one ResNetEncoder for a fixed (batch, H, W)."""

    def __init__(self, encoder: torch.nn.Module, batch: int, height: int, width: int, device: torch.device,
                 grad_of: Optional[Callable[[torch.Tensor], torch.Tensor]] = None):
        self.enc = encoder
        self.N, self.H, self.W = batch, height, width
        self.device = device
        self.grad_of = grad_of or _default_grad_of
        # Every launch goes to the caller's current stream.  (Measured and removed, DESIGN §7: weight-grad
        # convs / the downsample branch on auxiliary streams — a replayed graph with their ~50 cross-stream
        # edges ran ~30 % slower; BN
        # backward partials in the dgrad epilogue (conv +5 us per launch, step unchanged); bn1 + ReLU in conv2's
        # loader (tspm_conv_fwd_bnin: step 2.73 vs 2.70 ms); transposed wgrad operands (34.7k vs 36.1k
        # samples/s).  The ABI entry points stay, tested at the kernel level.)
        self.conv_timer = None  # optional: begin(op, kind)/end() around every conv launch (bench roofline)
        # BN statistics of the many-tile layers merged in two levels inside the conv forward (last arrivers,
        # tspm_bn_fuse.counters_len / partial_floats) instead of a tspm_bn_finalize launch.  Off: -5 us per step
        # at batch 128 (within the box-to-box spread), equal at 1024 (profiles/r4/r4n_ab_bn2.json,
        # r4o_ab_bn2_b1024.json), while the merge tails inflate the conv kernels' device time — the conv
        # roofline that tracks the conv kernels reads 0.193 instead of 0.205 (profiles/r4_v1_bench.json)
        self.bn_two_level = os.environ.get("TSPM_BN_TWO_LEVEL", "0") == "1"
        # the last block's BN apply also writes the average-pooled features (tspm_bn_apply_pool, ABI 17): one
        # launch less at the tail of each encoder's forward
        self.fuse_pool = True
        self.debug_hook = None  # optional: fn(name, tensor) called with backward intermediates (diagnostics)
        # optional step.AdamCarry: the single-GPU train step's Adam updates of finished blocks carried by later
        # backward launches (tspm_conv_bwd_adam, ABI 20); None = every update by the optimizer's own launches
        self.adam_carry = None
        # minimum dynamic LDS of this engine's LDS-staged conv launches (tspm_conv_algo.lds_floor, ABI 21 — a per-call
        # launch option, no library state): set by the train step around the encoder with slack (step._slack_floor)
        self.lds_floor = 0
        # the pooling backwards folded into the adjacent BN backward (tspm_bn_bwd_src, round 5); TSPM_BN_POOL_SRC=0
        # restores the separate tspm_avgpool_bwd / tspm_maxpool_bwd launches for A/B
        self.pool_src = os.environ.get("TSPM_BN_POOL_SRC", "1") != "0"
        # the BN backward's partial sums formed in the epilogue of the fused dgrad + wgrad launch that writes the BN's
        # incoming gradient (tspm_conv_bwd_ex / tspm_bn_bwd_apply_part, round 6) for the BNs of at most 128 32-row
        # tiles whose gradient a fused backward launch produces: one k_bn_bwd_partial launch fewer per such BN.
        # TSPM_BN_DGRAD_PART=0 restores the partial pass (A/B)
        self.bn_dgrad_part = os.environ.get("TSPM_BN_DGRAD_PART", "1") != "0"
        # ... for BNs of at most this many 32-row tiles (each apply workgroup merges them all in its prologue)
        self.bnp_max_tiles = int(os.environ.get("TSPM_BN_DGRAD_PART_TILES", "1024"))
        # ... including the stem BN's, gathered through the max pool's argmax taps (TSPM_BN_DGRAD_PART_STEM=0: off)
        self.bnp_stem = os.environ.get("TSPM_BN_DGRAD_PART_STEM", "1") != "0"
        # ... and for BNs of at most this many rows the WHOLE backward (merge + apply) in that epilogue, by the last
        # tile of each column block (tspm_bn_bwd_part.dy): no apply launch.  In-step A/B: 128 rows (ResNet34 layer4)
        # -11 us, 512 rows +16 us (one workgroup per column block applies the whole map), profiles/r6/r6h_ab_*.json;
        # TSPM_BN_BWD_EPI_ROWS=0: off
        self.bnx_max_rows = int(os.environ.get("TSPM_BN_BWD_EPI_ROWS", "128"))
        self._bnp_ready = set()
        self._bnx_done = set()
        # a downsampling block's first conv and its 1x1 downsample (same input, independent) in ONE forward launch
        # (tspm_conv_fwd_pair, round 6; the downsample takes the first conv's tile shape); TSPM_FWD_PAIR=0: two launches
        self.fwd_pair = os.environ.get("TSPM_FWD_PAIR", "1") != "0"
        # the forward BN statistics of convs that cannot merge them in-launch merged in the apply's prologue
        # (tspm_bn_apply_merge, round 6) instead of a tspm_bn_finalize launch; TSPM_BN_APPLY_MERGE=0 restores it
        self.apply_merge = os.environ.get("TSPM_BN_APPLY_MERGE", "1") != "0"
        # ... and the backward of its second conv together with the downsample's (tspm_conv_bwd_quad, round 6; the
        # downsample takes conv2's tile shapes); TSPM_BWD_QUAD=0: separate launches
        self.bwd_quad = os.environ.get("TSPM_BWD_QUAD", "1") != "0"
        # the stem's BN apply + ReLU + max pool forward in one launch (A/B switch TSPM_STEM_FUSE=0)
        self.stem_fuse = os.environ.get("TSPM_STEM_FUSE", "1") != "0"
        # the encoder fc forward (K = 512, 8-16 output tiles) split 8 ways over K: 2.4399 vs 2.4474 ms per step
        # (A/B, profiles/r5/r5fc_*); TSPM_FC_SPLITS=1 restores the one-launch product
        self.fc_splits = int(os.environ.get("TSPM_FC_SPLITS", "8"))
        self._fc_ws = None
        N = batch
        f32 = dict(device=device, dtype=torch.float32)
        c1 = encoder.conv1
        cin = c1.in_channels
        self.cin = cin
        p1, q1 = _out_hw(height, width, 7, 2, 3)
        self.stem = ConvOp(c1, L.ConvShape(N, height, width, cin, c1.out_channels, 7, 7, 2, 3, p1, q1))
        self.stem_bn = BNOp(encoder.bn1, p1 * q1 * N, c1.out_channels)
        p2, q2 = _out_hw(p1, q1, 3, 2, 1)
        self.mp_shape = (p1, q1, p2, q2)
        C0 = c1.out_channels
        self.y0 = torch.empty(p1 * q1 * N, C0, **f32)
        self.a0 = torch.empty(p1 * q1 * N, C0, **f32)
        self.mp = torch.empty(p2 * q2 * N, C0, **f32)
        self.mp_idx = torch.empty(p2 * q2 * N, C0, device=device, dtype=torch.uint8)

        self.blocks: List[BlockPlan] = []
        h, w, c = p2, q2, C0
        for layer in (encoder.layer1, encoder.layer2, encoder.layer3, encoder.layer4):
            for blk in layer:
                st = blk.conv1.stride[0]
                planes = blk.conv1.out_channels
                ho, wo = _out_hw(h, w, 3, st, 1)
                conv1 = ConvOp(blk.conv1, L.ConvShape(N, h, w, c, planes, 3, 3, st, 1, ho, wo))
                conv2 = ConvOp(blk.conv2, L.ConvShape(N, ho, wo, planes, planes, 3, 3, 1, 1, ho, wo))
                rows = ho * wo * N
                bp = BlockPlan(conv1, BNOp(blk.bn1, rows, planes), conv2, BNOp(blk.bn2, rows, planes), None, None)
                if blk.downsample is not None:
                    dc = blk.downsample[0]
                    dst = dc.stride[0]
                    bp.ds_conv = ConvOp(dc, L.ConvShape(N, h, w, c, planes, 1, 1, dst, 0, ho, wo))
                    bp.ds_bn = BNOp(blk.downsample[1], rows, planes)
                bp.y1 = torch.empty(rows, planes, **f32)
                bp.a1 = torch.empty(rows, planes, **f32)
                bp.y2 = torch.empty(rows, planes, **f32)
                bp.out = torch.empty(rows, planes, **f32)
                bp.g_y1 = torch.empty(rows * planes, **f32)
                bp.g_y2 = torch.empty(rows * planes, **f32)
                if bp.ds_conv is not None:
                    bp.yd = torch.empty(rows, planes, **f32)
                    bp.g_yd = torch.empty(rows * planes, **f32)
                self.blocks.append(bp)
                h, w, c = ho, wo, planes
        self.final_hw = (h, w)
        self.final_c = c
        # backward phase split: the first block of layer3 (ResNet18 [2,2,2,2] -> 4, ResNet34 [3,4,6,3] -> 7)
        self.split_block = len(encoder.layer1) + len(encoder.layer2)
        self._bw_state = None
        self.pooled = torch.empty(N, c, **f32)
        self.hidden = encoder.fc.out_features

        # BN saved statistics
        for bn in self.all_bns():
            bn.mean = torch.empty(bn.channels, **f32)
            bn.invstd = torch.empty(bn.channels, **f32)
        # dgrad-epilogue partial sums: bn1 of every block (conv2's input gradient) and bn2 of every block but the last
        # (the next block's conv1 input gradient); 3 planes (the downsample BN shares bn2's gradient)
        for i, bp in enumerate(self.blocks):
            for bn, ok in ((bp.bn1, True), (bp.bn2, i + 1 < len(self.blocks))):
                if ok and bn.rows % 32 == 0 and bn.rows // 32 <= 1024:
                    bn.part = torch.empty(3 * (bn.rows // 32) * bn.channels, **f32)
                    bn.cnt = torch.zeros(bn.channels // 32 + 1, device=device, dtype=torch.int32)
        # the stem BN: its sums over the max pool's input gradient gathered in the pooled domain by layer1's first
        # conv1 data gradient (tspm_bn_bwd_part.idx); tiles = the pooled map's 32-row tiles
        mp_rows = p2 * q2 * N
        if mp_rows % 32 == 0 and mp_rows // 32 <= 1024:
            self.stem_bn.part = torch.empty(3 * (mp_rows // 32) * C0, **f32)

        # backward scratch: grads of block outputs (ping-pong), dy buffers
        max_blk = max(bp.out.numel() for bp in self.blocks)
        max_blk = max(max_blk, self.mp.numel())
        self.gA = torch.empty(max_blk, **f32)
        self.gB = torch.empty(max_blk, **f32)
        self.da1 = torch.empty(max_blk, **f32)
        # the materialised max-pool gradient: only when the stem BN does not read it through the argmax taps
        self.g_stem = None if self.pool_src else torch.empty(self.a0.numel(), **f32)
        self.dy_stem = torch.empty(self.a0.numel(), **f32)
        self.g_pooled = torch.empty(N, c, **f32)
        self.g_final = torch.empty(h * w * N * c, **f32)
        self.set_algos(tuned_table())

    # ---------------------------------------------------------------------------------------
    def all_convs(self) -> List[ConvOp]:
        ops = [self.stem]
        for bp in self.blocks:
            ops += [bp.conv1, bp.conv2] + ([bp.ds_conv] if bp.ds_conv is not None else [])
        return ops

    def all_bns(self) -> List[BNOp]:
        ops = [self.stem_bn]
        for bp in self.blocks:
            ops += [bp.bn1, bp.bn2] + ([bp.ds_bn] if bp.ds_bn is not None else [])
        return ops

    def _alloc_workspace(self) -> None:
        lib = L.lib()
        conv_ws = max(op.ws_bytes(op is not self.stem) for op in self.all_convs())
        bn_ws = 0
        for bn in self.all_bns():
            bn_ws = max(bn_ws, lib.tspm_bn_stats_workspace(bn.rows, bn.channels),
                        lib.tspm_bn_bwd_workspace(bn.rows, bn.channels))
        self.ws_conv_bytes = max(conv_ws, 256)
        self.ws_bn_bytes = max(bn_ws, 256)
        # zero-filled once: the workspaces start with arrival counters that every call leaves zero; the fused
        # backward (tspm_conv_bwd) takes a second one for its weight-gradient half
        self.ws_conv = torch.zeros(self.ws_conv_bytes, device=self.device, dtype=torch.uint8)
        self.ws_conv2 = torch.zeros(self.ws_conv_bytes, device=self.device, dtype=torch.uint8)
        # the downsample half of a quad backward launch (its split-K data / weight gradients)
        self.ws_conv3 = torch.zeros(self.ws_conv_bytes, device=self.device, dtype=torch.uint8)
        self.ws_conv4 = torch.zeros(self.ws_conv_bytes, device=self.device, dtype=torch.uint8)
        self.ws_bn = torch.zeros(self.ws_bn_bytes, device=self.device, dtype=torch.uint8)
        # BN statistics merged in-launch (tspm_conv_fwd_bn_counters / _partial_floats)
        ncnt = max(op.bn_counters() for op in self.all_convs())
        self.bn_cnt = torch.zeros(ncnt, device=self.device, dtype=torch.int32)
        part = max(op.bn_partial_floats() for op in self.all_convs())
        self.bn_part = torch.empty(part, device=self.device, dtype=torch.float32)
        # the downsample half of a paired forward launch merges its BN statistics in buffers of its own
        ds = [bp.ds_conv for bp in self.blocks if bp.ds_conv is not None]
        for bp in self.blocks:
            if bp.ds_conv is not None:
                bp.ds_pair_algo = self._pair_algo(bp)
        ncnt2 = max([self._ds_fwd_algo_op(bp).bn_counters() for bp in self.blocks if bp.ds_conv is not None] + [1])
        part2 = max([self._ds_fwd_algo_op(bp).bn_partial_floats() for bp in self.blocks if bp.ds_conv is not None] + [1])
        self.bn_cnt2 = torch.zeros(ncnt2, device=self.device, dtype=torch.int32)
        self.bn_part2 = torch.empty(part2, device=self.device, dtype=torch.float32)

    def set_algos(self, table: Dict[Tuple, Tuple[int, int, int, int, int]]) -> None:
        """Override tile configs: key (kind, n,h,w,c,k,r,s,stride) -> (tm, tn, wm, wn, splits)."""
        for op in self.all_convs():
            s = op.shape
            base = (s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride)
            tuned_bwd = False
            for kind, key in (("fwd", "fwd"), ("dgrad", "dgrad"), ("wgrad", "wgrad")):
                v = table.get((key,) + base)
                if v is not None:
                    setattr(op, f"algo_{kind}", L.ConvAlgo(*v))
                    tuned_bwd = tuned_bwd or kind != "fwd"
            pair = table.get(("bwd",) + base)
            op.bwd_fused = None
            op.bn_inlaunch = None
            if pair is not None:  # the tuner found the fused launch faster: its (dgrad, wgrad) configs
                op.algo_dgrad, op.algo_wgrad = L.ConvAlgo(*pair[:6]), L.ConvAlgo(*pair[6:12])
            elif tuned_bwd:       # tuned, and the two separate launches won
                op.bwd_fused = False
        self._alloc_workspace()

    # ---------------------------------------------------------------------------------------
    @staticmethod
    def _w(op: ConvOp) -> torch.Tensor:
        w = op.module.weight
        if not w.is_contiguous(memory_format=torch.channels_last):
            raise L.TspmError("conv weight must be OHWI (channels_last); call prepare_encoder_layout() first")
        return w

    def _a(self, algo: L.ConvAlgo) -> L.ConvAlgo:
        """``algo`` with this engine's per-call launch options (the LDS floor)."""
        return algo.with_options(self.lds_floor) if self.lds_floor else algo

    def _conv_fwd(self, op: ConvOp, x_ptr: int, strides: L.Strides4, y: torch.Tensor, sh: int,
                  bnf: Optional[L.BnFuse] = None) -> None:
        lib = L.lib()
        s, a = op.shape, self._a(op.algo_fwd)
        ws = self.ws_conv
        if self.conv_timer:
            self.conv_timer.begin(op, "fwd")
        L.check(lib.tspm_conv_fwd(ctypes.byref(s), ctypes.byref(a), x_ptr, ctypes.byref(strides), self._w(op).data_ptr(),
                                  y.data_ptr(), None if bnf is None else ctypes.byref(bnf), ws.data_ptr(),
                                  self.ws_conv_bytes, sh), "conv_fwd")
        if self.conv_timer:
            self.conv_timer.end()

    def _bnf(self, bn: BNOp, second: bool = False) -> L.BnFuse:
        m = bn.module
        part, cnt = (self.bn_part2, self.bn_cnt2) if second else (self.bn_part, self.bn_cnt)
        return L.BnFuse(part.data_ptr(), cnt.data_ptr(), L.ptr(m.running_mean), L.ptr(m.running_var),
                        BN_MOMENTUM if m.momentum is None else m.momentum, m.eps, bn.mean.data_ptr(),
                        bn.invstd.data_ptr(), cnt.numel() if self.bn_two_level else 0, 0,
                        part.numel() if self.bn_two_level else 0)

    def _pair_algo(self, bp: "BlockPlan") -> L.ConvAlgo:
        """The downsample's algo inside the paired launch: the first conv's tile shape, the downsample's own tuned
        split count when its tuned tile is the same, else no split."""
        a1, ad = bp.conv1.algo_fwd, bp.ds_conv.algo_fwd
        same = (a1.tm, a1.tn, a1.wn, a1.wk, a1.variant) == (ad.tm, ad.tn, ad.wn, ad.wk, ad.variant)
        return L.ConvAlgo(a1.tm, a1.tn, a1.wn, a1.wk, ad.splits if same else 1, a1.variant)

    def _ds_fwd_algo_op(self, bp: "BlockPlan") -> ConvOp:
        return ConvOp(bp.ds_conv.module, bp.ds_conv.shape, algo_fwd=bp.ds_pair_algo)

    def _fwd_pair(self, bp: "BlockPlan", x_ptr: int, strides: L.Strides4, train: bool, sh: int) -> bool:
        """conv1 and the downsample of block ``bp`` in one launch (tspm_conv_fwd_pair); False = not supported for
        these algos (nothing launched)."""
        lib = L.lib()
        c1, cd = bp.conv1, bp.ds_conv
        a1, ad = self._a(c1.algo_fwd), self._a(bp.ds_pair_algo)
        if not self.fwd_pair or not lib.tspm_conv_fwd_pair_supported(
                ctypes.byref(c1.shape), ctypes.byref(a1), ctypes.byref(strides), ctypes.byref(cd.shape),
                ctypes.byref(ad), ctypes.byref(strides)):
            return False
        b1 = self._bnf(bp.bn1) if train else None
        b2 = self._bnf(bp.ds_bn, second=True) if train else None
        if train and self._merge_in_apply(c1, bp.bn1):  # conv1's statistics merged by the bn1 apply (round 6)
            b1.counters = None
            bp.bn1.pending = c1.stat_tiles()
        if self.conv_timer:
            from .roofline import OpGroup
            self.conv_timer.begin(OpGroup((c1, cd)), "fwdpair")
        L.check(lib.tspm_conv_fwd_pair(
            ctypes.byref(c1.shape), ctypes.byref(a1), x_ptr, ctypes.byref(strides), self._w(c1).data_ptr(),
            bp.y1.data_ptr(), ctypes.byref(b1) if b1 is not None else None, self.ws_conv.data_ptr(), self.ws_conv_bytes,
            ctypes.byref(cd.shape), ctypes.byref(ad), x_ptr, ctypes.byref(strides), self._w(cd).data_ptr(),
            bp.yd.data_ptr(), ctypes.byref(b2) if b2 is not None else None, self.ws_conv2.data_ptr(),
            self.ws_conv_bytes, sh), "conv_fwd_pair")
        if self.conv_timer:
            self.conv_timer.end()
        return True

    def _merge_in_apply(self, op: ConvOp, bn: BNOp) -> bool:
        """The conv cannot merge bn's statistics in-launch and the apply can (tspm_bn_apply_merge): the conv then only
        writes its partial tiles and the apply merges them (bn.pending)."""
        if not self.apply_merge or self.bn_two_level or bn.channels % 16:
            return False
        if op.bn_inlaunch is None:
            lib = L.lib()
            op.bn_inlaunch = bool(lib.tspm_conv_fwd_bn_inlaunch(ctypes.byref(op.shape), ctypes.byref(op.algo_fwd)))
        return not op.bn_inlaunch and op.stat_tiles()[0] <= 256

    def _conv_bn(self, op: ConvOp, bn: BNOp, x_ptr: int, strides: L.Strides4, y: torch.Tensor, sh: int,
                 merge_ok: bool = False) -> None:
        """conv forward whose epilogue emits the BN partial statistics and, in its last workgroup
        per channel block, merges them (save_mean/invstd + running statistics): one launch.  When the merge cannot
        run in-launch, the partials are left for the apply (round 6)."""
        if merge_ok and self._merge_in_apply(op, bn):  # (bn1 / bn2 of a block: their apply is tspm_bn_apply)
            bnf = self._bnf(bn)
            bnf.counters = None
            self._conv_fwd(op, x_ptr, strides, y, sh, bnf)
            bn.pending = op.stat_tiles()
            return
        self._conv_fwd(op, x_ptr, strides, y, sh, self._bnf(bn))

    def _apply(self, bn: BNOp, y, out, res_mode=0, res=None, bn2: Optional[BNOp] = None, relu=True, sh=0, train=True,
               pooled: Optional[torch.Tensor] = None):
        lib = L.lib()
        m = bn.module
        if pooled is not None:  # the last block: the adaptive average pool in the same launch
            if train and bn.pending is not None:  # (its conv left the statistics to merge: the finalize launch)
                tiles, rpt = bn.pending
                bn.pending = None
                L.check(lib.tspm_bn_finalize(bn.rows, bn.channels, tiles, rpt, self.bn_part.data_ptr(),
                                             L.ptr(m.running_mean), L.ptr(m.running_var),
                                             BN_MOMENTUM if m.momentum is None else m.momentum, m.eps,
                                             bn.mean.data_ptr(), bn.invstd.data_ptr(), sh), "bn_finalize")
            h, w = self.final_hw
            m2 = bn2.module if bn2 else None
            if train:
                st = (bn.mean, bn.invstd, bn2.mean if bn2 else None, bn2.invstd if bn2 else None)
            else:
                st = (m.running_mean, m.running_var, m2.running_mean if m2 else None, m2.running_var if m2 else None)
            L.check(lib.tspm_bn_apply_pool(h * w, self.N, bn.channels, y.data_ptr(), st[0].data_ptr(), st[1].data_ptr(),
                                           m.weight.data_ptr(), m.bias.data_ptr(), res_mode, L.ptr(res), L.ptr(st[2]),
                                           L.ptr(st[3]), L.ptr(m2.weight) if m2 else None,
                                           L.ptr(m2.bias) if m2 else None, 1 if relu else 0, 0 if train else 1, m.eps,
                                           out.data_ptr(), pooled.data_ptr(), sh), "bn_apply_pool")
            return
        if train and bn.pending is not None:  # the statistics merge of the conv before, in this launch (round 6)
            tiles, rpt = bn.pending
            bn.pending = None
            L.check(lib.tspm_bn_apply_merge(bn.rows, bn.channels, tiles, rpt, self.bn_part.data_ptr(),
                                            L.ptr(m.running_mean), L.ptr(m.running_var),
                                            BN_MOMENTUM if m.momentum is None else m.momentum, m.eps,
                                            bn.mean.data_ptr(), bn.invstd.data_ptr(), y.data_ptr(), m.weight.data_ptr(),
                                            m.bias.data_ptr(), res_mode, L.ptr(res),
                                            L.ptr(bn2.mean) if bn2 else None, L.ptr(bn2.invstd) if bn2 else None,
                                            L.ptr(bn2.module.weight) if bn2 else None,
                                            L.ptr(bn2.module.bias) if bn2 else None, 1 if relu else 0, out.data_ptr(),
                                            sh), "bn_apply_merge")
        elif train:
            L.check(lib.tspm_bn_apply(bn.rows, bn.channels, y.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                                      m.weight.data_ptr(), m.bias.data_ptr(), res_mode, L.ptr(res),
                                      L.ptr(bn2.mean) if bn2 else None, L.ptr(bn2.invstd) if bn2 else None,
                                      L.ptr(bn2.module.weight) if bn2 else None, L.ptr(bn2.module.bias) if bn2 else None,
                                      1 if relu else 0, out.data_ptr(), None, 0, sh), "bn_apply")
        else:
            m2 = bn2.module if bn2 else None
            L.check(lib.tspm_bn_apply_eval(bn.rows, bn.channels, y.data_ptr(), m.running_mean.data_ptr(),
                                           m.running_var.data_ptr(), m.eps, m.weight.data_ptr(), m.bias.data_ptr(),
                                           res_mode, L.ptr(res), L.ptr(m2.running_mean) if m2 else None,
                                           L.ptr(m2.running_var) if m2 else None, L.ptr(m2.weight) if m2 else None,
                                           L.ptr(m2.bias) if m2 else None, 1 if relu else 0, out.data_ptr(), sh),
                    "bn_apply_eval")

    # ---------------------------------------------------------------------------------------
    def input_strides(self, x: torch.Tensor) -> L.Strides4:
        """Strides of the reference's NCHW ([N,H,W] or [N,1,H,W]) input, read in place by the stem."""
        if x.dim() == 3:
            sn, sh_, sw = x.stride()
            sc = 0
        else:
            sn, sc, sh_, sw = x.stride()
        return L.Strides4(sn, sh_, sw, sc)

    def check_input(self, x: torch.Tensor) -> None:
        L.require_cuda_f32(x, "encoder input")
        shp = tuple(x.shape)
        want3 = (self.N, self.H, self.W)
        want4 = (self.N, self.cin, self.H, self.W)
        if shp != want3 and shp != want4:
            raise L.TspmError(f"encoder input shape {shp} != planned {want4}")
        if x.dim() == 3 and self.cin != 1:
            raise L.TspmError("3-D input requires in_channels == 1 (resnet.py:201-203)")

    def forward(self, x: torch.Tensor, emb: torch.Tensor, ld_emb: int, train: bool = True,
                bump_batches_tracked: bool = True) -> None:
        """x: reference-layout input [N,H,W] / [N,C,H,W] fp32 on device; emb: [N, >=hidden] output view
        (row stride ld_emb) that receives the fc output.  In training mode every BatchNorm's
        num_batches_tracked is incremented (nn.BatchNorm2d semantics) unless the caller does it."""
        self.check_input(x)
        if train and bump_batches_tracked:
            nbt = [bn.module.num_batches_tracked for bn in self.all_bns() if bn.module.num_batches_tracked is not None]
            if nbt:
                torch._foreach_add_(nbt, 1)
        sh = L.stream_handle()
        lib = L.lib()
        N = self.N
        self.x_in = x
        xs = self.input_strides(x)
        p1, q1, p2, q2 = self.mp_shape
        C0 = self.stem.shape.k
        if train:
            self._conv_bn(self.stem, self.stem_bn, x.data_ptr(), xs, self.y0, sh)
        else:
            self._conv_fwd(self.stem, x.data_ptr(), xs, self.y0, sh)
        if self.stem_fuse:  # BN apply + ReLU + max pool in one launch (tspm_bn_apply_maxpool, ABI 19)
            m = self.stem_bn.module
            mean, inv = ((self.stem_bn.mean, self.stem_bn.invstd) if train else (m.running_mean, m.running_var))
            L.check(lib.tspm_bn_apply_maxpool(N, p1, q1, C0, self.y0.data_ptr(), mean.data_ptr(), inv.data_ptr(),
                                              m.weight.data_ptr(), m.bias.data_ptr(), 0 if train else 1, m.eps,
                                              self.a0.data_ptr(), self.mp.data_ptr(), self.mp_idx.data_ptr(), p2, q2,
                                              sh), "bn_apply_maxpool")
        else:
            self._apply(self.stem_bn, self.y0, self.a0, relu=True, sh=sh, train=train)
            L.check(lib.tspm_maxpool_fwd(N, p1, q1, C0, 3, 2, 1, p2, q2, self.a0.data_ptr(), self.mp.data_ptr(),
                                         self.mp_idx.data_ptr(), None, 0, sh), "maxpool_fwd")
        xin = self.mp
        for bp in self.blocks:
            pool = self.pooled if (bp is self.blocks[-1] and self.fuse_pool) else None
            s1 = bp.conv1.shape
            xs_in = L.hwnc_strides(N, s1.h, s1.w, s1.c)
            paired = bp.ds_conv is not None and self._fwd_pair(bp, xin.data_ptr(), xs_in, train, sh)
            if paired:
                pass
            elif train:
                self._conv_bn(bp.conv1, bp.bn1, xin.data_ptr(), xs_in, bp.y1, sh, merge_ok=True)
            else:
                self._conv_fwd(bp.conv1, xin.data_ptr(), xs_in, bp.y1, sh)
            s2 = bp.conv2.shape
            xs_a1 = L.hwnc_strides(N, s2.h, s2.w, s2.c)
            self._apply(bp.bn1, bp.y1, bp.a1, relu=True, sh=sh, train=train)
            if train:
                self._conv_bn(bp.conv2, bp.bn2, bp.a1.data_ptr(), xs_a1, bp.y2, sh, merge_ok=True)
            else:
                self._conv_fwd(bp.conv2, bp.a1.data_ptr(), xs_a1, bp.y2, sh)
            if bp.ds_conv is not None:
                if paired:
                    pass
                elif train:
                    self._conv_bn(bp.ds_conv, bp.ds_bn, xin.data_ptr(), xs_in, bp.yd, sh)
                else:
                    self._conv_fwd(bp.ds_conv, xin.data_ptr(), xs_in, bp.yd, sh)
                self._apply(bp.bn2, bp.y2, bp.out, res_mode=2, res=bp.yd, bn2=bp.ds_bn, relu=True, sh=sh, train=train,
                            pooled=pool)
            else:
                self._apply(bp.bn2, bp.y2, bp.out, res_mode=1, res=xin, relu=True, sh=sh, train=train, pooled=pool)
            xin = bp.out
        if not self.fuse_pool:
            h, w = self.final_hw
            L.check(lib.tspm_avgpool_fwd(h * w, N, self.final_c, xin.data_ptr(), self.pooled.data_ptr(), sh),
                    "avgpool_fwd")
        fc = self.enc.fc
        ks = self.fc_splits
        if ks > 1:  # split-K fc forward (partials + one reduce launch; A/B switch TSPM_FC_SPLITS)
            need = lib.tspm_linear_fwd_splitk_workspace(N, self.final_c, self.hidden, ks)
            if self._fc_ws is None or self._fc_ws.numel() < need:
                self._fc_ws = torch.empty(max(need, 16), dtype=torch.uint8, device=self.device)
            L.check(lib.tspm_linear_fwd_splitk(N, self.final_c, self.hidden, self.pooled.data_ptr(), self.final_c,
                                               fc.weight.data_ptr(), L.ptr(fc.bias), 0, None, 1.0, emb.data_ptr(),
                                               ld_emb, ks, self._fc_ws.data_ptr(), self._fc_ws.numel(), sh),
                    "linear_fwd_splitk(fc)")
        else:
            L.check(lib.tspm_linear_fwd(N, self.final_c, self.hidden, self.pooled.data_ptr(), self.final_c,
                                        fc.weight.data_ptr(), L.ptr(fc.bias), 0, None, 1.0, emb.data_ptr(), ld_emb,
                                        sh), "linear_fwd(fc)")

    # ---------------------------------------------------------------------------------------
    def _grad(self, p: torch.Tensor) -> torch.Tensor:
        return self.grad_of(p)

    def _bn_bwd(self, bn: BNOp, g, out_mask, y, dy, bn2: Optional[BNOp] = None, y2=None, dy2=None, dres=None, sh=0):
        lib = L.lib()
        m = bn.module
        gw, gb = self._grad(m.weight), self._grad(m.bias)
        if bn2 is not None:
            m2 = bn2.module
            gw2, gb2 = self._grad(m2.weight), self._grad(m2.bias)
        L.check(lib.tspm_bn_bwd(bn.rows, bn.channels, g.data_ptr(), L.ptr(out_mask), y.data_ptr(), bn.mean.data_ptr(),
                                bn.invstd.data_ptr(), m.weight.data_ptr(), gw.data_ptr(), gb.data_ptr(), dy.data_ptr(),
                                L.ptr(y2), L.ptr(bn2.mean) if bn2 else None, L.ptr(bn2.invstd) if bn2 else None,
                                L.ptr(bn2.module.weight) if bn2 else None, L.ptr(gw2) if bn2 else None,
                                L.ptr(gb2) if bn2 else None, L.ptr(dy2), L.ptr(dres), None, None, 0,
                                self.ws_bn.data_ptr(), self.ws_bn_bytes, sh), "bn_bwd")

    def _bn_bwd_part(self, bn: BNOp, g, out_mask, y, dy, bn2: Optional[BNOp] = None, y2=None, dy2=None, dres=None,
                     sh=0):
        """_bn_bwd whose partial sums the producing dgrad epilogue already wrote (bn.part, tspm_conv_bwd_ex): the
        apply launch alone (tspm_bn_bwd_apply_part)."""
        m = bn.module
        gw, gb = self._grad(m.weight), self._grad(m.bias)
        if bn2 is not None:
            m2 = bn2.module
            gw2, gb2 = self._grad(m2.weight), self._grad(m2.bias)
        L.check(L.lib().tspm_bn_bwd_apply_part(
            bn.rows, bn.channels, bn.rows // 32, bn.part.data_ptr(), g.data_ptr(), out_mask.data_ptr(), y.data_ptr(),
            bn.mean.data_ptr(), bn.invstd.data_ptr(), m.weight.data_ptr(), gw.data_ptr(), gb.data_ptr(), dy.data_ptr(),
            L.ptr(y2), L.ptr(bn2.mean) if bn2 else None, L.ptr(bn2.invstd) if bn2 else None,
            L.ptr(bn2.module.weight) if bn2 else None, L.ptr(gw2) if bn2 else None, L.ptr(gb2) if bn2 else None,
            L.ptr(dy2), L.ptr(dres), sh), "bn_bwd_apply_part")

    def _bnp_stem_desc(self) -> Optional["L.BnBwdPart"]:
        """The stem BN's partial-sum descriptor in max-pool gather mode (layer1's first conv1 data gradient writes the
        pool's output gradient), or None."""
        bn = self.stem_bn
        if (not self.bn_dgrad_part or not self.bnp_stem or bn.part is None or self.debug_hook is not None or not self.pool_src
                or bn.part.numel() // (3 * bn.channels) > self.bnp_max_tiles):
            return None
        p1, q1, _, _ = self.mp_shape
        return L.BnBwdPart(self.a0.data_ptr(), self.y0.data_ptr(), bn.mean.data_ptr(), None, None, bn.part.data_ptr(),
                           self.mp_idx.data_ptr(), p1, q1)

    def _bnp_desc(self, bp: "BlockPlan", which: int, dres: Optional[torch.Tensor] = None) -> Optional["L.BnBwdPart"]:
        """The partial-sum descriptor for bn1 (which=1) or bn2 (which=2) of block ``bp``, or None when that BN takes
        the partial pass.  For BNs of at most ``bnx_max_rows`` rows the descriptor asks for the whole BN backward in
        the epilogue (``.dy`` set: bn1 -> g_y1; bn2 -> g_y2 [+ g_yd], ``dres`` = the block-input gradient buffer of
        an identity block)."""
        bn = bp.bn1 if which == 1 else bp.bn2
        if not self.bn_dgrad_part or bn.part is None or self.debug_hook is not None or bn.rows // 32 > self.bnp_max_tiles:
            return None
        if which == 1:
            d = L.BnBwdPart(bp.a1.data_ptr(), bp.y1.data_ptr(), bn.mean.data_ptr(), None, None, bn.part.data_ptr())
        else:
            two = bp.ds_conv is not None
            d = L.BnBwdPart(bp.out.data_ptr(), bp.y2.data_ptr(), bn.mean.data_ptr(), bp.yd.data_ptr() if two else None,
                            bp.ds_bn.mean.data_ptr() if two else None, bn.part.data_ptr())
        if bn.rows <= self.bnx_max_rows:
            m = bn.module
            d.invstd, d.gamma = bn.invstd.data_ptr(), m.weight.data_ptr()
            d.dgamma, d.dbeta = self._grad(m.weight).data_ptr(), self._grad(m.bias).data_ptr()
            d.dy = (bp.g_y1 if which == 1 else bp.g_y2).data_ptr()
            d.counters = bn.cnt.data_ptr()
            if which == 2 and bp.ds_conv is not None:
                m2 = bp.ds_bn.module
                d.invstd2, d.gamma2 = bp.ds_bn.invstd.data_ptr(), m2.weight.data_ptr()
                d.dgamma2, d.dbeta2 = self._grad(m2.weight).data_ptr(), self._grad(m2.bias).data_ptr()
                d.dy2 = bp.g_yd.data_ptr()
            elif which == 2:
                d.dres = dres.data_ptr()
        return d

    def _bn_bwd_src(self, bn: BNOp, src: "L.BnGSrc", out_mask, y, dy, bn2: Optional[BNOp] = None, y2=None, dy2=None,
                    dres=None, sh=0):
        """_bn_bwd with the incoming gradient formed on the fly from a pooling layer's output gradient
        (tspm_bn_bwd_src, ABI 19): the encoder's last BN reads the average pool's gradient, the stem's BN the
        max pool's — the pooling backward's launch and its [rows, C] gradient tensor disappear."""
        lib = L.lib()
        m = bn.module
        gw, gb = self._grad(m.weight), self._grad(m.bias)
        if bn2 is not None:
            m2 = bn2.module
            gw2, gb2 = self._grad(m2.weight), self._grad(m2.bias)
        L.check(lib.tspm_bn_bwd_src(bn.rows, bn.channels, ctypes.byref(src), L.ptr(out_mask), y.data_ptr(),
                                    bn.mean.data_ptr(), bn.invstd.data_ptr(), m.weight.data_ptr(), gw.data_ptr(),
                                    gb.data_ptr(), dy.data_ptr(), L.ptr(y2), L.ptr(bn2.mean) if bn2 else None,
                                    L.ptr(bn2.invstd) if bn2 else None, L.ptr(bn2.module.weight) if bn2 else None,
                                    L.ptr(gw2) if bn2 else None, L.ptr(gb2) if bn2 else None, L.ptr(dy2), L.ptr(dres),
                                    self.ws_bn.data_ptr(), self.ws_bn_bytes, sh), "bn_bwd_src")

    def _wgrad(self, op: ConvOp, x_ptr: int, strides: L.Strides4, dy: torch.Tensor, sh: int) -> None:
        gw = self._grad(op.module.weight)
        if not gw.is_contiguous(memory_format=torch.channels_last):
            raise L.TspmError("conv weight grad must be OHWI (channels_last)")
        if self.conv_timer:
            self.conv_timer.begin(op, "wgrad")
        aw = self._a(op.algo_wgrad)
        L.check(L.lib().tspm_conv_wgrad(ctypes.byref(op.shape), ctypes.byref(aw), x_ptr, ctypes.byref(strides),
                                        dy.data_ptr(), gw.data_ptr(), self.ws_conv.data_ptr(), self.ws_conv_bytes, sh),
                "conv_wgrad")
        if self.conv_timer:
            self.conv_timer.end()

    def _bwd_pair(self, op: ConvOp, x_ptr: int, strides: L.Strides4, dy: torch.Tensor, dx: torch.Tensor, beta: int,
                  sh: int, carry_share: float = 0.0, bnp: Optional["L.BnBwdPart"] = None) -> bool:
        """Input and weight gradient of ``op`` in one launch (tspm_conv_bwd: the two GEMMs read the same
        dy and are independent, so their workgroups share the grid).  False (nothing launched) when the
        pair is not built in or the tuner found the two separate launches faster; the caller then launches
        the two separately."""
        lib = L.lib()
        if op.bwd_fused is None:
            op.bwd_fused = bool(lib.tspm_conv_bwd_supported(ctypes.byref(op.shape), ctypes.byref(op.algo_dgrad),
                                                            ctypes.byref(op.algo_wgrad), ctypes.byref(strides)))
        if not op.bwd_fused:
            return False
        gw = self._grad(op.module.weight)
        if not gw.is_contiguous(memory_format=torch.channels_last):
            raise L.TspmError("conv weight grad must be OHWI (channels_last)")
        if self.conv_timer:
            self.conv_timer.begin(op, "bwd")
        job = self.adam_carry.take(carry_share) if self.adam_carry is not None else None
        ad, aw = self._a(op.algo_dgrad), self._a(op.algo_wgrad)
        if bnp is not None:  # the consuming BN's partial sums in the dgrad epilogue (+ the carried Adam job, if any)
            L.check(lib.tspm_conv_bwd_ex(ctypes.byref(op.shape), ctypes.byref(ad), ctypes.byref(aw), x_ptr,
                                         ctypes.byref(strides), dy.data_ptr(), self._w(op).data_ptr(), dx.data_ptr(),
                                         beta, gw.data_ptr(), ctypes.byref(job) if job is not None else None,
                                         ctypes.byref(bnp), self.ws_conv.data_ptr(), self.ws_conv_bytes,
                                         self.ws_conv2.data_ptr(), self.ws_conv_bytes, sh), "conv_bwd_ex")
        elif job is not None:  # an Adam update over earlier-finished parameters rides on this launch (ABI 20)
            L.check(lib.tspm_conv_bwd_adam(ctypes.byref(op.shape), ctypes.byref(ad), ctypes.byref(aw), x_ptr, ctypes.byref(strides), dy.data_ptr(),
                                           self._w(op).data_ptr(), dx.data_ptr(), beta, gw.data_ptr(), ctypes.byref(job),
                                           self.ws_conv.data_ptr(), self.ws_conv_bytes, self.ws_conv2.data_ptr(),
                                           self.ws_conv_bytes, sh), "conv_bwd_adam")
        else:
            L.check(lib.tspm_conv_bwd(ctypes.byref(op.shape), ctypes.byref(ad), ctypes.byref(aw),
                                      x_ptr, ctypes.byref(strides), dy.data_ptr(), self._w(op).data_ptr(), dx.data_ptr(),
                                      beta, gw.data_ptr(), self.ws_conv.data_ptr(), self.ws_conv_bytes,
                                      self.ws_conv2.data_ptr(), self.ws_conv_bytes, sh), "conv_bwd")
        if self.conv_timer:
            self.conv_timer.end()
        return True

    def _quad_algos(self, bp: "BlockPlan") -> Tuple[L.ConvAlgo, L.ConvAlgo]:
        """The downsample's (dgrad, wgrad) algos inside a quad launch: conv2's tile shapes, no dgrad split (one 1x1
        tap), conv2's weight-gradient split (the same reduction over the output rows)."""
        d, w = bp.conv2.algo_dgrad, bp.conv2.algo_wgrad
        return (L.ConvAlgo(d.tm, d.tn, d.wn, d.wk, 1, d.variant), L.ConvAlgo(w.tm, w.tn, w.wn, w.wk, w.splits, w.variant))

    def _bwd_quad(self, bp: "BlockPlan", xin: torch.Tensor, xs_in: L.Strides4, d2, da1, dd, Gnv, sh: int,
                  bnp: Optional["L.BnBwdPart"]) -> bool:
        """conv2's input + weight gradient (with bn1's partial sums when bnp) and the downsample's input gradient (into
        the block-input gradient, beta 0) + weight gradient in ONE launch (tspm_conv_bwd_quad); False = not supported
        (nothing launched)."""
        lib = L.lib()
        c2, cd = bp.conv2, bp.ds_conv
        s2 = c2.shape
        xs_a1 = L.hwnc_strides(self.N, s2.h, s2.w, s2.c)
        ad, aw = self._a(c2.algo_dgrad), self._a(c2.algo_wgrad)
        qd, qw = self._quad_algos(bp)
        qd, qw = self._a(qd), self._a(qw)
        if c2.bwd_fused is None:  # decided once, as _bwd_pair does: the eager and the captured steps agree
            c2.bwd_fused = bool(lib.tspm_conv_bwd_supported(ctypes.byref(s2), ctypes.byref(c2.algo_dgrad),
                                                            ctypes.byref(c2.algo_wgrad), ctypes.byref(xs_a1)))
        if (not self.bwd_quad or not c2.bwd_fused or
                not lib.tspm_conv_bwd_quad_supported(ctypes.byref(s2), ctypes.byref(ad), ctypes.byref(aw),
                                                     ctypes.byref(xs_a1), ctypes.byref(cd.shape), ctypes.byref(qd),
                                                     ctypes.byref(qw), ctypes.byref(xs_in))):
            return False
        g2, gd = self._grad(c2.module.weight), self._grad(cd.module.weight)
        job = self.adam_carry.take(0.5) if self.adam_carry is not None else None
        b = self.ws_conv_bytes
        if self.conv_timer:
            from .roofline import OpGroup
            self.conv_timer.begin(OpGroup((c2, cd)), "bwdquad")
        L.check(lib.tspm_conv_bwd_quad(
            ctypes.byref(s2), ctypes.byref(ad), ctypes.byref(aw), bp.a1.data_ptr(), ctypes.byref(xs_a1), d2.data_ptr(),
            self._w(c2).data_ptr(), da1.data_ptr(), 0, g2.data_ptr(), ctypes.byref(bnp) if bnp is not None else None,
            self.ws_conv.data_ptr(), b, self.ws_conv2.data_ptr(), b, ctypes.byref(cd.shape), ctypes.byref(qd),
            ctypes.byref(qw), xin.data_ptr(), ctypes.byref(xs_in), dd.data_ptr(), self._w(cd).data_ptr(), Gnv.data_ptr(),
            gd.data_ptr(), self.ws_conv3.data_ptr(), b, self.ws_conv4.data_ptr(), b,
            ctypes.byref(job) if job is not None else None, sh), "conv_bwd_quad")
        if self.conv_timer:
            self.conv_timer.end()
        return True

    def _dgrad(self, op: ConvOp, dy: torch.Tensor, dx: torch.Tensor, beta: int, sh: int) -> None:
        if self.conv_timer:
            self.conv_timer.begin(op, "dgrad")
        ad = self._a(op.algo_dgrad)
        L.check(L.lib().tspm_conv_dgrad(ctypes.byref(op.shape), ctypes.byref(ad), dy.data_ptr(),
                                        self._w(op).data_ptr(), dx.data_ptr(), beta, self.ws_conv.data_ptr(),
                                        self.ws_conv_bytes, sh), "conv_dgrad")
        if self.conv_timer:
            self.conv_timer.end()

    def block_params(self, bp: "BlockPlan") -> List[torch.nn.Parameter]:
        ms = [bp.conv1.module, bp.bn1.module, bp.conv2.module, bp.bn2.module]
        if bp.ds_conv is not None:
            ms += [bp.ds_conv.module, bp.ds_bn.module]
        return [p for m in ms for p in m.parameters(recurse=False)]

    def phase_params(self, phase: int) -> List[torch.nn.Parameter]:
        """Parameters whose gradients backward phase `phase` (1 or 2) writes: phase 1 = fc and the
        blocks from layer3 on, phase 2 = layer1, layer2 and the stem."""
        split = self.split_block
        mods = []
        if phase == 1:
            mods = [self.enc.fc] + [bp for bp in self.blocks[split:]]
        else:
            mods = [self.enc.conv1, self.enc.bn1] + [bp for bp in self.blocks[:split]]
        out = []
        for m in mods:
            if isinstance(m, BlockPlan):
                ms = [m.conv1.module, m.bn1.module, m.conv2.module, m.bn2.module]
                if m.ds_conv is not None:
                    ms += [m.ds_conv.module, m.ds_bn.module]
            else:
                ms = [m]
            for mm in ms:
                out += [p for p in mm.parameters(recurse=False)]
        return out

    def backward(self, g_emb: Optional[torch.Tensor], ld_g: int, phase: int = 0) -> None:
        """g_emb: [N, hidden] gradient of the fc output (row stride ld_g).  Writes every parameter
        gradient of the encoder (overwrite semantics) through ``grad_of``.  phase 0 runs the whole
        backward; phase 1 the fc and the blocks from ``split_block`` (first block of layer3) on,
        phase 2 (g_emb unused) the remaining blocks and the stem — the DP exchange of phase 1's
        gradients overlaps phase 2."""
        sh = L.stream_handle()
        lib = L.lib()
        N = self.N
        if phase in (0, 1):
            self._bnp_ready = set()
            self._bnx_done = set()
            fc = self.enc.fc
            linear_bwd(N, self.final_c, self.hidden, self.pooled.data_ptr(), self.final_c, g_emb.data_ptr(), ld_g,
                       fc.weight.data_ptr(), self._grad(fc.weight).data_ptr(),
                       self._grad(fc.bias).data_ptr() if fc.bias is not None else None, self.g_pooled.data_ptr(),
                       self.final_c, sh)
            if self.adam_carry is not None:
                self.adam_carry.ready([p for p in fc.parameters()])
            h, w = self.final_hw
            G, Gn = self.gA, self.gB
            # the last BN reads the average pool's gradient directly (no broadcast tensor) unless a debug hook
            # wants the materialised block-output gradient
            pool_src = None
            if self.pool_src and self.debug_hook is None:
                pool_src = L.BnGSrc(kind=L.GSRC_AVGPOOL, n=N, h=h, w=w, p=0, q=0, npos=h * w, ldg=self.final_c,
                                    gp=self.g_pooled.data_ptr(), idx=None)
            else:
                L.check(lib.tspm_avgpool_bwd(h * w, N, self.final_c, self.g_pooled.data_ptr(), self.final_c,
                                             G.data_ptr(), sh), "avgpool_bwd")
            lo, hi = (self.split_block if phase == 1 else 0), len(self.blocks)
        else:
            G, Gn = self._bw_state
            lo, hi = 0, self.split_block
        for i in range(hi - 1, lo - 1, -1):
            bp = self.blocks[i]
            xin = self.blocks[i - 1].out if i > 0 else self.mp
            s1 = bp.conv1.shape
            xs_in = L.hwnc_strides(N, s1.h, s1.w, s1.c)
            n_out = bp.out.numel()
            n_in = xin.numel()
            Gv = G[:n_out]
            Gnv = Gn[:n_in]
            d2 = bp.g_y2
            src = pool_src if (phase in (0, 1) and i == len(self.blocks) - 1) else None
            # bn2's partial sums came with the gradient when the next block's conv1 backward wrote them (round 6) —
            # or its whole backward did (then no launch here)
            bn2_fn = self._bn_bwd_part if (src is None and id(bp.bn2) in self._bnp_ready) else self._bn_bwd
            bn2_done = src is None and id(bp.bn2) in self._bnx_done
            self._bnp_ready.discard(id(bp.bn2))
            self._bnx_done.discard(id(bp.bn2))
            if bp.ds_conv is not None:
                dd = bp.g_yd
                if bn2_done:
                    pass
                elif src is not None:
                    self._bn_bwd_src(bp.bn2, src, bp.out, bp.y2, d2, bn2=bp.ds_bn, y2=bp.yd, dy2=dd, sh=sh)
                else:
                    bn2_fn(bp.bn2, Gv, bp.out, bp.y2, d2, bn2=bp.ds_bn, y2=bp.yd, dy2=dd, sh=sh)
            elif bn2_done:
                pass
            elif src is not None:
                self._bn_bwd_src(bp.bn2, src, bp.out, bp.y2, d2, dres=Gnv, sh=sh)
            else:
                # identity residual: g' goes straight to the block-input gradient buffer
                bn2_fn(bp.bn2, Gv, bp.out, bp.y2, d2, dres=Gnv, sh=sh)
            s2 = bp.conv2.shape
            xs_a1 = L.hwnc_strides(N, s2.h, s2.w, s2.c)
            da1 = self.da1[:n_out]
            bnp1 = self._bnp_desc(bp, 1)
            # downsampling block: conv2's backward and the downsample's in one launch when supported (round 6)
            quad = bp.ds_conv is not None and self._bwd_quad(bp, xin, xs_in, d2, da1, dd, Gnv, sh, bnp1)
            if quad:
                bnp1_done = bnp1 is not None
            elif self._bwd_pair(bp.conv2, bp.a1.data_ptr(), xs_a1, d2, da1, 0, sh, carry_share=0.5, bnp=bnp1):
                bnp1_done = bnp1 is not None
            else:
                self._wgrad(bp.conv2, bp.a1.data_ptr(), xs_a1, d2, sh)
                self._dgrad(bp.conv2, d2, da1, 0, sh)
                bnp1_done = False
            d1 = bp.g_y1
            if bnp1_done and bnp1.dy:
                pass  # the whole bn1 backward ran in conv2's dgrad epilogue
            elif bnp1_done:
                self._bn_bwd_part(bp.bn1, da1, bp.a1, bp.y1, d1, sh=sh)
            else:
                self._bn_bwd(bp.bn1, da1, bp.a1, bp.y1, d1, sh=sh)
            if self.debug_hook is not None:
                self.debug_hook(f"block{i}.g_out", Gv)
                self.debug_hook(f"block{i}.d_y2", d2)
                self.debug_hook(f"block{i}.d_a1", da1)
                self.debug_hook(f"block{i}.d_y1", d1)
            # the downsample's input gradient overwrites Gnv before conv1's accumulates onto it
            if bp.ds_conv is not None and not quad and not self._bwd_pair(bp.ds_conv, xin.data_ptr(), xs_in, dd, Gnv, 0, sh):
                self._wgrad(bp.ds_conv, xin.data_ptr(), xs_in, dd, sh)
                self._dgrad(bp.ds_conv, dd, Gnv, 0, sh)
            # conv1's input gradient accumulates last onto the previous block's output gradient (whose bn2 partial sums
            # its epilogue forms, round 6)
            # (block i-1's identity-residual dres goes to this block's output-gradient buffer G, free once bn2 above ran)
            bnp2 = self._bnp_desc(self.blocks[i - 1], 2, dres=G[:n_in]) if i > 0 else self._bnp_stem_desc()
            if self._bwd_pair(bp.conv1, xin.data_ptr(), xs_in, d1, Gnv, 1, sh, carry_share=1.0, bnp=bnp2):
                if bnp2 is not None:
                    tgt = id(self.blocks[i - 1].bn2 if i > 0 else self.stem_bn)
                    (self._bnx_done if bnp2.dy else self._bnp_ready).add(tgt)
            else:
                self._wgrad(bp.conv1, xin.data_ptr(), xs_in, d1, sh)
                self._dgrad(bp.conv1, d1, Gnv, 1, sh)
            if self.adam_carry is not None:  # this block's parameters are final and read by no later launch
                self.adam_carry.ready(self.block_params(bp))
            G, Gn = Gn, G
        if phase == 1:
            self._bw_state = (G, Gn)
            return
        # stem: maxpool -> relu/bn -> conv1 (weight grad only)
        p1, q1, p2, q2 = self.mp_shape
        C0 = self.stem.shape.k
        if self.pool_src:  # the stem BN reads the max pool's gradient through its argmax taps (no g_stem tensor)
            src = L.BnGSrc(kind=L.GSRC_MAXPOOL, n=N, h=p1, w=q1, p=p2, q=q2, npos=0, ldg=0, gp=G.data_ptr(),
                           idx=self.mp_idx.data_ptr())
            if id(self.stem_bn) in self._bnp_ready:  # its partial sums came with layer1's first data gradient
                self._bnp_ready.discard(id(self.stem_bn))
                bn, m = self.stem_bn, self.stem_bn.module
                L.check(lib.tspm_bn_bwd_apply_part_src(
                    bn.rows, bn.channels, bn.part.numel() // (3 * bn.channels), bn.part.data_ptr(), ctypes.byref(src),
                    self.a0.data_ptr(), self.y0.data_ptr(), bn.mean.data_ptr(), bn.invstd.data_ptr(),
                    m.weight.data_ptr(), self._grad(m.weight).data_ptr(), self._grad(m.bias).data_ptr(),
                    self.dy_stem.data_ptr(), sh), "bn_bwd_apply_part_src")
            else:
                self._bn_bwd_src(self.stem_bn, src, self.a0, self.y0, self.dy_stem, sh=sh)
        else:
            if self.g_stem is None:  # pool_src switched off after construction
                self.g_stem = torch.empty(self.a0.numel(), device=self.device, dtype=torch.float32)
            L.check(lib.tspm_maxpool_bwd(N, p1, q1, C0, 3, 2, 1, p2, q2, G.data_ptr(), self.mp_idx.data_ptr(),
                                         self.g_stem.data_ptr(), sh), "maxpool_bwd")
            self._bn_bwd(self.stem_bn, self.g_stem, self.a0, self.y0, self.dy_stem, sh=sh)
        self._wgrad(self.stem, self.x_in.data_ptr(), self.input_strides(self.x_in), self.dy_stem, sh)


def _default_grad_of(p: torch.Tensor) -> torch.Tensor:
    """Return p.grad, (re)allocating it in p's memory format when absent."""
    g = p.grad
    if g is None or g.shape != p.shape:
        fmt = torch.channels_last if (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last)
                                      and not p.is_contiguous()) else torch.contiguous_format
        if p.dim() == 4:
            fmt = torch.channels_last
        g = torch.empty_like(p, memory_format=fmt)
        p.grad = g
    return g


def prepare_encoder_layout(encoder: torch.nn.Module) -> None:
    """Re-lay every conv weight of the encoder as OHWI (channels_last view of the OIHW parameter).
    Shapes, values and state_dict keys are unchanged."""
    for m in encoder.modules():
        if isinstance(m, torch.nn.Conv2d):
            w = m.weight
            if not w.is_contiguous(memory_format=torch.channels_last):
                w.data = w.data.contiguous(memory_format=torch.channels_last)
            if w.grad is not None and not w.grad.is_contiguous(memory_format=torch.channels_last):
                w.grad = w.grad.contiguous(memory_format=torch.channels_last)
