"""ctypes binding of libtspm.so (the C ABI declared in ``include/tspm.h``).

This is the "reference-side binding" of the drop-in boundary: plain device pointers, sizes and a
hipStream_t cross the ABI; PyTorch only supplies device memory and the current stream.  The library
is loaded lazily and every call checks its status code — there is no fallback: a missing or broken
library raises ``TspmLibraryError`` (the product path never silently runs on ATen or the CPU).
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import POINTER, Structure, c_float, c_int32, c_int64, c_size_t, c_uint64, c_void_p
from typing import Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSPM_LIB", os.path.join(_HERE, "libtspm.so"))
ABI_VERSION = 22
COUNTER_BYTES = 65536     # TSPM_COUNTER_BYTES: arrival-counter header of a split wgrad workspace


class TspmLibraryError(RuntimeError):
    pass


class TspmError(RuntimeError):
    pass


class ConvShape(Structure):
    _fields_ = [(n, c_int32) for n in ("n", "h", "w", "c", "k", "r", "s", "stride", "pad", "p", "q")]


ALGO_HANDOFF_ACQUIRE = 1  # tspm_conv_algo.flags (ABI 21)


class ConvAlgo(Structure):
    """tspm_conv_algo: (tm, tn, wn, wk, splits[, variant[, lds_floor, flags]]); variant 1 = LDS-staged kernels.
    lds_floor / flags (ABI 21) are per-call launch options: the LDS floor (scheduling only) and the hand-off mode."""
    _fields_ = [(n, c_int32) for n in ("tm", "tn", "wn", "wk", "splits", "variant", "lds_floor", "flags")]

    def with_options(self, lds_floor: int = 0, flags: int = 0) -> "ConvAlgo":
        """A copy with the per-call launch options set (the tile configuration unchanged)."""
        return ConvAlgo(self.tm, self.tn, self.wn, self.wk, self.splits, self.variant, int(lds_floor), int(flags))


class Strides4(Structure):
    _fields_ = [(n, c_int64) for n in ("sn", "sh", "sw", "sc")]


class BnFuse(Structure):
    """tspm_bn_fuse: BatchNorm statistics produced by the conv forward epilogue."""
    _fields_ = [("partial", c_void_p), ("counters", c_void_p), ("running_mean", c_void_p),
                ("running_var", c_void_p), ("momentum", c_float), ("eps", c_float), ("save_mean", c_void_p),
                ("save_invstd", c_void_p), ("counters_len", c_int32), ("reserved_", c_int32),
                ("partial_floats", c_int64)]


class AdamJob(ctypes.Structure):
    """tspm_adam_job (ABI 20): an Adam update over `count` elements of FusedAdam's flat buffers (pointers at the
    range start) carried by `blocks` extra workgroups of a tspm_conv_bwd_adam launch."""
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("count", ctypes.c_int64), ("hyper", ctypes.c_void_p),
                ("blocks", ctypes.c_int32), ("pad_", ctypes.c_int32)]


class BnBwdPart(Structure):
    """tspm_bn_bwd_part (ABI 21, round 6): the BN backward's partial sums formed by the dgrad epilogue that writes its
    incoming gradient (tspm_conv_bwd_ex), consumed by tspm_bn_bwd_apply_part."""
    _fields_ = [(n, c_void_p) for n in ("out", "y", "mean", "y2", "mean2", "part", "idx")] + \
        [("pool_h", c_int32), ("pool_w", c_int32)] + \
        [(n, c_void_p) for n in ("invstd", "gamma", "dgamma", "dbeta", "dy", "invstd2", "gamma2", "dgamma2", "dbeta2",
                                 "dy2", "dres", "counters")]


class BnGSrc(Structure):
    """tspm_bn_gsrc (ABI 19): a pooling layer's output gradient as the BN backward's gradient source."""
    _fields_ = [(n, c_int32) for n in ("kind", "n", "h", "w", "p", "q", "npos", "ldg")] + \
        [("gp", c_void_p), ("idx", c_void_p)]


GSRC_AVGPOOL, GSRC_MAXPOOL = 1, 2


class AdamHyper(Structure):
    _fields_ = [("lr", ctypes.c_double), ("beta1", ctypes.c_double), ("beta2", ctypes.c_double),
                ("eps", ctypes.c_double), ("weight_decay", ctypes.c_double), ("grad_scale", ctypes.c_double),
                ("step", c_int64), ("pad_", c_int64)]

HYPER_STEP_OFFSET = 48  # byte offset of tspm_adam_hyper.step


class LinearBwdDesc(Structure):
    """tspm_linear_bwd_desc: one Linear's backward for tspm_linear_bwd_multi."""
    _fields_ = [(n, c_int32) for n in ("n", "in_", "out", "ldx", "ldy", "lddx")] + \
               [(n, c_void_p) for n in ("x", "dy", "w", "dw", "db", "dx")]


class HeadDesc(Structure):
    """tspm_head_desc (ABI 16; adam_step ABI 20; rows_per_block ABI 21): the AVMNIST fusion head's train step in
    two launches."""
    _fields_ = [(n, c_int32) for n in ("n", "in_", "hidden", "hidden2", "classes", "ldx", "lddx", "gen_keep")] + \
        [(n, c_void_p) for n in ("x", "w0", "b0", "w3", "b3", "w5", "b5")] + \
        [("p", c_float), ("loss_weight", c_float), ("seed", c_uint64)] + \
        [(n, c_void_p) for n in ("counter", "keep", "labels", "h1", "hh", "logits", "dlogits", "dz3", "dz0", "dx",
                                 "row_ws", "gw0", "gb0", "gw3", "gb3", "gw5", "gb5", "loss", "stats", "adam_step")] + \
        [("rows_per_block", c_int32), ("reserved_", c_int32)]


# name -> (restype, argtypes)
_P = c_void_p
class LstmFwdDesc(Structure):
    """tspm_lstm_fwd_desc (ABI 12; argmax ABI 14)."""
    _fields_ = [(n, c_int32) for n in ("batch", "steps", "hidden", "ld_out")] + \
        [(n, c_void_p) for n in ("xg", "w_hh", "b_hh", "gates", "cs", "hs", "h_out", "argmax")]


class LstmBwdDesc(Structure):
    """tspm_lstm_bwd_desc (ABI 12; argmax ABI 14)."""
    _fields_ = [(n, c_int32) for n in ("batch", "steps", "hidden", "ld_dh")] + \
        [(n, c_void_p) for n in ("w_hh", "gates", "cs", "dh", "dgates", "argmax")]


_SIGS = {
    "tspm_abi_version": (c_int32, []),
    "tspm_status_string": (ctypes.c_char_p, [c_int32]),
    "tspm_conv_fwd": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo), _P, POINTER(Strides4), _P, _P, POINTER(BnFuse),
                                _P, c_size_t, _P]),
    "tspm_conv_fwd_tiles": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_fwd_tile_rows": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_fwd_bn_counters": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_fwd_bn_partial_floats": (c_int64, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_fwd_workspace": (c_size_t, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_dgrad": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo), _P, _P, _P, c_int32, _P, c_size_t, _P]),
    "tspm_conv_dgrad_workspace": (c_size_t, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_wgrad": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo), _P, POINTER(Strides4), _P, _P, _P, c_size_t, _P]),
    "tspm_conv_wgrad_workspace": (c_size_t, [POINTER(ConvShape), POINTER(ConvAlgo)]),
    "tspm_conv_bwd_supported": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo), POINTER(ConvAlgo), POINTER(Strides4)]),
    "tspm_conv_bwd": (c_int32, [POINTER(ConvShape), POINTER(ConvAlgo), POINTER(ConvAlgo), _P, POINTER(Strides4), _P, _P,
                                _P, c_int32, _P, _P, c_size_t, _P, c_size_t, _P]),
    "tspm_bn_stats": (c_int32, [c_int64, c_int32, _P, c_int32, c_int64, _P, _P, _P, c_float, c_float, _P, _P, _P,
                                c_size_t, _P]),
    "tspm_bn_stats_workspace": (c_size_t, [c_int64, c_int32]),
    "tspm_bn_finalize": (c_int32, [c_int64, c_int32, c_int32, c_int64, _P, _P, _P, c_float, c_float, _P, _P, _P]),
    "tspm_bn_apply": (c_int32, [c_int64, c_int32, _P, _P, _P, _P, _P, c_int32, _P, _P, _P, _P, _P, c_int32, _P, _P,
                                c_int64, _P]),
    "tspm_bn_apply_eval": (c_int32, [c_int64, c_int32, _P, _P, _P, c_float, _P, _P, c_int32, _P, _P, _P, _P, _P,
                                     c_int32, _P, _P]),
    # ABI 17: the last block's apply with the average pool folded in
    "tspm_bn_apply_pool": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, c_int32, _P, _P, _P, _P, _P,
                                     c_int32, c_int32, c_float, _P, _P, _P]),
    "tspm_bn_bwd": (c_int32, [c_int64, c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                              _P, _P, c_int64, _P, c_size_t, _P]),
    "tspm_bn_bwd_workspace": (c_size_t, [c_int64, c_int32]),
    # ABI 19: the stem's apply + ReLU + max pool in one launch; the BN backward reading a pooling layer's gradient
    # ABI 20: the fused backward launch carrying an Adam update over earlier-finished parameters
    "tspm_conv_bwd_adam": (c_int32, [_P] * 8 + [c_int32, _P, _P, _P, c_size_t, _P, c_size_t, _P]),
    "tspm_bn_apply_maxpool": (c_int32, [c_int32] * 4 + [_P] * 5 + [c_int32, c_float, _P, _P, _P, c_int32, c_int32, _P]),
    "tspm_bn_bwd_src": (c_int32, [c_int64, c_int32, POINTER(BnGSrc)] + [_P] * 17 + [c_size_t, _P]),
    # round 6: the BN backward's partial sums in the producing dgrad's epilogue, and the apply launch alone
    "tspm_conv_bwd_ex": (c_int32, [_P] * 8 + [c_int32, _P, _P, POINTER(BnBwdPart), _P, c_size_t, _P, c_size_t, _P]),
    "tspm_bn_bwd_apply_part": (c_int32, [c_int64, c_int32, c_int32] + [_P] * 18 + [_P]),
    "tspm_bn_bwd_apply_part_src": (c_int32, [c_int64, c_int32, c_int32] + [_P] * 10 + [_P]),
    # round 6: a downsampling block's first conv and its 1x1 downsample in one launch
    "tspm_conv_fwd_pair_supported": (c_int32, [_P] * 6),
    "tspm_conv_fwd_pair": (c_int32, [_P] * 7 + [_P, c_size_t] + [_P] * 7 + [_P, c_size_t, _P]),
    # round 6: the forward statistics merge in the apply's prologue
    "tspm_conv_fwd_bn_inlaunch": (c_int32, [_P, _P]),
    "tspm_bn_apply_merge": (c_int32, [c_int64, c_int32, c_int32, c_int64, _P, _P, _P, c_float, c_float] + [_P] * 5 +
                            [c_int32] + [_P] * 5 + [c_int32, _P, _P]),
    # round 6: a downsampling block's conv2 backward and its downsample's backward in one launch
    "tspm_conv_bwd_quad_supported": (c_int32, [_P] * 8),
    "tspm_conv_bwd_quad": (c_int32, [_P] * 8 + [c_int32, _P, _P, _P, c_size_t, _P, c_size_t] + [_P] * 9 +
                           [_P, c_size_t, _P, c_size_t, _P, _P]),
    "tspm_maxpool_fwd": (c_int32, [c_int32] * 9 + [_P, _P, _P, _P, c_int64, _P]),
    "tspm_maxpool_bwd": (c_int32, [c_int32] * 9 + [_P, _P, _P, _P]),
    "tspm_avgpool_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, _P, _P]),
    "tspm_avgpool_bwd": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, _P]),
    "tspm_linear_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, c_float, _P, c_int32, _P]),
    "tspm_linear_fwd_splitk": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, c_float, _P,
                                         c_int32, c_int32, _P, c_size_t, _P]),
    "tspm_linear_fwd_splitk_workspace": (c_size_t, [c_int32, c_int32, c_int32, c_int32]),
    "tspm_linear_bwd": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P, _P, _P, c_int32, _P]),
    "tspm_linear_bwd_multi": (c_int32, [c_int32, POINTER(LinearBwdDesc), _P]),
    "tspm_linear_bwd_data": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P]),
    "tspm_linear_bwd_weight": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P, _P]),
    "tspm_linear_bwd_weight_splitk": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P, c_int32,
                                                _P, c_size_t, _P]),
    "tspm_linear_bwd_weight_splitk_workspace": (c_size_t, [c_int32, c_int32, c_int32, c_int32]),
    "tspm_act_bwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, c_int32, c_float, _P]),
    "tspm_dropout_mask": (c_int32, [c_int64, c_float, c_uint64, _P, _P, _P]),
    "tspm_cross_entropy": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, c_float, _P, _P]),
    "tspm_counters_add": (c_int32, [_P, c_int64, c_int64, _P]),
    # ABI 16: the fusion head's train step (fwd + CE + bwd) in two launches
    "tspm_head_train_step": (c_int32, [POINTER(HeadDesc), _P]),
    # ABI 15: step flags (the DP step's exchange ordering across the graph boundary)
    "tspm_flag_create": (c_int32, [POINTER(c_void_p)]),
    "tspm_flag_destroy": (c_int32, [_P]),
    "tspm_flag_bump": (c_int32, [_P, _P]),
    "tspm_flag_host_wait": (c_int32, [_P, ctypes.c_uint64, c_int32]),
    "tspm_adam_begin": (c_int32, [_P, _P]),
    "tspm_adam_step": (c_int32, [c_int64, _P, _P, _P, _P, _P, _P]),
    "tspm_image_lut": (c_int32, [c_int64, _P, _P, _P, _P]),
    "tspm_avmnist_gather": (c_int32, [c_int64, _P, c_int64, _P, c_int32, _P, c_int32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tspm_classify_update": (c_int32, [c_int32, c_int32, _P, _P, _P, c_int32, _P, _P, _P, _P, _P, c_int64, _P]),
    "tspm_classify_update_ex": (c_int32, [c_int32, c_int32, _P, _P, _P, c_int32, _P, _P, _P, _P, _P, c_int64, c_int32,
                                          _P]),
    "tspm_reduce_slabs": (c_int32, [c_int64, c_int32, c_int64, _P, _P, _P]),
    "tspm_gmu_fwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, _P, c_int32, _P]),
    "tspm_pool_act_fwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, c_float, _P, _P, _P]),
    "tspm_pool_mix_fwd": (c_int32, [c_int32, c_int32, c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, c_int32, _P]),
    "tspm_pool_mix_bwd": (c_int32, [c_int32, c_int32, c_int32, c_int32, _P, c_int32, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tspm_pool_act_bwd": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, c_float, _P, _P]),
    "tspm_gmu_bwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, c_int32, _P, _P, _P, c_int32, _P, _P]),
    "tspm_maxout_fwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, c_float, _P, c_int32, _P]),
    "tspm_maxout_fwd_rng": (c_int32, [c_int32, c_int32, _P, c_int32, c_float, c_uint64, _P, c_int64, _P, c_float, _P,
                                      c_int32, _P]),
    "tspm_maxout_bwd": (c_int32, [c_int32, c_int32, _P, c_int32, _P, c_int32, _P, c_float, _P, c_int32, _P]),
    "tspm_bn1d_fwd": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, _P, c_float, c_float, _P, _P, _P, _P]),
    "tspm_bn1d_bwd": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tspm_bn1d_fwd_drop": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, _P, c_float, c_float, _P, _P, _P, c_float, _P,
                                     _P]),
    "tspm_bn1d_bwd_drop_relu": (c_int32, [c_int32, c_int32, _P, _P, c_float, _P, _P, _P, _P, _P, _P, _P, _P]),
    "tspm_bn1d_fwd_pair": (c_int32, [c_int32] + ([c_int32, _P, _P, _P, _P, _P, c_float, c_float, _P, _P, _P] * 2)
                           + [_P]),
    "tspm_bn1d_bwd_pair": (c_int32, [c_int32] + ([c_int32] + [_P] * 8) * 2 + [_P]),
    "tspm_linear_fwd_pair": (c_int32, [c_int32, c_int32, c_int32] + [_P, c_int32, _P, _P, c_int32] * 2 + [_P]),
    "tspm_bce_logits": (c_int32, [c_int32, c_int32, _P, _P, _P, _P, c_float, c_float, _P, _P]),
    # ABI 12: MOSI UTT-Fusion
    "tspm_adam_step_clip": (c_int32, [c_int64, _P, _P, _P, _P, _P, _P, _P]),
    "tspm_lstm_fwd": (c_int32, [c_int32, POINTER(LstmFwdDesc), _P]),
    "tspm_lstm_bwd": (c_int32, [c_int32, POINTER(LstmBwdDesc), _P]),
    "tspm_textcnn_pool_fwd": (c_int32, [c_int32, c_int32, c_int32, _P, c_int32, _P, _P, _P, c_float, _P, _P, _P,
                                        c_int32, _P]),
    "tspm_textcnn_bwd": (c_int32, [c_int32, c_int32, c_int32, c_int32, _P, c_int32, _P, _P, c_int32, _P, c_float, _P,
                                   _P, _P, _P, _P, _P]),
    "tspm_grad_clip_workspace": (c_size_t, []),
    "tspm_grad_clip_coef": (c_int32, [c_int64, _P, c_float, c_float, _P, _P, _P, c_size_t, _P]),
    "tspm_seq_gather": (c_int32, [c_int32, _P, c_int64, _P, _P, _P, c_int32, c_int32, _P, c_int64, c_int64, _P, _P, _P,
                                  _P]),
}

EXPORTED = tuple(_SIGS)

_lib = None
_lock = threading.Lock()


def load(path: Optional[str] = None):
    """Load libtspm.so (import torch first so the process shares torch's HIP runtime)."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise TspmLibraryError(
                f"libtspm.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C task-specific-pretraining-multimodal_amd/csrc`). There is no fallback path.")
        try:
            lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - environment specific
            raise TspmLibraryError(f"failed to load {p}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)  # AttributeError -> missing export = broken build
            fn.restype = res
            fn.argtypes = args
        v = lib.tspm_abi_version()
        if v != ABI_VERSION:
            raise TspmLibraryError(f"libtspm ABI version {v} != expected {ABI_VERSION}")
        if path is None:
            _lib = lib
        return lib


def lib():
    return _lib if _lib is not None else load()


def check(status: int, what: str) -> None:
    if status != 0:
        msg = lib().tspm_status_string(status).decode()
        raise TspmError(f"{what} failed: {msg} (status {status})")


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


_SHARED_STREAMS: dict = {}


def shared_streams(device, n: int = 3):
    """The process's side streams for the captured steps, created ONCE per device and reused by every step
    build.  A HIP stream is bound to one of the process's hardware queues (4 by default) when it is
    created; a step whose side stream shares the main stream's queue runs its two branches serially (one
    build in 24 ran 1.1 ms slower per step when each build took fresh pool streams, round 2).  With one
    set per process every step runs on the streams the first build measured."""
    dev = torch.device(device)
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    have = _SHARED_STREAMS.setdefault(key, [])
    while len(have) < n:
        have.append(torch.cuda.Stream(device=dev))
    return tuple(have[:n])


def require_cuda_f32(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise TspmError(f"{name} must be a ROCm device tensor (got {t.device}); the HIP path has no CPU fallback")
    if t.dtype != torch.float32:
        raise TspmError(f"{name} must be float32 (got {t.dtype})")


def hwnc_strides(n: int, h: int, w: int, c: int) -> Strides4:
    return Strides4(c, w * n * c, n * c, 1)


def counters_add(t: torch.Tensor, value: int = 1, stream: Optional[int] = None) -> None:
    """t (contiguous int64 on the device) += value in one libtspm launch (num_batches_tracked)."""
    if t.dtype != torch.int64 or not t.is_cuda or not t.is_contiguous():
        raise TspmError("counters_add: contiguous int64 device tensor")
    check(lib().tspm_counters_add(t.data_ptr(), t.numel(), int(value), stream_handle() if stream is None else stream),
          "counters_add")


class DeviceFlag:
    """A point inside a captured step graph the HOST can wait for: ``bump`` enqueues a one-thread kernel
    (+1 on a device counter, the new value stored to a coherent pinned host word); ``host_wait(v)`` spins
    (GIL released, in C) until the word reaches ``v``.  ROCm 7 refuses graph-external event records, the
    CUDA idiom, and a stream waiting on the word (hipStreamWaitValue64) stalled the graph's queues."""

    def __init__(self):
        h = c_void_p()
        check(lib().tspm_flag_create(ctypes.byref(h)), "flag_create")
        self.handle = h.value
        self.count = 0  # executions of the bump enqueued so far (host bookkeeping)

    def bump(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        sh = stream_handle() if stream is None else stream.cuda_stream
        check(lib().tspm_flag_bump(self.handle, sh), "flag_bump")

    def host_wait(self, value: int, timeout_ms: int = 60000) -> None:
        if not self.handle:
            raise TspmError("DeviceFlag used after close()")
        check(lib().tspm_flag_host_wait(self.handle, int(value), int(timeout_ms)), "flag_host_wait (timeout)")

    def close(self) -> None:
        """Free the flag's device word and pinned host word.  Only call this once no captured graph that
        bumps the flag can run again and the device is idle (``FusedTrainStep.close`` does both first):
        ``tspm_flag_destroy`` synchronises the device and frees memory."""
        h, self.handle = getattr(self, "handle", None), None
        if h and _lib is not None:
            check(_lib.tspm_flag_destroy(h), "flag_destroy")

    def __del__(self):
        # No HIP call at garbage-collection time: a collection can run while another stream is being
        # captured (where hipFree / hipHostFree are illegal), while a graph that bumps this flag is still
        # alive, or during the process group's teardown.  A flag nobody closed leaks its 128 bytes.
        self.handle = None


def linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream) -> None:
    """Backward of one nn.Linear (AVMNIST head / encoder fc, monomodal classifier, MMIMDb, MOSI): dw = dy^T @ x
    (+ db = column sums of dy) and, if dx is given, dx = dy @ w — ONE ``tspm_linear_bwd`` launch (bitwise the two
    separate products; 2.88 -> 2.81 ms per AVMNIST step when introduced)."""
    check(lib().tspm_linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream), "linear_bwd")


def graph_capture(graph: "torch.cuda.CUDAGraph"):
    """``torch.cuda.graph(graph)`` in thread-local capture mode — every captured step of this package uses it.
    In torch's default global mode any HIP call from ANOTHER thread during the capture is illegal, and
    torch.distributed's NCCL watchdog thread polls the end events of outstanding collectives with
    hipEventQuery: a step captured while an all-reduce of the previous (eager) step is still in the watchdog's
    list made that query fail with "operation not permitted when stream is capturing", the watchdog threw and
    the process aborted (round 4's abort in destroy_process_group, reproduced and read in round 5:
    gpurun_out/r5a_phased.err).  Thread-local mode forbids the unsafe calls only in the capturing thread."""
    return torch.cuda.graph(graph, capture_error_mode="thread_local")
