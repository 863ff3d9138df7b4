"""Algorithmic work accounting for the roofline numbers.

* Nominal dense conv FLOPs: 2 * P*Q*N * K * R*S*C per pass (fwd, dgrad, wgrad; no dgrad for the
  1-channel stems) — 1,049,740,032 FLOP/sample for the late-fusion step including the linears.
* Valid-tap FLOPs: only (output position, tap) pairs whose input pixel is inside the image —
  641,174,016 FLOP/sample.  The HIP kernels skip padding taps, so achieved MFMA throughput is
  quoted on the valid-tap count (it cannot exceed what the hardware executed).
"""
from __future__ import annotations

from typing import Iterable, Tuple


def _valid_1d(size_in: int, size_out: int, k: int, stride: int, pad: int) -> int:
    """Number of (output index, tap) pairs along one axis whose input index is in range."""
    n = 0
    for o in range(size_out):
        base = o * stride - pad
        for t in range(k):
            if 0 <= base + t < size_in:
                n += 1
    return n


def conv_macs(n, h, w, c, k, r, s, stride, pad) -> Tuple[int, int]:
    """(nominal MACs, valid-tap MACs) of one pass of a conv."""
    p = (h + 2 * pad - r) // stride + 1
    q = (w + 2 * pad - s) // stride + 1
    nominal = p * q * n * k * r * s * c
    valid = _valid_1d(h, p, r, stride, pad) * _valid_1d(w, q, s, stride, pad) * n * k * c
    return nominal, valid


def encoder_convs(layers, h: int, w: int, cin: int = 1):
    """Yield (name, conv shape tuple without batch) for a ResNet18/34 encoder on an h x w input."""
    def out(hh, ww, k, st, p):
        return (hh + 2 * p - k) // st + 1, (ww + 2 * p - k) // st + 1
    yield "stem", (h, w, cin, 64, 7, 7, 2, 3)
    h, w = out(h, w, 7, 2, 3)
    h, w = out(h, w, 3, 2, 1)
    c = 64
    for li, (planes, nb) in enumerate(zip((64, 128, 256, 512), layers)):
        for b in range(nb):
            st = 2 if (b == 0 and li > 0) else 1
            ho, wo = out(h, w, 3, st, 1)
            yield f"layer{li + 1}.{b}.conv1", (h, w, c, planes, 3, 3, st, 1)
            yield f"layer{li + 1}.{b}.conv2", (ho, wo, planes, planes, 3, 3, 1, 1)
            if b == 0 and (st != 1 or c != planes):
                yield f"layer{li + 1}.{b}.downsample", (h, w, c, planes, 1, 1, st, 0)
            h, w, c = ho, wo, planes


def step_flops_per_sample(audio_hw=(32, 94), image_hw=(28, 28), audio_hidden=64, image_hidden=128,
                          head_hidden=128) -> Tuple[int, int]:
    """(nominal, valid-tap) train-step FLOPs per sample: fwd + dgrad + wgrad, no stem dgrad."""
    nom = val = 0
    for layers, (h, w) in (((2, 2, 2, 2), audio_hw), ((3, 4, 6, 3), image_hw)):
        for name, (hh, ww, c, k, r, s, st, p) in encoder_convs(layers, h, w):
            a, b = conv_macs(1, hh, ww, c, k, r, s, st, p)
            passes = 2 if name == "stem" else 3
            nom += 2 * passes * a
            val += 2 * passes * b
    lin = 512 * audio_hidden + 512 * image_hidden + (audio_hidden + image_hidden) * head_hidden \
        + head_hidden * (head_hidden // 2) + (head_hidden // 2) * 10
    nom += 2 * 3 * lin
    val += 2 * 3 * lin
    return nom, val


def eval_flops_per_sample(audio_hw=(32, 94), image_hw=(28, 28), audio_hidden=64, image_hidden=128,
                          head_hidden=128) -> Tuple[int, int]:
    """(nominal, valid-tap) FLOPs per sample of the evaluation forward (validation_step)."""
    nom = val = 0
    for layers, (h, w) in (((2, 2, 2, 2), audio_hw), ((3, 4, 6, 3), image_hw)):
        for _, (hh, ww, c, k, r, s, st, p) in encoder_convs(layers, h, w):
            a, b = conv_macs(1, hh, ww, c, k, r, s, st, p)
            nom += 2 * a
            val += 2 * b
    lin = 512 * audio_hidden + 512 * image_hidden + (audio_hidden + image_hidden) * head_hidden \
        + head_hidden * (head_hidden // 2) + (head_hidden // 2) * 10
    return nom + 2 * lin, val + 2 * lin


def mono_flops_per_sample(layers=(2, 2, 2, 2), hw=(32, 94), hidden=64, classes=10) -> Tuple[int, int]:
    """(nominal, valid-tap) FLOPs per sample of the monomodal pre-training step (train_monomodal.py:
    97-260, default: ResNet18 audio + Linear(64, 10)): encoder fwd + dgrad + wgrad (no stem dgrad),
    encoder fc and classifier (3 passes each)."""
    nom = val = 0
    for name, (hh, ww, c, k, r, s, st, p) in encoder_convs(layers, hw[0], hw[1]):
        a, b = conv_macs(1, hh, ww, c, k, r, s, st, p)
        passes = 2 if name == "stem" else 3
        nom += 2 * passes * a
        val += 2 * passes * b
    lin = 512 * hidden + hidden * classes
    return nom + 6 * lin, val + 6 * lin


FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 dense peak
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E spec peak


# ------------------------------------------------------------------------------------------------
# Device-side kernel durations (measurement only; bench.py's roofline line)
# ------------------------------------------------------------------------------------------------
import re as _re

CONV_KERNEL = _re.compile(r"\bk_(fwd_lds|fwd_pair_lds|bwd_lds|bwd_quad_lds|dgrad_lds|wgrad_lds|fwd_x9|fwd_pair_x9|bwd_x9|bwd_quad_x9|dgrad_x9|wgrad_x9|conv_fwd_vec|conv_fwd_gather|conv_dgrad|"
                          r"conv_wgrad|conv_wgrad_t|stem_fwd|stem_wgrad|reduce_slabs|reduce_slabs_wide)\b")
CONV_SECONDARY = _re.compile(r"\bk_reduce_slabs(_wide)?\b")  # second kernel of a split-K wgrad launch (variant 0)


def device_kernels(run, replays: int):
    """Run ``run()`` ``replays`` times under torch.profiler (kineto / rocprofiler on ROCm: the same
    device timestamps rocprofv3 reports, including the kernels of replayed HIP graphs) and return the
    GPU kernel records as dicts {name, stream, ts (us), dur (us)} sorted by start time."""
    import json
    import os
    import tempfile

    import torch
    from torch.profiler import ProfilerActivity, profile
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(replays):
            run()
        torch.cuda.synchronize()
    fd, path = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    try:
        prof.export_chrome_trace(path)
        with open(path) as f:
            trace = json.load(f)
    finally:
        os.remove(path)
    ks = [{"name": e["name"], "stream": e.get("args", {}).get("stream"), "ts": float(e["ts"]), "dur": float(e["dur"])}
          for e in trace.get("traceEvents", []) if e.get("cat") == "kernel"]
    return sorted(ks, key=lambda k: k["ts"])


class LaunchRecorder:
    """engine.EncoderEngine.conv_timer hook that only records the (op, kind) of every conv launch in
    issue order (kind: fwd / dgrad / wgrad / bwd = dgrad + wgrad in one launch)."""

    def __init__(self):
        self.launches = []

    def begin(self, op, kind):
        self.launches.append((op, kind))

    def end(self):
        pass


class OpGroup:
    """Two convs in one launch (engine: the paired forward ``fwdpair`` = conv1 + downsample, the quad backward
    ``bwdquad`` = conv2 + downsample dgrad and wgrad): ``shape`` is the first (3x3) conv's, the FLOPs are both."""

    def __init__(self, ops):
        self.ops = tuple(ops)
        self.shape = self.ops[0].shape


def launch_flops(op, kind) -> int:
    """Valid-tap FLOPs of one conv launch (both convs of a paired / quad launch)."""
    if kind in ("fwdpair", "bwdquad"):
        return sum(launch_flops(o, "fwd" if kind == "fwdpair" else "bwd") for o in op.ops)
    s = op.shape
    _, valid = conv_macs(s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride, s.pad)
    return 2 * valid * (2 if kind == "bwd" else 1)


def attribute_conv_kernels(kernels, launches, replays: int):
    """Map the conv-family kernels of ONE stream (``kernels``, start-ordered, ``replays`` step replays)
    to that stream's conv launch sequence (``launches`` from a LaunchRecorder, one step).  A split-K
    reduce kernel is charged to the launch before it.  Returns per-launch average durations (us), or
    None when the kernel count does not match the launch sequence."""
    main = [k for k in kernels if not CONV_SECONDARY.search(k["name"])]
    if len(main) != replays * len(launches):
        return None
    per = [0.0] * len(launches)
    li = -1
    for k in kernels:
        if CONV_SECONDARY.search(k["name"]):
            if li >= 0:
                per[li % len(launches)] += k["dur"]
            continue
        li += 1
        per[li % len(launches)] += k["dur"]
    return [d / replays for d in per]
