"""Measure every supported conv tile configuration on every distinct conv launch of the bench
workload and write the fastest per (kind, shape) as a table the engine loads at plan time.

    python scripts/tune_convs.py --batch 128 --out task-specific-pretraining-multimodal_amd/tuned/mi355x.json

Candidates: the configuration currently in the table (or the heuristic) and every supported
variant-1 (LDS-staged) configuration.  Each candidate is checked against the baseline's output
(max |diff| <= 1e-5 x max |y|) before it may win; timings are HIP-graph replays of back-to-back
launches on one stream (graph_time).
"""
from __future__ import annotations

import argparse
import ctypes
import itertools
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tspm_amd  # noqa: E402
from tspm_amd import _lib as L  # noqa: E402
from tspm_amd.engine import EncoderEngine, prepare_encoder_layout  # noqa: E402

TILES = [(1, 1), (1, 2), (2, 2)]
WNS = [1, 2, 4]
WKS = [1, 2, 4, 8, 16]
SPLITS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64]


def candidates(kind):
    for (tm, tn), wn, wk in itertools.product(TILES, WNS, WKS):
        sps = SPLITS if kind.startswith("wgrad") else [1]
        for sp in sps:
            yield (tm, tn, wn, wk, sp)


def distinct_ops(batch, dev):
    """(kind, ConvShape, input strides) of every conv launch of the late-fusion step."""
    out = {}
    encs = [(tspm_amd.ResNet18(1, 64), 32, 94, True), (tspm_amd.ResNet34(1, 128), 28, 28, False)]
    for enc, h, w, three_d in encs:
        enc = enc.to(dev)
        prepare_encoder_layout(enc)
        eng = EncoderEngine(enc, batch, h, w, dev)
        for op in eng.all_convs():
            s = op.shape
            key = (s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride, s.pad)
            if op is eng.stem:
                # (sn, sh, sw, sc) of the reference NCHW input, as EncoderEngine.input_strides: [N,H,W] audio, [N,1,H,W] image
                xs = L.Strides4(h * w, w, 1, 0) if three_d else L.Strides4(h * w, w, 1, h * w)
                kinds = ("fwd", "wgrad")
            else:
                xs = L.hwnc_strides(s.n, s.h, s.w, s.c)
                kinds = ("fwd", "dgrad", "wgrad")
            for kind in kinds:
                out.setdefault((kind,) + key, (s, xs, op is eng.stem))
    return out


class Bufs:
    def __init__(self, s, stem, dev):
        g = torch.Generator(device="cpu").manual_seed(0)
        n_in = s.n * s.h * s.w * s.c
        self.x = torch.randn(n_in, generator=g).abs_().to(dev) if stem else torch.randn(n_in, generator=g).to(dev)
        self.w = (torch.randn(s.k * s.r * s.s * s.c, generator=g) * 0.05).to(dev)
        self.y = torch.empty(s.n * s.p * s.q * s.k, device=dev)
        self.dy = torch.randn(s.n * s.p * s.q * s.k, generator=g).to(dev)
        self.dx = torch.empty(n_in, device=dev)
        self.dw = torch.empty(s.k * s.r * s.s * s.c, device=dev)
        self.part = torch.empty(3 * (s.n * s.p * s.q // 32 + 1) * s.k, device=dev)
        # transposed operands of wgrad_t ([C][rows]); the values only matter for the cross-check
        self.x_t = self.x.view(-1, s.c).t().contiguous() if not stem else None
        self.dy_t = self.dy.view(-1, s.k).t().contiguous()
        self.ws = torch.zeros(1, dtype=torch.uint8, device=dev)
        self.ws2 = torch.zeros(1, dtype=torch.uint8, device=dev)  # the wgrad side of a fused tspm_conv_bwd
        self.cnt = torch.zeros(s.k // 32 + 1, dtype=torch.int32, device=dev)
        self.mean = torch.empty(s.k, device=dev)
        self.inv = torch.empty(s.k, device=dev)


def launcher(kind, s, xs, b, algo):
    lib = L.lib()
    a = L.ConvAlgo(*algo)
    sh = L.stream_handle()
    if kind.startswith("wgrad"):
        need = lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(a))
        if need > b.ws.numel():
            b.ws = torch.zeros(need, dtype=torch.uint8, device=b.x.device)
        wsb = b.ws.numel()

        if kind == "wgrad_t":
            def f():
                return lib.tspm_conv_wgrad_t(ctypes.byref(s), ctypes.byref(a), b.x_t.data_ptr(), b.x_t.shape[1],
                                             b.dy_t.data_ptr(), b.dy_t.shape[1], b.dw.data_ptr(), b.ws.data_ptr(), wsb,
                                             sh)
        else:
            def f():
                return lib.tspm_conv_wgrad(ctypes.byref(s), ctypes.byref(a), b.x.data_ptr(), ctypes.byref(xs),
                                           b.dy.data_ptr(), b.dw.data_ptr(), b.ws.data_ptr(), wsb, sh)
        return f, b.dw
    if kind == "dgrad":
        need = lib.tspm_conv_dgrad_workspace(ctypes.byref(s), ctypes.byref(a))
        if need > b.ws.numel():
            b.ws = torch.zeros(need, dtype=torch.uint8, device=b.x.device)
        wsb = b.ws.numel()

        def f():
            return lib.tspm_conv_dgrad(ctypes.byref(s), ctypes.byref(a), b.dy.data_ptr(), b.w.data_ptr(),
                                       b.dx.data_ptr(), 0, b.ws.data_ptr(), wsb, sh)
        return f, b.dx

    bnf = L.BnFuse(b.part.data_ptr(), b.cnt.data_ptr(), None, None, 0.1, 1e-5, b.mean.data_ptr(), b.inv.data_ptr())

    need = lib.tspm_conv_fwd_workspace(ctypes.byref(s), ctypes.byref(a))
    if need > b.ws.numel():
        b.ws = torch.zeros(need, dtype=torch.uint8, device=b.x.device)
    wsb = b.ws.numel()

    def f():  # the engine's launch: conv + BN statistics merged in-launch
        return lib.tspm_conv_fwd(ctypes.byref(s), ctypes.byref(a), b.x.data_ptr(), ctypes.byref(xs), b.w.data_ptr(),
                                 b.y.data_ptr(), ctypes.byref(bnf), b.ws.data_ptr(), wsb, sh)
    return f, b.y


def bwd_launcher(s, xs, b, ad, aw):
    """tspm_conv_bwd (dgrad + wgrad in one launch) with separate split-K workspaces."""
    lib = L.lib()
    A, W = L.ConvAlgo(*ad), L.ConvAlgo(*aw)
    nd = lib.tspm_conv_dgrad_workspace(ctypes.byref(s), ctypes.byref(A))
    nw = lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(W))
    if nd > b.ws.numel():
        b.ws = torch.zeros(nd, dtype=torch.uint8, device=b.x.device)
    if nw > b.ws2.numel():
        b.ws2 = torch.zeros(nw, dtype=torch.uint8, device=b.x.device)
    sh = L.stream_handle()

    def f():
        return lib.tspm_conv_bwd(ctypes.byref(s), ctypes.byref(A), ctypes.byref(W), b.x.data_ptr(), ctypes.byref(xs),
                                 b.dy.data_ptr(), b.w.data_ptr(), b.dx.data_ptr(), 0, b.dw.data_ptr(), b.ws.data_ptr(),
                                 b.ws.numel(), b.ws2.data_ptr(), b.ws2.numel(), sh)
    return f


def bwd_pairs(ops, timings, args, dev, topk=4):
    """Fused dgrad + wgrad launches (tspm_conv_bwd): the `topk` fastest built LDS-staged configurations
    of each side, timed together; an entry {"kind": "bwd", "algo": dgrad(6) + wgrad(6)} is written only
    where the fused launch beats the two best separate launches (graph-timed, boundaries included).
    Each fused result is checked bitwise against the two separate launches with the same configs."""
    lib = L.lib()
    out = []
    for key, (s, xs, stem, count, base) in sorted(ops.items(), key=lambda kv: str(kv[0])):
        wkey = ("wgrad",) + key[1:]
        if key[0] != "dgrad" or key not in timings or wkey not in timings:
            continue

        def top(k):
            res = []
            for _, a in sorted(timings[k]):
                if len(a) == 6 and a[5] in (1, 4) and a not in res:
                    res.append(a)
                if len(res) == topk:
                    break
            return res
        sep = min(timings[key])[0] + min(timings[wkey])[0]
        b = Bufs(s, stem, dev)
        best = None
        for ad, aw in itertools.product(top(key), top(wkey)):
            if ad[5] != aw[5]:  # one launch, one kernel build
                continue
            A, W = L.ConvAlgo(*ad), L.ConvAlgo(*aw)
            if not lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(A), ctypes.byref(W), ctypes.byref(xs)):
                continue
            fd, dx = launcher("dgrad", s, xs, b, ad)
            fd()
            want_dx = dx.clone()
            fw, dw = launcher("wgrad", s, xs, b, aw)
            fw()
            want_dw = dw.clone()
            b.dx.fill_(float("nan"))
            b.dw.fill_(float("nan"))
            if bwd_launcher(s, xs, b, ad, aw)() != 0:
                continue
            torch.cuda.synchronize()
            if not (torch.equal(b.dx, want_dx) and torch.equal(b.dw, want_dw)):
                print(f"  MISMATCH bwd {tuple(key[1:])} {ad} {aw}", flush=True)
                continue
            t = graph_time(lambda: bwd_launcher(s, xs, b, ad, aw), args.reps, args.iters)
            if t is not None and (best is None or t < best[0]):
                best = (t, ad, aw)
        del b
        if best is None:
            continue
        fused = best[0] < sep
        print(f"bwd   {str(tuple(key[1:])):42s} x{count:2d} separate {sep:7.2f} us  fused {best[0]:7.2f} us  "
              f"{best[1]} + {best[2]}  -> {'fused' if fused else 'separate'}", flush=True)
        if fused:
            out.append({"kind": "bwd", "shape": list(key[1:]), "algo": list(best[1]) + list(best[2]),
                        "us": round(best[0], 2), "separate_us": round(sep, 2), "count": count})
    return out


def graph_time(make, reps, iters=20):
    """Per-launch time of `reps` back-to-back launches captured in one HIP graph and replayed
    `iters` times (device time + the dependent-launch boundary; no host launch overhead).  make()
    returns the launch closure; it is called inside the capture so the closure binds the capture
    stream.  Returns None if the launch fails."""
    if make()() != 0:
        return None
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        f = make()
        for _ in range(reps):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / (iters * reps)


LDS_TILES = [(1, 1), (1, 2), (2, 1), (2, 2)]
LDS_WAVES = [(1, 1), (2, 1), (4, 1), (1, 2), (2, 2), (1, 4)]   # (wn, wk); wm = 4 / (wn * wk)
LDS_SPLITS = [1, 2, 3, 4, 6, 8, 12, 16, 24, 32]


MAX_WGS = int(os.environ.get("TUNE_MAX_WGS", "0"))  # > 0: only grids up to this many workgroups


def lds_candidates(kind, s, variants=(1,)):
    """Supported LDS-staged configurations of one launch (variant 1; with --variants also 2 and / or 4 — variant 4
    takes wk <= 2 only), with split-K only while the grid stays under ~2048 workgroups (TUNE_MAX_WGS: a tighter cap,
    for concurrency experiments)."""
    for v in variants:
        for a in _lds_candidates_v1(kind, s):
            if v == 4 and a[3] > 2:
                continue
            yield a[:5] + (v,)


def _lds_candidates_v1(kind, s):
    for (tm, tn), (wn, wk) in itertools.product(LDS_TILES, LDS_WAVES):
        wm = 4 // (wn * wk)
        bm, bn = wm * tm * 32, wn * tn * 32
        if kind == "fwd":
            if s.c % 32 or s.n % bm:
                continue
            wgs = (s.p * s.q * s.n // bm) * -(-s.k // bn)
        elif kind == "dgrad":
            if s.k % 32 or s.n % bm:
                continue
            wgs = (s.h * s.w * s.n // bm) * -(-s.c // bn)
        else:
            if s.n % 32 or s.c % bn:
                continue
            wgs = -(-s.k // bm) * (s.r * s.s * s.c // bn)
        for sp in LDS_SPLITS:
            if sp > 1 and wgs * sp > 2048:
                break
            if MAX_WGS and wgs * sp > MAX_WGS and sp > 1:
                break
            yield (tm, tn, wn, wk, sp, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--only-kind", default=None)
    ap.add_argument("--encoders", default="audio,image", help="audio (ResNet18), image (ResNet34) or both")
    ap.add_argument("--no-bwd", action="store_true", help="skip the fused dgrad + wgrad pair pass")
    ap.add_argument("--variants", default="1", help="LDS variants to search: 1 (default), 2, 4 (comma-separated)")
    args = ap.parse_args()
    variants = tuple(int(v) for v in args.variants.split(","))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conv_bench import step_ops
    table = []
    t0 = time.time()
    tot_base, tot_best = 0.0, 0.0
    timings = {}
    ops = step_ops(args.batch, dev, tuple(args.encoders.split(",")))
    for key, (s, xs, stem, count, base) in sorted(ops.items(), key=lambda kv: str(kv[0])):
        kind = key[0]
        if args.only_kind and kind != args.only_kind:
            continue
        b = Bufs(s, stem, dev)
        t_base = graph_time(lambda: launcher(kind, s, xs, b, base)[0], args.reps, args.iters)
        _, out = launcher(kind, s, xs, b, base)
        ref = out.clone()
        scale = float(ref.abs().max()) + 1e-30
        best = (tuple(base), t_base)
        timings[key] = [(t_base, tuple(base))] if t_base is not None else []
        n_ok = 0
        cands = [] if stem else list(lds_candidates(kind, s, variants))
        for algo in cands:
            f, out = launcher(kind, s, xs, b, algo)
            out.fill_(float("nan"))
            if f() != 0:
                continue
            torch.cuda.synchronize()
            err = float((out - ref).abs().max())
            if not err <= 1e-5 * scale:
                print(f"  MISMATCH {kind} {tuple(key[1:])} {algo} err={err:.3e} scale={scale:.3e}", flush=True)
                continue
            t = graph_time(lambda: launcher(kind, s, xs, b, algo)[0], args.reps, args.iters)
            if t is None:
                continue
            n_ok += 1
            timings[key].append((t, tuple(algo)))
            if t < best[1]:
                best = (algo, t)
        t_best = graph_time(lambda: launcher(kind, s, xs, b, best[0])[0], args.reps, 4 * args.iters)
        tot_base += (t_base if t_base is not None else t_best) * count
        tot_best += t_best * count
        table.append({"kind": kind, "shape": list(key[1:]), "algo": list(best[0]), "us": round(t_best, 2),
                      "base_us": round(t_base, 2), "base_algo": list(base), "count": count, "candidates": n_ok})
        print(f"{kind:5s} {str(tuple(key[1:])):42s} x{count:2d} base {t_base:7.2f} us  best {t_best:7.2f} us  "
              f"{best[0]}  ({n_ok} ok, {time.time() - t0:.0f}s)", flush=True)
        del b
    print(f"per-step sum over launches: base {tot_base:.0f} us, tuned {tot_best:.0f} us", flush=True)
    if not args.no_bwd:
        pairs = bwd_pairs(ops, timings, args, dev)
        table += pairs
        saved = sum((e["separate_us"] - e["us"]) * e["count"] for e in pairs)
        print(f"fused dgrad+wgrad pairs: {len(pairs)}, saving {saved:.0f} us per step (graph-timed)", flush=True)
    doc = {"device": torch.cuda.get_device_name(0), "batch": args.batch, "timing": "hip-graph replay",
           "entries": table}
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump(doc, fh, indent=1)
        print("wrote", args.out)


if __name__ == "__main__":
    main()
