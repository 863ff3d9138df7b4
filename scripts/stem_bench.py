"""Graph-timed stem convolutions (the 1-channel 7x7/2 stems of both encoders) in isolation: the tuned gather
kernels (variant 0) vs the band kernels (variant 3, stem.hip), forward (+ BN finalize) and weight gradient,
with each launch's kernels' device durations from torch.profiler.

    python scripts/stem_bench.py [--batch 128] [--stamps]   (--stamps: phase stamps, needs `make stamps`)
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

STAMPS = "--stamps" in sys.argv
if STAMPS:
    os.environ["TSPM_LIB"] = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                          "task-specific-pretraining-multimodal_amd", "libtspm_stamps.so")

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import tspm_amd  # noqa: E402,F401
from tspm_amd import _lib as L  # noqa: E402
from tspm_amd.engine import tuned_table  # noqa: E402
from tspm_amd.roofline import device_kernels  # noqa: E402


def timed(fn, reps=50):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (5 * reps)
    ks = device_kernels(lambda: g.replay(), 1)
    per = {}
    for k in ks:
        nm = k["name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:40]
        per[nm] = round(per.get(nm, 0.0) + k["dur"] / reps, 2)
    return round(us, 2), per


def stamps(lib, fn, names):
    """Phase durations (p50 / max over waves, us) of one launch of ``fn`` from the stem kernels' stamps."""
    lib.tspm_debug_stamps_stem.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    torch.cuda.synchronize()
    assert lib.tspm_debug_stamps_stem_clear() == 0
    torch.cuda.synchronize()
    fn()
    torch.cuda.synchronize()
    buf = np.zeros((1 << 18) * 12, dtype=np.uint64)
    assert lib.tspm_debug_stamps_stem(buf.ctypes.data, buf.nbytes) == 0
    st = buf.reshape(-1, 12).astype(np.int64)
    st = st[st[:, 0] > 0]
    t0 = st[:, 0].min()
    out = {"waves": int(len(st)), "span_us": round(float((st[:, :len(names)].max() - t0) * 0.01), 2),
           "entry_spread_max_us": round(float((st[:, 0].max() - t0) * 0.01), 2)}
    for i in range(1, len(names)):
        ok = (st[:, i] > 0) & (st[:, i - 1] > 0)
        d = (st[ok, i] - st[ok, i - 1]) * 0.01
        if len(d):
            out[names[i]] = [round(float(np.percentile(d, 50)), 2), round(float(d.max()), 2)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--stamps", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lib = L.lib()
    tab = tuned_table()
    # the gather configurations the tables held before the band kernels (entries' "algo_before_r4")
    before = {}
    tdir = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "task-specific-pretraining-multimodal_amd", "tuned")
    for f in os.listdir(tdir):
        for e in json.load(open(os.path.join(tdir, f))).get("entries", []):
            before[(e["kind"],) + tuple(e["shape"][:8])] = tuple(e.get("algo_before_r4", e["algo"]))
    out = {}
    for name, (h, w) in (("audio", (32, 94)), ("image", (28, 28))):
        n = a.batch
        p, q = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
        shp = L.ConvShape(n, h, w, 1, 64, 7, 7, 2, 3, p, q)
        x = torch.randn(n, 1, h, w, device=dev)
        st = L.Strides4(h * w, w, 1, 0)
        wt = (torch.randn(64, 1, 7, 7, device=dev) * 0.1).contiguous(memory_format=torch.channels_last)
        y = torch.empty(p * q * n, 64, device=dev)
        dy = torch.randn(p * q * n, 64, device=dev)
        dw = torch.empty_like(wt)
        mean, inv = torch.empty(64, device=dev), torch.empty(64, device=dev)
        key = (n, h, w, 1, 64, 7, 7, 2)
        res = {}
        gf = before.get(("fwd",) + key, (0, 0, 0, 0, 0, 0))
        gw = before.get(("wgrad",) + key, (0, 0, 0, 0, 0, 0))
        gf, gw = (gf if gf[5:6] != (3,) else (0, 0, 0, 0, 0, 0)), (gw if gw[5:6] != (3,) else (0, 0, 0, 0, 0, 0))
        for tag, fa, wa in (("gather", gf, gw), ("band", (0, 0, 0, 0, 0, 3), (0, 0, 0, 0, 0, 3)),
                            ("table", tab.get(("fwd",) + key, gf), tab.get(("wgrad",) + key, gw))):
            af, aw = L.ConvAlgo(*fa), L.ConvAlgo(*wa)
            part = torch.empty(max(lib.tspm_conv_fwd_bn_partial_floats(ctypes.byref(shp), ctypes.byref(af)), 16), device=dev)
            cnt = torch.zeros(64, dtype=torch.int32, device=dev)
            bnf = L.BnFuse(part.data_ptr(), cnt.data_ptr(), None, None, 0.1, 1e-5, mean.data_ptr(), inv.data_ptr(), 0, 0, 0)
            wsb = max(lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(aw)),
                      lib.tspm_conv_fwd_workspace(ctypes.byref(shp), ctypes.byref(af)), 256)
            ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)

            def fwd():
                L.check(lib.tspm_conv_fwd(ctypes.byref(shp), ctypes.byref(af), x.data_ptr(), ctypes.byref(st), wt.data_ptr(),
                                          y.data_ptr(), ctypes.byref(bnf), ws.data_ptr(), wsb,
                                          torch.cuda.current_stream().cuda_stream), "fwd")

            def wgr():
                L.check(lib.tspm_conv_wgrad(ctypes.byref(shp), ctypes.byref(aw), x.data_ptr(), ctypes.byref(st), dy.data_ptr(),
                                            dw.data_ptr(), ws.data_ptr(), wsb, torch.cuda.current_stream().cuda_stream), "wgrad")
            res[tag] = {"algo_fwd": list(fa), "algo_wgrad": list(wa), "fwd+bn": timed(fwd), "wgrad": timed(wgr)}
            if a.stamps and tag == "band":
                res[tag]["fwd_stamps"] = stamps(lib, fwd, ["entry", "staged", "mfma", "stores", "bn_partials"])
                res[tag]["wgrad_stamps"] = stamps(lib, wgr, ["entry", "staged(first band)", "mma(all bands)", "combine+slab"])
        out[name] = res
        print(name, json.dumps(res), flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
