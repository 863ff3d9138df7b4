"""How much of the benched step a one-launch (persistent) ResNet34 layer4 could remove (verdict r3 item 2).

Replays the benched two-stream step graph under kineto (device timestamps; the two streams are not
serialised) and takes the image encoder's stream: its conv kernels are mapped to the image engine's
recorded launch sequence (same order on that stream), layer4 launches are the ones with 512 input or
output channels, and for layer4's forward (first layer4 conv → the global average pool) and backward
(average-pool backward → end of the last layer4 conv backward) it reports the window's span, the
stream's busy time inside it (union of kernel intervals), the idle gaps between its kernels and the
kernel count.  A persistent kernel replaces the window's launches by one launch with a grid barrier per
dependent phase, so it can save at most the gaps plus each kernel's ramp-up / tail, and pays its
barriers (measured ≈1.5-4 µs each on this chip).

    python scripts/layer_span.py [--batch 128] [--replays 20] > gpurun_out/<tag>_layer_span.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tspm_amd  # noqa: E402
from tspm_amd.roofline import CONV_KERNEL, CONV_SECONDARY, LaunchRecorder, device_kernels  # noqa: E402


def union(iv):
    tot, end = 0.0, None
    for a, b in sorted(iv):
        if end is None or a >= end:
            tot, end = tot + b - a, b
        elif b > end:
            tot, end = tot + b - end, b
    return tot


def window(ks, t0, t1):
    sel = [k for k in ks if k["ts"] >= t0 - 1e-3 and k["ts"] + k["dur"] <= t1 + 1e-3]
    busy = union([(k["ts"], k["ts"] + k["dur"]) for k in sel])
    return {"span_us": round(t1 - t0, 2), "busy_us": round(busy, 2), "gaps_us": round(t1 - t0 - busy, 2),
            "kernels": len(sel), "kernel_us_sum": round(sum(k["dur"] for k in sel), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--replays", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    step = tspm_amd.FusedTrainStep(model, opt, None, a.batch)
    feed = bench.corpus_loader(step, a.batch, 1234, dev, 16384)
    rec = LaunchRecorder()
    step.eng_i.conv_timer = rec
    next(feed)
    step.run()  # eager step records the image launch order (the graph is captured from the same calls)
    step.eng_i.conv_timer = None
    seq = rec.launches
    for _ in range(10):
        next(feed)
        step.run()
    torch.cuda.synchronize()
    ks = device_kernels(lambda: (next(feed), step.run()), a.replays)
    # steps: cut before each input gather (the first kernel of a step; the Adam launches are several per
    # step under the split schedules)
    steps, cur = [], []
    for k in ks:
        if "k_avmnist_gather" in k["name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(k)
    res = []
    for st in steps[1:]:
        conv_streams = {}
        for k in st:
            if CONV_KERNEL.search(k["name"]) and not CONV_SECONDARY.search(k["name"]):
                conv_streams[k["stream"]] = conv_streams.get(k["stream"], 0) + 1
        img = [s for s, n in conv_streams.items() if n == len(seq)]
        if len(img) != 1:
            continue
        side = [k for k in st if k["stream"] == img[0]]
        conv = [k for k in side if CONV_KERNEL.search(k["name"]) and not CONV_SECONDARY.search(k["name"])]
        l4 = [i for i, (op, kind) in enumerate(seq) if op.shape.c == 512 or op.shape.k == 512]
        fwd = [i for i in l4 if seq[i][1] == "fwd"]
        bwd = [i for i in l4 if seq[i][1] != "fwd"]
        pool_f = [k for k in side if "avgpool_fwd" in k["name"]]
        pool_b = [k for k in side if "avgpool_bwd" in k["name"]]
        if not (fwd and bwd and pool_f and pool_b):
            continue
        f0 = conv[fwd[0]]["ts"]
        f1 = pool_f[0]["ts"]
        b0 = pool_b[0]["ts"] + pool_b[0]["dur"]
        last = conv[bwd[-1]]
        tail = [k for k in side if CONV_SECONDARY.search(k["name"]) and k["ts"] >= last["ts"]][:1]
        b1 = max([last["ts"] + last["dur"]] + [k["ts"] + k["dur"] for k in tail])
        t0 = min(k["ts"] for k in st)
        t1 = max(k["ts"] + k["dur"] for k in st)
        res.append({"step_span_us": round(t1 - t0, 1), "image_stream": window(side, min(k["ts"] for k in side),
                                                                             max(k["ts"] + k["dur"] for k in side)),
                    "layer4_fwd": window(side, f0, f1), "layer4_bwd": window(side, b0, b1),
                    "layer4_conv_launches": {"fwd": len(fwd), "bwd": len(bwd)}})
    if not res:
        print(json.dumps({"error": "no step could be attributed", "launches": len(seq), "steps": len(steps)}))
        return

    def med(path):
        vals = sorted(r[path[0]][path[1]] if len(path) == 2 else r[path[0]] for r in res)
        return vals[len(vals) // 2]
    out = {"batch": a.batch, "steps": len(res), "what": __doc__.split("\n\n")[0],
           "median": {f"{w}.{f}": med((w, f)) for w in ("layer4_fwd", "layer4_bwd", "image_stream")
                      for f in ("span_us", "busy_us", "gaps_us", "kernels", "kernel_us_sum")},
           "step_span_us_median": med(("step_span_us",)), "layer4_conv_launches": res[0]["layer4_conv_launches"],
           "per_step": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
