"""Where the benched two-stream step spends its time: kineto (torch.profiler = rocprofiler device timestamps)
kernel records of replays of the captured FusedTrainStep graph, split per stream (main = audio encoder +
head + Adam, side = image encoder), with each stream's busy time, the union, the time only one stream is
busy, and the step's phases (encoder forwards, head, backwards, Adam).  Unlike rocprofv3 kernel tracing,
kineto does not serialise the two streams.

    python scripts/overlap_probe.py [--batch 128] [--replays 10] > gpurun_out/<tag>_overlap.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tspm_amd  # noqa: E402
from tspm_amd.roofline import device_kernels  # noqa: E402


def union(iv):
    tot, end = 0.0, None
    for a, b in sorted(iv):
        if end is None or a >= end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--replays", type=int, default=10)
    ap.add_argument("--dump", default="", help="write one step's kernels (stream, start, duration, name) here")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    step = tspm_amd.FusedTrainStep(model, opt, None, a.batch)
    feed = bench.corpus_loader(step, a.batch, 1234, dev, 16384)
    for _ in range(20):
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
        t0 = min(k["ts"] for k in st)
        t1 = max(k["ts"] + k["dur"] for k in st)
        by = {}
        for k in st:
            by.setdefault(k["stream"], []).append((k["ts"], k["ts"] + k["dur"]))
        streams = sorted(by, key=lambda s: -len(by[s]))
        busy = {str(s): round(union(v), 1) for s, v in by.items()}
        u = union([iv for v in by.values() for iv in v])
        both = sum(union(v) for v in by.values()) - u
        head = [k for k in st if "k_head_rows" in k["name"]]
        hs = head[0]["ts"] - t0 if head else None
        he = (head[0]["ts"] + head[0]["dur"] - t0) if head else None
        side = streams[1] if len(streams) > 1 else None
        side_end_fwd = max((e for s, e in by.get(side, []) if s - t0 < (hs or 0)), default=t0) - t0 if side else None
        main_fwd_end = max((e for s, e in by[streams[0]] if s - t0 < (hs or 0) and e - t0 <= (hs or 0)), default=t0) - t0
        adam = [k for k in st if k["name"].startswith("k_adam") or "k_adam(" in k["name"]]
        res.append({"span_us": round(t1 - t0, 1), "union_busy_us": round(u, 1), "both_streams_busy_us": round(both, 1),
                    "idle_us": round(t1 - t0 - u, 1), "per_stream_busy_us": busy,
                    "kernels_per_stream": {str(s): len(v) for s, v in by.items()},
                    "head_start_us": round(hs, 1) if hs is not None else None, "head_end_us": round(he, 1) if he else None,
                    "fwd_end_main_us": round(main_fwd_end, 1), "fwd_end_side_us": round(side_end_fwd, 1) if side else None,
                    "adam_start_us": round(adam[-1]["ts"] - t0, 1) if adam else None,
                    "bwd_end_side_us": round(max(e for _, e in by[side]) - t0, 1) if side else None})
    if a.dump and len(steps) > 2:
        st = steps[len(steps) // 2]
        t0 = min(k["ts"] for k in st)
        with open(a.dump, "w") as f:
            for k in sorted(st, key=lambda k: k["ts"]):
                f.write(f"{k['stream']:>3} {k['ts'] - t0:9.1f} {k['dur']:7.1f} {k['name'][:110]}\n")
    med = lambda key: (lambda v: v[len(v) // 2] if v else None)(sorted(r[key] for r in res if r[key] is not None))  # noqa: E731
    out = {"batch": a.batch, "steps": len(res), "median": {k: med(k) for k in
                                                          ("span_us", "union_busy_us", "both_streams_busy_us", "idle_us",
                                                           "head_start_us", "head_end_us", "fwd_end_main_us",
                                                           "fwd_end_side_us", "adam_start_us", "bwd_end_side_us")},
           "per_step": res}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
