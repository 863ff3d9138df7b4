"""Per-step check of the BatchNorm batch statistics the captured train step produces: after every graph
replay, each BN layer's save_mean / save_invstd (merged in two levels inside the conv, or by
tspm_bn_finalize) against the mean / biased variance of the conv output the same step left in the engine's
buffers, recomputed in fp64 by torch.  A hand-off race in the in-launch merge would show as a step whose
error jumps far above float rounding.

    python scripts/bn_stats_check.py [--steps 300] [--batch 128] [--finalize]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tspm_amd  # noqa: E402


def bn_pairs(eng):
    yield "stem", eng.stem_bn, eng.y0
    for i, bp in enumerate(eng.blocks):
        yield f"b{i}.bn1", bp.bn1, bp.y1
        yield f"b{i}.bn2", bp.bn2, bp.y2
        if bp.ds_bn is not None:
            yield f"b{i}.ds", bp.ds_bn, bp.yd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--finalize", action="store_true", help="tspm_bn_finalize launches instead of the in-conv merge")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    step = tspm_amd.FusedTrainStep(model, opt, None, a.batch)
    for e in (step.eng_a, step.eng_i):
        e.bn_two_level = not a.finalize
    feed = bench.corpus_loader(step, a.batch, 1234, dev, 16384)
    worst = {}
    per_step = []
    for it in range(a.steps):
        next(feed)
        step.run()
        torch.cuda.synchronize()
        smax = 0.0
        for tag, eng in (("audio", step.eng_a), ("image", step.eng_i)):
            for name, bn, y in bn_pairs(eng):
                yd = y.double()
                m = yd.mean(0)
                v = yd.var(0, unbiased=False)
                eps = bn.module.eps
                inv = 1.0 / torch.sqrt(v + eps)
                # mean error in units of the channel's standard deviation; invstd relative error
                em = ((bn.mean.double() - m).abs() / torch.sqrt(v + eps)).max().item()
                ei = ((bn.invstd.double() - inv).abs() / inv).max().item()
                e = max(em, ei)
                k = f"{tag}.{name}"
                if e > worst.get(k, (0.0, -1))[0]:
                    worst[k] = (e, it)
                smax = max(smax, e)
        per_step.append(smax)
        if it % 50 == 0:
            print(f"step {it}: max error {smax:.3e}", flush=True)
    top = sorted(worst.items(), key=lambda kv: -kv[1][0])[:8]
    out = {"mode": "finalize" if a.finalize else "two-level in-conv merge", "steps": a.steps, "batch": a.batch,
           "max_error_over_steps": max(per_step), "median_step_max_error": sorted(per_step)[len(per_step) // 2],
           "steps_above_1e-4": sum(1 for x in per_step if x > 1e-4), "worst_layers": {k: v for k, v in top}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
