"""Paired A/B of FusedTrainStep construction options in ONE process (same box, same streams): each variant is
built on its own seed-0 model, fed the same device-gathered batches, and timed in alternating rounds of graph
replays (driver-style: host wall time over K steps after a synchronize).  Also checks that the variants'
parameters stay bitwise equal after the same steps (options that only reschedule work must not change
results).

    python scripts/ab_step.py --variants plain:{} split:{"adam_split":true} [--batch 128] [--rounds 8] [--k 50]
    (a variant's "_stem": [tm, tn, wn, wk, splits, variant] overrides both stems' forward algo)
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tspm_amd  # noqa: E402


def build(batch, kw, dev):
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    kw = dict(kw)
    stem = kw.pop("_stem", None)    # stem forward algo override for both encoders, e.g. [0,0,0,0,0,3]
    stemw = kw.pop("_stemw", None)  # stem weight-gradient algo override
    bn2 = kw.pop("_bn2", None)      # encoders ("a", "i") whose BN statistics merge in two levels in the conv
    pool = kw.pop("_pool", None)    # False: a separate tspm_avgpool_fwd launch after the last block's apply
    bnp = kw.pop("_bnp", None)      # encoders ("a", "i") whose BN backward partial sums come from the dgrad epilogue
    floor = kw.pop("_floor", None)  # the audio encoder's LDS floor (bytes) instead of the default
    am = kw.pop("_am", None)        # the forward BN merge in the apply (tspm_bn_apply_merge) on / off
    bnps = kw.pop("_bnps", None)    # the stem BN's partial sums gathered by layer1's first data gradient on / off
    bnx = kw.pop("_bnx", None)      # rows up to which the whole BN backward runs in the dgrad epilogue (0: off)
    bnpt = kw.pop("_bnpt", None)    # the largest BN (in 32-row tiles) whose backward partial sums come from the dgrad
    step = tspm_amd.FusedTrainStep(model, opt, None, batch, **kw)
    if stem is not None or stemw is not None:
        from tspm_amd import _lib as L
        for e in (step.eng_a, step.eng_i):
            if stem is not None:
                e.stem.algo_fwd = L.ConvAlgo(*stem)
            if stemw is not None:
                e.stem.algo_wgrad = L.ConvAlgo(*stemw)
            e._alloc_workspace()
    if pool is not None:
        step.eng_a.fuse_pool = step.eng_i.fuse_pool = bool(pool)
    if bnp is not None:
        step.eng_a.bn_dgrad_part, step.eng_i.bn_dgrad_part = "a" in bnp, "i" in bnp
    if bnx is not None:
        step.eng_a.bnx_max_rows = step.eng_i.bnx_max_rows = int(bnx)
    if bnps is not None:
        step.eng_a.bnp_stem = step.eng_i.bnp_stem = bool(bnps)
    if am is not None:
        step.eng_a.apply_merge = step.eng_i.apply_merge = bool(am)
    if bnpt is not None:
        step.eng_a.bnp_max_tiles = step.eng_i.bnp_max_tiles = int(bnpt)
    if floor is not None:
        step.slack_lds_floor = int(floor)
    if bn2 is not None:
        step.eng_a.bn_two_level, step.eng_i.bn_two_level = "a" in bn2, "i" in bn2
    feed = bench.corpus_loader(step, batch, 1234, dev, 16384)
    return model, step, feed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", nargs="+", required=True, help="name:json-kwargs")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--k", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    vs = []
    for spec in a.variants:
        name, _, js = spec.partition(":")
        vs.append((name, json.loads(js or "{}")))
    built = {name: build(a.batch, kw, dev) for name, kw in vs}
    for name, (model, step, feed) in built.items():  # identical batches and steps: eager, capture, replays
        for _ in range(5):
            next(feed)
            step.run()
    torch.cuda.synchronize()
    ref = None
    same = {}
    tol = {}
    for name, (model, _, _) in built.items():
        p = torch.cat([q.detach().reshape(-1) for q in model.parameters()])
        if ref is None:
            ref = p
        same[name] = bool(torch.equal(p, ref))
        tol[name] = float(((p - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item())
    times = {name: [] for name in built}
    for r in range(a.rounds):
        order = list(built) if r % 2 == 0 else list(built)[::-1]
        for name in order:
            _, step, feed = built[name]
            for _ in range(5):
                next(feed)
                step.run()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.k):
                next(feed)
                step.run()
            torch.cuda.synchronize()
            times[name].append((time.perf_counter() - t0) / a.k * 1e3)
    out = {"batch": a.batch, "rounds": a.rounds, "steps_per_round": a.k,
           "bitwise_equal_to_first_after_5_steps": same, "max_rel_param_diff_after_5_steps": tol,
           "ms_per_step": {n: {"median": round(sorted(t)[len(t) // 2], 4), "all": [round(x, 4) for x in t]}
                           for n, t in times.items()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
