"""Tune conv tile configurations INSIDE the captured train step (round-2 finding: configurations that
win in isolation, scripts/tune_convs.py, do not transfer to the two-stream step, where the audio and
image chains run concurrently and compete for CUs).

Greedy coordinate descent over the conv launches of the bench step, most expensive first.  For each
(kind, shape) key the candidates are the current configuration's split-K neighbours (half, double)
plus the `--top` fastest LDS-staged configurations in isolation (fused dgrad + wgrad pairs: the
split-K neighbours of either side); each is first checked against the
current configuration's output in isolation (max |diff| <= 1e-5 x max |y|, as tune_convs does), then
a FusedTrainStep is built with it next to a freshly built step of the current table (build order
alternating) and the two are timed PAIRED: `--rounds` rounds of `--steps` replays each, alternating, on
the same stream.  A null test (the current table against itself) is logged first.  A candidate is accepted when the median
per-step difference is below -`--min-gain-us` and at least 3/4 of the rounds agree in sign.  Progress
and the resulting table (the current tuned entries with the accepted changes) are written after each
key, so a run cut short still leaves its result.

    python scripts/tune_in_step.py --out gpurun_out/in_step.json --budget-s 900
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
import tspm_amd  # noqa: E402
from tspm_amd import _lib as L  # noqa: E402
from tspm_amd import engine as E  # noqa: E402
from conv_bench import step_ops  # noqa: E402
from tune_convs import Bufs, bwd_launcher, graph_time, launcher, lds_candidates  # noqa: E402

B = int(os.environ.get("TUNE_BATCH", "128"))  # per-rank batch of the tuned step
VARIANTS = tuple(int(v) for v in os.environ.get("TUNE_VARIANTS", "1").split(","))  # LDS variants searched


def build(table, dev):
    E._tuned_cache = dict(table)
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    step = tspm_amd.FusedTrainStep(model, opt, None, B, use_graph=True)
    g = torch.Generator().manual_seed(1234)  # AVMNIST-shaped random batch (values do not affect timing)
    step.A.copy_((10.0 ** (torch.randn(B, 32, 94, generator=g) * 2)).to(dev))
    step.I.copy_(torch.rand(B, 1, 28, 28, generator=g).to(dev))
    step.labels.copy_(torch.randint(0, 10, (B,), generator=g).to(dev))
    for _ in range(5):
        step.run()
    torch.cuda.synchronize()
    return step


def time_steps(step, n):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        step.run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def paired(s0, s1, rounds, n):
    d = []
    for r in range(rounds):
        if r % 2:
            b = time_steps(s1, n)
            a = time_steps(s0, n)
        else:
            a = time_steps(s0, n)
            b = time_steps(s1, n)
        d.append(b - a)
    return statistics.median(d), d


def candidates(kind, s, xs, base, top, dev):
    """(isolation-checked) alternatives to `base` for one launch."""
    b = Bufs(s, False, dev)
    f, out = launcher(kind, s, xs, b, base)
    if f() != 0:
        return []
    torch.cuda.synchronize()
    ref = out.clone()
    scale = float(ref.abs().max()) + 1e-30
    timed, seen = [], {tuple(base)}
    neigh = []
    for sp in (base[4] // 2, base[4] * 2):
        if sp >= 1 and base[5] in (1, 4):
            neigh.append(tuple(base[:4]) + (sp, base[5]))
    if base[5] in (1, 2) and base[3] <= 2:  # round 6: the variant-4 twin (bf16-piece products) of the current config
        neigh.append(tuple(base[:5]) + (4,))
    allc = list(lds_candidates(kind, s, VARIANTS))
    for algo in neigh + allc:
        algo = tuple(algo)
        if algo in seen:
            continue
        seen.add(algo)
        f, out = launcher(kind, s, xs, b, algo)
        out.fill_(float("nan"))
        if f() != 0:
            continue
        torch.cuda.synchronize()
        if not float((out - ref).abs().max()) <= 1e-5 * scale:
            continue
        t = graph_time(lambda: launcher(kind, s, xs, b, algo)[0], 10, 3)
        if t is not None:
            timed.append((algo in neigh, t, algo))
    del b
    picked = [a for isn, _, a in timed if isn]
    for _, _, a in sorted((x for x in timed if not x[0]), key=lambda x: x[1]):
        if len(picked) >= len(neigh) + top:
            break
        if a not in picked:
            picked.append(a)
    return picked


def bwd_candidates(s, xs, base, dev):
    """Split-K neighbours (half, double) on either side of a fused dgrad + wgrad pair, checked against
    the current pair's outputs in isolation."""
    import ctypes
    lib = L.lib()
    b = Bufs(s, False, dev)
    ad, aw = tuple(base[:6]), tuple(base[6:12])
    if bwd_launcher(s, xs, b, ad, aw)() != 0:
        return []
    torch.cuda.synchronize()
    rdx, rdw = b.dx.clone(), b.dw.clone()
    sx, sw = float(rdx.abs().max()) + 1e-30, float(rdw.abs().max()) + 1e-30
    out = []
    if ad[5] == aw[5] and ad[5] in (1, 2) and ad[3] <= 2 and aw[3] <= 2:  # round 6: the pair's variant-4 twin
        d, w = ad[:5] + (4,), aw[:5] + (4,)
        A, W = L.ConvAlgo(*d), L.ConvAlgo(*w)
        if lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(A), ctypes.byref(W), ctypes.byref(xs)):
            b.dx.fill_(float("nan"))
            b.dw.fill_(float("nan"))
            if bwd_launcher(s, xs, b, d, w)() == 0:
                torch.cuda.synchronize()
                if float((b.dx - rdx).abs().max()) <= 1e-5 * sx and float((b.dw - rdw).abs().max()) <= 1e-5 * sw:
                    out.append(d + w)
    for side in (0, 1):
        for f in (0.5, 2.0):
            d, w = list(ad), list(aw)
            t = d if side == 0 else w
            t[4] = int(t[4] * f)
            if t[4] < 1:
                continue
            A, W = L.ConvAlgo(*d), L.ConvAlgo(*w)
            if not lib.tspm_conv_bwd_supported(ctypes.byref(s), ctypes.byref(A), ctypes.byref(W), ctypes.byref(xs)):
                continue
            b.dx.fill_(float("nan"))
            b.dw.fill_(float("nan"))
            if bwd_launcher(s, xs, b, tuple(d), tuple(w))() != 0:
                continue
            torch.cuda.synchronize()
            if float((b.dx - rdx).abs().max()) <= 1e-5 * sx and float((b.dw - rdw).abs().max()) <= 1e-5 * sw:
                out.append(tuple(d) + tuple(w))
    del b
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--top", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--min-gain-us", type=float, default=2.0)
    ap.add_argument("--budget-s", type=float, default=900.0)
    ap.add_argument("--skip", default=None, help="a previous --out: its keys are not tried again")
    a = ap.parse_args()
    t0 = time.time()
    dev = torch.device("cuda", 0)
    base_table = dict(E.tuned_table())
    table = dict(base_table)
    done = set()
    log = []
    if a.skip and os.path.exists(a.skip):
        with open(a.skip) as fh:
            prev = json.load(fh)
        done = {tuple(k) for k in prev.get("keys_done", [])}
        log = prev.get("log", [])
    ops = step_ops(B, dev)
    order = []
    for key, (s, xs, stem, count, base) in ops.items():
        tk = (key[0],) + tuple(key[1:9])
        if stem or tk in done:
            continue
        pk = ("bwd",) + tuple(key[1:9])
        if key[0] != "fwd" and pk in table:  # a fused dgrad + wgrad pair owns both configs
            if key[0] == "dgrad" and pk not in done:
                b = Bufs(s, False, dev)
                t = graph_time(lambda: bwd_launcher(s, xs, b, table[pk][:6], table[pk][6:12]), 10, 3)
                del b
                order.append(((t or 0.0) * count, pk, s, xs, tuple(table[pk])))
            continue
        b = Bufs(s, False, dev)
        t = graph_time(lambda: launcher(key[0], s, xs, b, tuple(base))[0], 10, 3)
        del b
        order.append(((t or 0.0) * count, tk, s, xs, tuple(base)))
    order.sort(key=lambda x: -x[0])
    print(f"{len(order)} keys to try ({time.time() - t0:.0f}s)", flush=True)

    s0 = build(table, dev)
    base_us = statistics.median(time_steps(s0, a.steps) for _ in range(5))
    print(f"start: {base_us:.1f} us/step", flush=True)
    del s0
    gc.collect()

    def dump(final=False):
        changed = [{"kind": k[0], "shape": list(k[1:]), "algo": list(v)} for k, v in table.items()
                   if base_table.get(k) != v]
        entries = [{"kind": k[0], "shape": list(k[1:]), "algo": list(v)} for k, v in sorted(table.items())]
        doc = {"batch": B, "timing": "paired FusedTrainStep replays (scripts/tune_in_step.py)", "start_us": base_us,
               "final": final, "elapsed_s": round(time.time() - t0, 1), "changed": changed,
               "keys_done": [list(k) for k in done], "log": log, "entries": entries}
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(doc, fh, indent=1)

    # a fresh build next to an older one is not timed alike (a step built later ran ~15 us slower in a
    # first run), so every comparison is between two steps built back to back, in alternating order
    n_pair = [0]

    def compare(t_base, t_cand):
        n_pair[0] += 1
        first, second = (t_base, t_cand) if n_pair[0] % 2 else (t_cand, t_base)
        x = build(first, dev)
        y = build(second, dev)
        sb, sc = (x, y) if n_pair[0] % 2 else (y, x)
        med, d = paired(sb, sc, a.rounds, a.steps)
        del x, y, sb, sc
        gc.collect()
        torch.cuda.empty_cache()
        return med, d

    null = [compare(table, table) for _ in range(2)]
    log.append({"null_test_median_diff_us": [round(m, 2) for m, _ in null]})
    print("null test (same table twice):", [f"{m:+.2f}" for m, _ in null], flush=True)
    dump()

    for cost, tk, s, xs, base in order:
        if time.time() - t0 > a.budget_s:
            print("budget spent", flush=True)
            break
        cur = tuple(table.get(tk, base))
        cands = (bwd_candidates(s, xs, cur, dev) if tk[0] == "bwd" else
                 candidates(tk[0], s, xs, cur, a.top, dev))
        best = None
        for c in cands:
            trial = dict(table)
            trial[tk] = c
            try:
                med, d = compare(table, trial)
            except L.TspmError as e:
                log.append({"key": list(tk), "algo": list(c), "error": str(e)})
                continue
            agree = sum(x < 0 for x in d)
            log.append({"key": list(tk), "from": list(cur), "algo": list(c), "median_diff_us": round(med, 2),
                        "neg_rounds": agree, "rounds": len(d)})
            print(f"  {tk} {cur} -> {c}: {med:+.2f} us ({agree}/{len(d)} faster)", flush=True)
            if med < -a.min_gain_us and agree * 4 >= 3 * len(d) and (best is None or med < best[0]):
                best = (med, c)
        if best is not None:
            table[tk] = best[1]
            print(f"ACCEPT {tk}: {cur} -> {best[1]} ({best[0]:+.2f} us)", flush=True)
        done.add(tk)
        dump()
    med, d = compare(base_table, table)
    log.append({"final_vs_start_median_diff_us": round(med, 2), "rounds": [round(x, 2) for x in d]})
    print(f"end: tuned table vs start table {med:+.2f} us/step (paired, fresh builds)", flush=True)
    dump(final=True)



if __name__ == "__main__":
    main()
