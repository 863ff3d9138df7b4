"""Benchmark: samples/sec (node) of the AVMNIST late-fusion train step on 1..8 MI355X.

One rank per GPU (torchrun env).  Per rank: batch 128 (BASELINE.json configs[2]: global 1024 on 8
GPUs), a synthetic AVMNIST-shaped corpus resident in HBM, random-init weights (seed 0).  A
"step" = batch assembly on device (tspm_avmnist_gather from the corpus into the step's static
buffers: the reference's __getitem__/collate_fn/H2D) → ResNet18(audio) ‖
ResNet34(image) forward → fusion head → cross-entropy → backward → [RCCL all-reduce] → Adam,
all in fp32 on the libtspm HIP kernels (graph-replayed).

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline     — the conv implicit-GEMM kernel family (dominant: ~90 % of step FLOPs): valid-tap
                 FLOPs of every conv launch of one step ÷ the summed DEVICE duration of those kernels
                 (torch.profiler = rocprofiler timestamps) over replays of the step re-captured on one
                 stream after the timed region; peak = fp32 MFMA 157.3 TF/s.
  cpu_baseline — the oracle (CPU fp32 restatement of the reference train step, bit-identical to it
                 on CPU) timed on this host at batch 128, rank 0 / N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "samples/sec (node) AVMNIST late-fusion train step at 1/2/4/8 MI355X"
PER_RANK_BATCH = 128


def corpus_loader(step, batch: int, seed: int, dev, n_corpus: int):
    """The input stage: a synthetic AVMNIST corpus (SURVEY.md §8(d) distributions; no dataset download
    here) resident in HBM, read in shuffled epochs by data.DeviceLoader — one tspm_avmnist_gather
    launch per step (index gather + colormap LUT + 1/255 + pattern masks + labels) writing straight
    into the fused step's static input buffers."""
    from tspm_amd.data import AVMNIST, synthetic_corpus
    ds = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=synthetic_corpus(n_corpus, seed),
                 device=dev)
    ds.device_corpus  # upload once, outside the timed region
    loader = ds.device_loader(batch, shuffle=True, drop_last=True, generator=torch.Generator().manual_seed(seed),
                              out=(step.A, step.I, step.labels))

    def batches():
        epoch = 0
        while True:
            loader.set_epoch(epoch)
            yield from loader
            epoch += 1
    return batches()


def host_cpu():
    """The host's CPU as this process sees it: model name, logical CPUs in the affinity mask, physical
    cores behind them (distinct (package, core) pairs of /proc/cpuinfo) and the cgroup CPU quota."""
    info = {"model": None, "logical": len(os.sched_getaffinity(0)), "physical": None, "cgroup_cpus": None}
    try:
        aff = os.sched_getaffinity(0)
        cores, cur = set(), {}
        with open("/proc/cpuinfo") as f:
            for line in list(f) + [""]:
                if not line.strip():
                    if cur.get("processor") is not None and int(cur["processor"]) in aff:
                        cores.add((cur.get("physical id", "0"), cur.get("core id", cur["processor"])))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                cur[k.strip()] = v.strip()
                if k.strip() == "model name" and info["model"] is None:
                    info["model"] = v.strip()
        info["physical"] = len(cores) or None
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            info["cgroup_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return info


def cpu_threads():
    """Threads for the CPU baseline: every physical core this process may use (capped by the cgroup
    CPU quota when one is set — threads beyond the quota only queue)."""
    h = host_cpu()
    n = h["physical"] or h["logical"]
    if h["cgroup_cpus"]:
        n = min(n, max(1, int(h["cgroup_cpus"])))
    return max(1, n), h


def _union_us(kl):
    """Total time (us) during which at least one of the kernels ``kl`` runs (intervals merged)."""
    tot, end = 0.0, None
    for k in sorted(kl, key=lambda k: k["ts"]):
        a, b = k["ts"], k["ts"] + k["dur"]
        if end is None or a >= end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def conv_roofline(seq, run_serial, replays: int, run_concurrent=None):
    """Conv-family roofline from DEVICE kernel durations (torch.profiler = the rocprofiler timestamps
    rocprofv3 reports; no host gaps) of ``replays`` replays of the step captured on ONE stream — the
    kernels run back to back, each alone on the chip, which is also how rocprofv3's kernel tracing
    executes the captured graph, so the durations agree with the committed rocprofv3 summary.  One
    stream also fixes the kernel order, so every conv kernel maps to its launch (``seq``: [(encoder,
    op, kind)] in issue order, from LaunchRecorders): achieved = valid-tap FLOPs of the step's conv
    launches / their summed duration; the ResNet34 3x3 subset and the per-launch table come from the
    same mapping.  ``run_concurrent``: optionally also profile the benched two-stream graph (kernels
    of the two encoders overlap there and stretch each other)."""
    from tspm_amd.roofline import CONV_KERNEL, attribute_conv_kernels, device_kernels, launch_flops
    ks_all = device_kernels(run_serial, replays)
    if sum(1 for k in ks_all if CONV_KERNEL.search(k["name"])) < len(seq):
        # the profiler occasionally returns garbled kernel names for a whole capture ("void " / ""; seen with
        # "ROCTracer produced duplicate flow start"): profile once more before giving up on attribution
        ks_all = device_kernels(run_serial, replays)
    # split the trace into steps before each input gather (``run_serial`` = gather + step: the first kernel of
    # every step; the optimizer launches Adam once per encoder, so k_adam does not mark step ends) and
    # keep only COMPLETE steps: the profiler drops a few records in a long capture (up to ~5 % of a
    # 10-replay trace), so a chunk is kept when its conv-kernel count equals the recorded launch
    # sequence and its kernel count equals the largest such chunk's (a chunk that lost its gather
    # spans two steps and fails the first test)
    from tspm_amd.roofline import CONV_SECONDARY
    steps, cur = [], []
    for k in ks_all:
        if "k_avmnist_gather" in k["name"] and cur:
            steps.append(cur)
            cur = []
        cur.append(k)
    if cur:
        steps.append(cur)
    full = [st for st in steps if sum(1 for k in st if CONV_KERNEL.search(k["name"])
                                      and not CONV_SECONDARY.search(k["name"])) == len(seq)]
    most = max((len(st) for st in full), default=0)
    good = [st for st in full if len(st) == most]
    dropped = replays - len(good)
    if good:
        replays = len(good)
        ks = [k for st in good for k in st]
    else:
        ks = ks_all
    conv = [k for k in ks if CONV_KERNEL.search(k["name"])]
    conv_us = sum(k["dur"] for k in conv) / replays
    flops = sum(launch_flops(op, kind) for _, op, kind in seq)
    out = {"conv_kernel_ms_per_step": conv_us / 1e3, "valid_tap_flop_per_step": flops,
           "achieved": flops / (conv_us * 1e-6) / 1e12 if conv_us else None,
           "kernel_ms_per_step": sum(k["dur"] for k in ks) / replays / 1e3, "kernels_per_step": len(ks) / replays,
           "conv_launches_per_step": len(seq), "families": {}, "profiled_steps": replays,
           "incomplete_steps_dropped": dropped,
           # round 6: the share of the conv family's device time in the variant-4 kernels (k_*_x9: fp32 products
           # from exact bf16 pieces on the bf16 MFMA), whose own product-rate ceiling is 2.5 PF / 9 bf16 products
           "x9_conv_ms_per_step": sum(k["dur"] for k in conv if "_x9" in k["name"]) / replays / 1e3}
    for k in ks:
        fam = ("conv" if CONV_KERNEL.search(k["name"]) else "bn" if "k_bn_" in k["name"] else
               "adam" if "k_adam" in k["name"] else "pool" if "pool" in k["name"] else "other")
        out["families"][fam] = out["families"].get(fam, 0.0) + k["dur"] / replays / 1e3
    per = attribute_conv_kernels(conv, [(op, kind) for _, op, kind in seq], replays)
    out["per_launch"] = None if per is None else [(name, op, kind, us) for (name, op, kind), us in zip(seq, per)]
    if per is None:
        names = {}
        for k in conv:
            key = k["name"].split("(")[0][-60:]
            names[key] = names.get(key, 0) + 1
        out["attribution_failed"] = {"conv_kernels": len(conv), "replays": replays, "launches_per_step": len(seq),
                                     "kinds": sorted({kind for _, _, kind in seq}), "names": names}
    if run_concurrent is not None:
        kc = [k for k in device_kernels(run_concurrent, replays) if CONV_KERNEL.search(k["name"])]
        out["concurrent"] = {"conv_kernel_ms_per_step": round(sum(k["dur"] for k in kc) / replays / 1e3, 4),
                             "conv_busy_ms_per_step": round(_union_us(kc) / replays / 1e3, 4)}
    return out


def _stats(xs):
    xs = sorted(xs)
    if not xs:
        return None
    return {"mean": round(sum(xs) / len(xs), 4), "median": round(xs[len(xs) // 2], 4), "max": round(xs[-1], 4)}


def exchange_block(step, one, args, world: int, ms_per_step: float) -> dict:
    """How much of the DP gradient exchange the phased step hides (every rank takes part; after the timed
    region).  (1) ``--exchange-steps`` more phased steps with ``FusedTrainStep.exchange_probe`` on: the host's
    wait for each backward phase's step flag and the device time from the end of the fwd+bwd graph to the end
    of the step — the exposed tail: the last phase's all-reduce and its Adam ranges, plus whatever of the
    first two phases' exchange + Adam had not finished on the comm stream by then; (2) the same number of
    LOCAL steps (the plain step re-captured: same kernels, no collective) timed like the headline, so
    ``ms_per_step - local_step_ms`` is the exchange's total exposed cost.  Values are maxima over ranks."""
    ar = step.allreduce
    P = args.exchange_steps
    probe = []
    step.exchange_probe = probe
    for i in range(P):
        one(i)
    torch.cuda.synchronize()
    step.exchange_probe = None
    w0 = [p["host_wait_ms"][0] for p in probe]
    w1 = [p["host_wait_ms"][1] for p in probe]
    tail = [p["events"][0].elapsed_time(p["events"][1]) for p in probe]
    win0 = [p["window_ms"][0] for p in probe]
    win1 = [p["window_ms"][1] for p in probe]
    phase_bytes = [sum(v.numel() * 4 for v in ph) for ph in ar.phases]
    step.allreduce, step.graph, step.graph_opt = None, None, None
    for i in range(3):  # capture + settle the local step
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(P):
        one(i)
    torch.cuda.synchronize()
    local_ms = (time.perf_counter() - t0) / P * 1e3
    vals = [local_ms, sum(tail) / len(tail), max(tail), sum(w0) / len(w0), sum(w1) / len(w1),
            sum(win0) / len(win0), sum(win1) / len(win1)]
    if world > 1:
        t = torch.tensor(vals, dtype=torch.float64, device=step.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = t.tolist()
    out = exchange_summary(vals, phase_bytes, [len(ph) for ph in ar.phases], world, ms_per_step, P)
    out["rank0_tail_ms"] = _stats(tail)
    out["rank0_host_wait_ms"] = {"phase0": _stats(w0), "phase1": _stats(w1)}
    out["rank0_window_ms"] = {"phase0": _stats(win0), "phase1": _stats(win1)}
    return out


def exchange_summary(vals, phase_bytes, buckets, world: int, ms_per_step: float, steps: int) -> dict:
    """The line's ``exchange`` block from [local_ms, tail_mean, tail_max, wait0_mean, wait1_mean[, window0_mean,
    window1_mean]] (maxima over ranks; shared by the GPU bench and the gloo dry run).  window = the rest of the
    backward after the host saw a late phase's flag: the span that phase's exchange (+ its Adam ranges) must fit in
    to stay hidden — at N > 1 compare it with the phase's bytes over the measured RCCL rate (round 6, VERDICT r5
    item 7)."""
    win = {}
    if len(vals) >= 7:
        win = {"late_phase_window_ms_per_step": {"phase0_mean": round(vals[5], 4), "phase1_mean": round(vals[6], 4)}}
    return {**win, "rccl_world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": str(dist.get_backend()) if dist.is_initialized() else None,
            "forced_1rank_exchange": world == 1,
            "phases": len(phase_bytes), "bytes_per_phase": phase_bytes, "buckets_per_phase": buckets,
            "steps_probed": steps,
            "exposed_tail_ms_per_step": {"mean": round(vals[1], 4), "max": round(vals[2], 4)},
            "host_wait_ms_per_step": {"phase0_flag_mean": round(vals[3], 4), "phase1_flag_mean": round(vals[4], 4)},
            "local_step_ms": round(vals[0], 4),
            "exchange_exposed_ms_per_step": round(ms_per_step - vals[0], 4),
            "what": "phased DP step (ddp.PhasedGradAllReduce): the all-reduce of each backward phase starts when the "
                    "host sees that phase's step flag and runs on the comm stream beside the rest of the backward; "
                    "exposed tail = device time from the fwd+bwd graph's end to the step's end; local_step_ms = the "
                    "same kernels without the collective, timed after the timed region; exchange_exposed = "
                    "ms_per_step - local_step_ms (maxima over ranks)"}


def subset_roofline(per_launch, pred, peak):
    """Valid-tap TFLOP/s of the launches (encoder, op, kind, us) satisfying ``pred(encoder, op)``."""
    if not per_launch:
        return None
    from tspm_amd.roofline import launch_flops
    sel = [(op, kind, us) for name, op, kind, us in per_launch if pred(name, op)]
    us = sum(u for _, _, u in sel)
    fl = sum(launch_flops(op, kind) for op, kind, _ in sel)
    if not us:
        return None
    tf = fl / (us * 1e-6) / 1e12
    return {"achieved": round(tf, 3), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4),
            "launches": len(sel), "ms_per_step": round(us / 1e3, 4), "valid_tap_flop_per_step": fl}


class _EngineRecorder:
    """conv_timer hook of one engine appending (encoder, op, kind) to a shared launch list."""

    def __init__(self, name, seq):
        self.name, self.seq = name, seq

    def begin(self, op, kind):
        self.seq.append((self.name, op, kind))

    def end(self):
        pass


def pmc_traffic(family: str = "conv", path: str = "main"):
    """HBM bytes per step of one kernel family from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by scripts/pmc_traffic.sh + pmc_traffic.py: FETCH_SIZE and
    WRITE_SIZE passes over this same bench command, gfx950 read correction applied).  None if absent."""
    import glob
    import re

    def ver(p):  # newest = highest r<round>_v<version> (mtimes are equal on a fresh checkout)
        m = re.search(r"r(\d+)_v(\d+)", os.path.basename(p))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    def tag(p):  # rR_vV_pmc_traffic.json -> "main"; rR_vV_<workload>_pmc_traffic.json -> <workload>
        m = re.match(r"r\d+_v\d+_(?:(\w+?)_)?pmc_traffic\.json$", os.path.basename(p))
        return (m.group(1) or "main") if m else None
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), key=ver)
    # "main": the AVMNIST summaries; "mmimdb" / "mosi": that workload's own summaries
    files = [f for f in files if tag(f) == path]
    if not files:
        return None, None, None
    with open(files[-1]) as f:
        d = json.load(f)
    if family == "step":
        tot = d.get("per_step_total_bytes")
        return (tot, None, os.path.relpath(files[-1], REPO)) if tot else (None, None, None)
    fam = d.get("per_step_bytes", {}).get(family)
    if not fam:
        return None, None, None
    return fam["total"], fam.get("launches"), os.path.relpath(files[-1], REPO)


def mfma_counters(batch: int):
    """The conv family's MFMA-busy / wave-state PMC counters at this batch from the newest committed summary
    (profiles/r<round>_b<batch>_mfma_busy.json, scripts/pmc_mfma.sh + pmc_mfma.py over this bench command):
    MFMA pipe utilisation and where the conv waves' cycles go.  None if no summary for this batch."""
    import glob
    import re
    def ver(p):  # r<round>[_v<version>]_b<batch>_mfma_busy.json: newest = highest (round, version)
        m = re.match(r"r(\d+)(?:_v(\d+))?_b\d+_mfma_busy\.json$", os.path.basename(p))
        return (int(m.group(1)), int(m.group(2) or 0)) if m else (-1, -1)
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_b{batch}_mfma_busy.json")), key=ver)
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    c = d.get("families", {}).get("conv")
    if not c:
        return None
    waits = {"frac_wait_inst_any": c["frac_wait_inst_any"], "frac_wait_any": c["frac_wait_any"],
             "frac_active_inst": c["frac_active_inst"]}
    return {"source": os.path.relpath(files[-1], REPO), "batch": batch,
            "mfma_busy_cycles_per_step": c["mfma_busy_cycles"] / max(1, d.get("steps_in_run", 1)),
            "mfma_util": c["mfma_util_at_2p4GHz"], "clock": "priced at 2.4 GHz (the chip's maximum)",
            "wave_state": waits, "capping_state": max(waits, key=waits.get),
            "what": "SQ_VALU_MFMA_BUSY_CYCLES over the conv kernels' device time x 256 CUs x 4 SIMDs x clock "
                    "(64 busy cycles per f32 32x32x2 MFMA); wave_state = fractions of SQ_WAVE_CYCLES"}


def mmimdb_flops_per_sample(di=4096, dt=300, e=512, d=512, h=512, c=23):
    """Algorithmic train FLOPs per sample of the MMIMDb step: 2 x MACs of forward + data-grad + weight-grad
    of every product (the encoder Linears' data-grad feeds the input BatchNorm1d's gamma/beta gradients)."""
    enc = di * e + dt * e
    rest = 2 * e * d + 2 * d + d * 2 * h + h * 2 * h + h * c
    return 2 * 3 * (enc + rest)


def mmimdb_bench(args) -> None:
    """--mmimdb: BASELINE.json configs[3] — the MMIMDb image+text late-fusion train step
    (MML_Suite/models/mmimdb.py:203-245 with configs/mmimdb/centralised/mmimdb_baseline.yaml: BN1d+Linear
    encoders over 4096-d image / 300-d text features, GMU, MaxOut MLP, BCEWithLogits, Adam) as one
    FusedMMIMDbStep graph replay per step; per-rank batch --mmimdb-batch.  Inputs: 16 synthetic batches
    resident in HBM, one device-to-device copy into the step's input buffers per step.  Roofline: the
    whole step's algorithmic FLOPs (small-GEMM dominated) over its time vs the fp32 MFMA peak."""
    import tspm_amd
    from tspm_amd import mmimdb as M
    from tspm_amd.roofline import FP32_MFMA_PEAK_TFLOPS
    from tspm_amd import ddp
    rank, world, local = ddp.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B = args.mmimdb_batch
    torch.manual_seed(0)
    ie, te = M.MMIMDbModalityEncoder(4096, 512), M.MMIMDbModalityEncoder(300, 512)
    if args.mmimdb_pooling:  # configs/mmimdb/centralised/pooling/mmimdb_pooling_<kind>.yaml
        clf = M.MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
        model = M.MMIMDb(ie, te, multimodal_pooling={"pooling_type": args.mmimdb_pooling, "hidden_dim": 512,
                                                      "dropout": 0.1}, classifier=clf).to(dev)
    else:
        gmu = M.GatedBiModalNetwork(input_one_dim=512, output_one_dim=512, input_two_dim=512, output_two_dim=512)
        clf = M.MLPGenreClassifier(input_size=512, hidden_size=512, output_size=23)
        model = M.MMIMDb(ie, te, gated_bimodal_network=gmu, classifier=clf).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=1e-5, weight_decay=1e-3, grad_scale=1.0 / world)
    allreduce = None
    if world > 1:  # data parallel: one RCCL all-reduce of the flat gradient buffer (15.4 MB) per step
        for fg in opt.flat_groups():
            dist.broadcast(fg.param, src=0)
        allreduce = ddp.GradAllReduce([fg.grad for fg in opt.flat_groups()])
    st = M.FusedMMIMDbStep(model, opt, None, B, allreduce=allreduce)
    batches = [tuple(t.to(dev) for t in M.synthetic_features(B, seed=1234 + 100 * rank + i)) for i in range(16)]

    def one(i):
        I, T, y = batches[i % len(batches)]
        st.eng.I.copy_(I, non_blocking=True)
        st.eng.T.copy_(T, non_blocking=True)
        st.eng.labels.copy_(y, non_blocking=True)
        st.run()
    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    value = args.steps * B * world / el
    fps = mmimdb_flops_per_sample()
    tf = fps * value / 1e12
    nparam = sum(p.numel() for p in model.parameters())
    traffic, _, traffic_src = pmc_traffic("step", "mmimdb") if B == 256 else (None, None, None)
    res = {"metric": "samples/sec MMIMDb image+text late-fusion (GMU) train step, 1 MI355X (BASELINE.json configs[3])",
           "value": round(value, 2), "unit": "samples/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32",
           "data": "synthetic MM-IMDb-shaped features (4096-d ReLU image, 300-d text, 23 multi-hot genres), 16 "
                   "batches resident in HBM; random-init weights (seed 0)",
           "config": {"workload": "mmimdb_late_fusion_train_step(bn1d+linear encoders, "
                                  f"{('pooling_' + args.mmimdb_pooling) if args.mmimdb_pooling else 'gmu'}, "
                                  "maxout mlp, bce, adam)",
                      "per_rank_batch": B, "global_batch": B * world, "parallelism": f"dp{world}", "params": nparam},
           "roofline": {"bound": "mfma", "kernel": "whole step (k_gemm_small MFMA products dominate the FLOPs)",
                        "achieved": round(tf, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tf / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": traffic,
                        "traffic_unit": "HBM bytes per step, all kernels (PMC: 2 x FETCH_SIZE + WRITE_SIZE; batch 256)",
                        "traffic_source": traffic_src,
                        "flop_per_sample": fps, "adam_bytes_per_step": 28 * nparam},
           "final_loss": round(st.eng.loss.item(), 5), "process_group": process_group_info()}
    if not args.no_cpu_baseline and rank == 0:
        from oracle import mmimdb_ref as orc
        from oracle.avmnist_ref import OracleAdam
        threads, hcpu = cpu_threads()
        torch.set_num_threads(threads)
        ref = orc.build_oracle_mmimdb(0, pooling=None if not args.mmimdb_pooling else {
            "pooling_type": args.mmimdb_pooling, "hidden_dim": 512, "dropout": 0.1})
        ropt = OracleAdam(list(ref.parameters()), lr=1e-5, weight_decay=1e-3)
        I, T, y = orc.synthetic_batch(B, seed=1234)
        orc.train_step(ref, ropt, I, T, y)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and n < 2000:
            orc.train_step(ref, ropt, I, T, y)
            n += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * B / el, 1), "unit": "samples/sec", "cores": threads, "cpu_model": hcpu["model"], "host_cpus": hcpu, "kind": "port",
                               "sample": f"{n} oracle MMIMDb train steps (fwd+BCE+bwd+Adam, fp32) at batch {B}, "
                                         f"{el:.1f}s, torch.set_num_threads({threads})"}
    if rank == 0:
        emit(res)
    if world > 1:
        dist.destroy_process_group()


def _time_oracle_step(batch: int, budget_s: float):
    from oracle import avmnist_ref as orc
    model = orc.build_oracle_avmnist(0)
    opt = orc.OracleAdam(list(model.parameters()), lr=5e-4, weight_decay=1e-4)
    audio, image, labels, _ = orc.synthetic_batch(batch, seed=1234)
    orc.train_step(model, opt, audio, image, labels)  # warm-up
    n = 0
    t0 = time.perf_counter()
    while True:
        orc.train_step(model, opt, audio, image, labels)
        n += 1
        el = time.perf_counter() - t0
        if el > budget_s or n >= 200:
            break
    return n, el


def cpu_baseline(batch: int, budget_s: float = 15.0):
    """Time the oracle's CPU train step (bit-identical to the reference's on CPU) on this host's
    physical cores, at the benched per-rank batch and at BASELINE configs[0]'s batch 32."""
    threads, hcpu = cpu_threads()
    torch.set_num_threads(threads)
    n, el = _time_oracle_step(batch, budget_s)
    n32, el32 = _time_oracle_step(32, budget_s / 2)
    return {"value": round(n * batch / el, 1), "unit": "samples/sec", "cores": threads, "cpu_model": hcpu["model"],
            "host_cpus": hcpu, "kind": "port",
            "sample": f"{n} oracle train steps (fwd+CE+bwd+Adam, fp32) at batch {batch} on CPU, {el:.1f}s, "
                      f"torch.set_num_threads({threads})",
            "c1_batch32": {"value": round(n32 * 32 / el32, 1), "unit": "samples/sec",
                           "sample": f"{n32} oracle train steps at batch 32 (BASELINE configs[0]), {el32:.1f}s"}}


INPUT_BYTES_PER_SAMPLE = (12032 + 784 + 8 + 8 + 8) + (12032 + 3136 + 8)  # reads (audio, image u8, label,
# index, 2 masks) + writes (audio, image f32, label) of tspm_avmnist_gather, per sample


def input_stage_bench(args) -> None:
    """--input-stage: the AVMNIST input stage alone.  Reports samples/s of
    (a) the drop-in path (torch DataLoader → AVMNIST.__getitems__ → collate_fn: one pinned ≈2 KB H2D
    + one gather launch per batch, Python included), (b) DeviceLoader epochs, with the gather kernel's
    HBM roofline at batch 128 and 1024, and a CPU baseline: the reference's per-sample host path
    (torch.load + cm.gist_earth + PIL + stack + .to(device)) restated in oracle/avmnist_data_ref.py."""
    import tempfile
    from tspm_amd.data import AVMNIST, synthetic_corpus
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.corpus_input
    t0 = time.perf_counter()
    corpus = synthetic_corpus(n, 1234)
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"], corpus=corpus, device=dev)
    dc = ds.device_corpus
    torch.cuda.synchronize()
    upload_s = time.perf_counter() - t0
    res = {"metric": "samples/sec AVMNIST input stage (batch assembly into HBM)", "unit": "samples/sec",
           "corpus_samples": n, "corpus_bytes_hbm": n * (12032 + 784 + 8),
           "corpus_build_and_upload_s": round(upload_s, 2)}
    kern = {}
    for B in (128, 1024):
        idx = torch.randint(0, n, (B,), device=dev)
        am = torch.ones(B, device=dev)
        im = torch.ones(B, device=dev)
        out = (torch.empty(B, 32, 94, device=dev), torch.empty(B, 1, 28, 28, device=dev),
               torch.empty(B, dtype=torch.int64, device=dev))
        for _ in range(20):
            dc.gather(idx, am, im, out=out)
        # device time per launch: R launches captured in one HIP graph, replayed (the host-side
        # ctypes launch path, ~9 us per call, would otherwise be what is measured)
        R = 100
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(R):
                dc.gather(idx, am, im, out=out)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (5 * R)
        gbs = INPUT_BYTES_PER_SAMPLE * B / (us * 1e-6) / 1e9
        kern[B] = {"us_per_launch": round(us, 3), "achieved_GBps": round(gbs, 1), "samples_per_s": round(B / us * 1e6)}
    res["gather_kernel"] = kern
    # (a) drop-in DataLoader path
    B = 128
    dl = torch.utils.data.DataLoader(ds, batch_size=B, shuffle=True, collate_fn=ds.collate_fn)
    it = iter(dl)
    for _ in range(5):
        next(it)
    torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    for _ in range(K):
        next(it)
    torch.cuda.synchronize()
    res["dataloader_dropin_samples_per_s"] = round(K * B / (time.perf_counter() - t0))
    # (b) DeviceLoader: one epoch over the 3-pattern valid split (3n items), epoch setup included
    dv = ds.device_loader(B, shuffle=True)
    t0 = time.perf_counter()
    cnt = 0
    for b in dv:
        cnt += b["labels"].numel()
    torch.cuda.synchronize()
    res["device_loader_epoch_samples_per_s"] = round(cnt / (time.perf_counter() - t0))
    res["value"] = res["dataloader_dropin_samples_per_s"]
    k = kern[128]
    res["roofline"] = {"bound": "hbm", "kernel": "k_avmnist_gather", "achieved": k["achieved_GBps"], "peak": 8000.0,
                       "unit": "GB/s", "frac": round(k["achieved_GBps"] / 8000.0, 4),
                       "traffic": pmc_traffic("gather")[0], "traffic_unit": "HBM bytes per 128-sample launch (PMC)",
                       "bytes_per_sample": INPUT_BYTES_PER_SAMPLE, "batch": 128}
    # CPU baseline: the reference's host path on a bounded sample of files
    from oracle import avmnist_data_ref as dref
    torch.set_num_threads(1)
    root = tempfile.mkdtemp(prefix="tspm_ref_corpus_")
    m = args.cpu_input_samples
    small = corpus.subset(range(m))
    csv = dref.write_reference_files(root, small.audio, small.image, small.labels)
    for _ in dref.reference_host_batches(csv, B, dev):  # warm-up: matplotlib / PIL / file cache
        break
    t0 = time.perf_counter()
    cnt = 0
    for b in dref.reference_host_batches(csv, B, dev):
        cnt += b["labels"].numel()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    res["cpu_baseline"] = {"value": round(cnt / el, 1), "unit": "samples/sec", "cores": 1, "kind": "port",
                           "sample": f"{cnt} samples in the reference file layout through the reference's "
                                     f"per-sample host path (torch.load x2, cm.gist_earth, PIL convert L, "
                                     f"ToDtype scale, mask, stack, .to(cuda)), batch {B}, 1 thread, {el:.1f}s"}
    emit(res)


def eval_bench(args) -> None:
    """--eval: the evaluation path on one GPU — validation_step as one
    FusedEvalStep graph per batch (eval forward of both encoders, head, CE, on-device prediction /
    confusion / loss bookkeeping) fed by the device gather, over an AVMNIST-validation-sized corpus
    with the 3 missing-data patterns; plus whole epochs through harness.EpochRunner (validation with
    the YAML's 12 metrics, and a training epoch) and a CPU baseline: the oracle's validation_step."""
    import tspm_amd
    from tspm_amd.data import AVMNIST, synthetic_corpus
    from tspm_amd.harness import EpochRunner
    from tspm_amd.metrics import ClassificationLog
    from tspm_amd.roofline import FP32_MFMA_PEAK_TFLOPS, eval_flops_per_sample
    from tspm_amd.step import FusedEvalStep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch_per_rank
    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    ds = AVMNIST(None, "valid", "multimodal", selected_patterns=["ai", "a", "i"],
                 corpus=synthetic_corpus(args.eval_corpus, 4321), device=dev)
    log = ClassificationLog(dev)
    st = FusedEvalStep(model, None, B, log)
    loader = ds.device_loader(B, shuffle=True, drop_last=True, generator=torch.Generator().manual_seed(0),
                              out=(st.A, st.I, st.labels))

    def feed():
        while True:
            for b in loader:
                st.groups.copy_(b["pattern_ids"], non_blocking=True)
                yield b
    f = feed()
    from tspm_amd.roofline import LaunchRecorder
    rec = LaunchRecorder()
    st.eng.conv_timer = rec
    for _ in range(args.warmup):
        next(f)
        st.run()
        st.eng.conv_timer = None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        next(f)
        st.run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    value = args.steps * B / el
    nom, valid = eval_flops_per_sample()
    tflops = valid * value / 1e12
    res = {"metric": "samples/sec AVMNIST validation step (eval fwd + CE + on-device metrics), 1 MI355X",
           "value": round(value, 1), "unit": "samples/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "dtype": "fp32",
           "data": f"synthetic AVMNIST-shaped validation corpus of {args.eval_corpus} samples x 3 patterns in HBM",
           "config": {"workload": "avmnist_validation_step(resnet18_audio+resnet34_image+mlp_head, CE, metrics)",
                      "batch": B},
           "roofline": {"bound": "mfma", "kernel": "whole eval step (conv family dominant)",
                        "achieved": round(tflops, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(tflops / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                        "valid_tap_flop_per_sample": valid}}
    # whole epochs through the harness (metrics computed at the end of each)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    runner = EpochRunner(model, opt, None)
    vl = ds.device_loader(B)
    runner.validate_epoch(vl)  # capture
    t0 = time.perf_counter()
    _, _, metrics, nb = runner.validate_epoch(vl)
    el = time.perf_counter() - t0
    res["validate_epoch"] = {"samples": len(ds), "batches": nb, "seconds": round(el, 4),
                             "samples_per_s": round(len(ds) / el, 1), "accuracy_AI": float(metrics["accuracy_AI"])}
    tr = AVMNIST(None, "train", "multimodal", selected_patterns=["ai"], corpus=synthetic_corpus(args.eval_corpus, 99),
                 device=dev)
    tl = tr.device_loader(B, shuffle=True, drop_last=True)
    runner.train_epoch(tl)
    t0 = time.perf_counter()
    _, _, _, nb = runner.train_epoch(tl)
    el = time.perf_counter() - t0
    res["train_epoch"] = {"samples": nb * B, "batches": nb, "seconds": round(el, 4),
                          "samples_per_s": round(nb * B / el, 1)}
    if not args.no_cpu_baseline:
        from oracle import avmnist_eval_ref as eref
        from oracle import avmnist_ref as orc
        threads, hcpu = cpu_threads()
        torch.set_num_threads(threads)
        ref = orc.build_oracle_avmnist(0)
        audio, image, labels, _ = orc.synthetic_batch(B, seed=1234)
        eref.validation_step(ref, audio, image, labels)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and n < 400:
            eref.validation_step(ref, audio, image, labels)
            n += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * B / el, 1), "unit": "samples/sec", "cores": threads, "cpu_model": hcpu["model"], "host_cpus": hcpu, "kind": "port",
                               "sample": f"{n} oracle validation steps (eval fwd + CE + softmax argmax) at batch {B}, "
                                         f"{el:.1f}s, torch.set_num_threads({threads})"}
    emit(res)


def mono_bench(args) -> None:
    """--mono: BASELINE.json configs[1] — the monomodal ResNet18 audio pre-training step
    (MML_Suite/train_monomodal.py:97-260: encoder → classifier → CE → backward → Adam, argmax
    predictions) at batch 256 on one MI355X as one FusedMonoStep graph replay per step, each batch
    gathered on device from an HBM-resident synthetic corpus; conv roofline as for the main line; CPU
    baseline: the oracle's monomodal step (bit-identical to the reference's on CPU)."""
    import tspm_amd
    from tspm_amd.data import AVMNIST, synthetic_corpus
    from tspm_amd.monomodal import FusedMonoStep, MonomodalEncoder
    from tspm_amd.roofline import FP32_MFMA_PEAK_TFLOPS, mono_flops_per_sample
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.mono_batch
    torch.manual_seed(0)
    model = MonomodalEncoder(tspm_amd.ResNet18(1, 64), 64, 10).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4)
    st = FusedMonoStep(model, opt, None, (B, 32, 94))
    ds = AVMNIST(None, "train", "audio", selected_patterns=["a"], corpus=synthetic_corpus(args.corpus, 1234),
                 device=dev)
    ds.device_corpus  # upload once, outside the timed region
    loader = ds.device_loader(B, shuffle=True, drop_last=True, generator=torch.Generator().manual_seed(1234),
                              out=(st.X, None, st.labels))

    def feed():
        epoch = 0
        while True:
            loader.set_epoch(epoch)
            yield from loader
            epoch += 1
    f = feed()
    for _ in range(args.warmup):
        next(f)
        st.run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        next(f)
        st.run()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    value = args.steps * B / el
    # roofline: device kernel durations of further graph replays (outside the timed region); the graph
    # is re-captured once with a recorder on the engine so every conv launch maps to its shape
    roof = None
    if args.profile_steps > 0:
        seq = []
        st.graph, st.eng.conv_timer = None, _EngineRecorder("audio", seq)
        next(f)
        st.run()
        st.eng.conv_timer = None
        roof = conv_roofline(seq, lambda: (next(f), st.run()), args.profile_steps)
    achieved = roof["achieved"] if roof else float("nan")
    conv_ms = roof["conv_kernel_ms_per_step"] if roof else float("nan")
    conv_flops = roof["valid_tap_flop_per_step"] if roof else None
    n_launch = roof["conv_launches_per_step"] if roof else None
    nominal, valid = mono_flops_per_sample()
    step_tf = valid * value / 1e12
    res = {"metric": "samples/sec AVMNIST monomodal ResNet18 audio pre-train step, 1 MI355X (BASELINE.json configs[1])",
           "value": round(value, 2), "unit": "samples/sec", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32",
           "data": f"synthetic AVMNIST-shaped audio corpus of {args.corpus} samples resident in HBM, gathered on "
                   "device each step; random-init weights (seed 0)",
           "config": {"workload": "avmnist_monomodal_train_step(resnet18_audio+linear(64,10), CE, Adam)", "batch": B},
           "roofline": {"bound": "mfma", "kernel": "conv implicit-GEMM family (LDS-staged + register-direct), "
                                                   "fp32 MFMA 32x32x2",
                        "achieved": round(achieved, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                        "launches_per_step": n_launch, "conv_ms_per_step": round(conv_ms, 4),
                        "valid_tap_flop_per_step": conv_flops, "step_valid_tflops": round(step_tf, 3),
                        "step_frac_of_peak": round(step_tf / FP32_MFMA_PEAK_TFLOPS, 4),
                        "valid_tap_flop_per_sample": valid, "nominal_flop_per_sample": nominal},
           "final_loss": round(st.loss.item(), 5)}
    if not args.no_cpu_baseline:
        from oracle import avmnist_ref as orc
        from oracle import monomodal_ref as mref
        threads, hcpu = cpu_threads()
        torch.set_num_threads(threads)
        ref = mref.build_oracle_monomodal("audio", 0)
        ropt = orc.OracleAdam(list(ref.parameters()), lr=5e-4, weight_decay=1e-4)
        audio, _, labels, _ = orc.synthetic_batch(B, seed=1234)
        mref.train_step(ref, ropt, audio, labels)  # warm-up
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and n < 200:
            mref.train_step(ref, ropt, audio, labels)
            n += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * B / el, 1), "unit": "samples/sec", "cores": threads, "cpu_model": hcpu["model"], "host_cpus": hcpu, "kind": "port",
                               "sample": f"{n} oracle monomodal train steps (ResNet18 + Linear, CE, Adam, fp32) at "
                                         f"batch {B}, {el:.1f}s, torch.set_num_threads({threads})"}
    emit(res)


def _mosi_family(name: str) -> str:
    from tspm_amd.roofline import CONV_KERNEL
    for key, fam in (("k_lstm_fwd", "lstm_fwd"), ("k_lstm_bwd", "lstm_bwd"), ("k_textcnn", "textcnn_pool_wgrad"),
                     ("k_seq_gather", "seq_gather"), ("k_adam", "adam"), ("k_sumsq", "clip"), ("k_clip", "clip")):
        if key in name:
            return fam
    if CONV_KERNEL.search(name):
        return "textcnn_conv"
    return "gemm_other"


def mosi_bench(args) -> None:
    """--mosi: BASELINE.json configs[4] — the MOSI UTT-Fusion train step (models/msa/utt_fusion.py:151-200 with
    configs/mosi/centralised/utt_fusion_base_training.yaml: LSTM audio 5→64 and video 20→64, TextCNN over
    768-d text, FcClassifier 192→192/64/32→3, CE, clip_grad_norm_ 1.0, Adam) at per-rank batch --mosi-batch
    as one FusedMosiStep graph replay per step.  Input stage in the step: a ragged synthetic MOSI corpus
    (lengths uniform in [20, 50]) resident in HBM, each batch padded to the aligned length 50 and gathered
    time-major straight into the step's inputs (3 tspm_seq_gather launches; 'atv' training pattern).
    Roofline: the TextCNN convolution (the step's FLOP-dominant kernel, implicit GEMM on MFMA) from device
    kernel durations of graph replays after the timed region; the LSTM recurrences are latency-bound
    (T=50 dependent steps) and reported by time."""
    import tspm_amd
    from tspm_amd import ddp
    from tspm_amd import mosi as M
    from tspm_amd.mosi_data import MOSI, synthetic_mosi_corpus
    from tspm_amd.roofline import CONV_KERNEL, FP32_MFMA_PEAK_TFLOPS, device_kernels
    rank, world, local = ddp.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    from types import SimpleNamespace
    cname = "mosei" if args.mosei else "mosi"
    cfg = SimpleNamespace(**M.YAML_CONFIGS[cname])
    B, T = args.mosi_batch or cfg.batch, 50
    torch.manual_seed(0)
    model = M.build_utt_fusion(cname).to(dev)
    netT = model.netT
    opt = tspm_amd.FusedAdam(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay, grad_scale=1.0 / world)
    st = model.fused_step(opt, None, B, T)  # None: the config's single cross-entropy term, weight 1.0
    if world > 1:  # data parallel: one RCCL all-reduce of the flat gradient buffer per step, then clip + Adam
        for fg in opt.flat_groups():
            dist.broadcast(fg.param, src=0)
        st.allreduce = ddp.GradAllReduce([fg.grad for fg in opt.flat_groups()])
    ds = MOSI(split="train", corpus=synthetic_mosi_corpus(args.mosi_corpus, 1234 + rank, T, min_len=20,
                                                          feats=(cfg.audio_dim, cfg.video_dim, 768)),
              selected_patterns=["atv"], device=dev, seed=rank)
    ds.device_corpus  # upload once, outside the timed region
    gen = torch.Generator().manual_seed(1234 + rank)

    def feed():
        while True:
            yield from ds.device_loader(B, shuffle=True, drop_last=True, generator=gen,
                                        step_for=lambda b, t: st, pad_to=T)
    f = feed()

    def one():
        next(f)
        st.run()
    for _ in range(args.warmup):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    value = args.steps * B * world / el
    heights, C, Ft = netT.heights, netT.out_channels, netT.input_size
    conv_flops = sum(2 * B * (T - h + 1) * h * Ft * C for h in heights)  # valid MACs x 2, one launch per height
    roof = {"bound": "mfma", "kernel": "TextCNN convolutions: (h x 768) kernels over [B, T, 768] as implicit GEMM "
                                       "(LDS-staged MFMA 32x32x2 fp32), 3 launches per step",
            "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "traffic": None,
            "flop_per_step": conv_flops, "achieved": None, "frac": None}
    tr, tr_launches, tr_src = pmc_traffic("conv", "mosi") if (B == 128 and not args.mosei) else (None, None, None)
    if tr:
        roof.update({"traffic": tr, "traffic_per_launch": round(tr / tr_launches) if tr_launches else None,
                     "traffic_unit": "HBM bytes per step of the TextCNN convs (PMC: 2 x FETCH_SIZE + WRITE_SIZE)",
                     "traffic_source": tr_src})
    if args.profile_steps > 0 and world == 1:
        R = args.profile_steps
        ks = device_kernels(one, R)
        fams, names = {}, {}
        for k in ks:
            fam = _mosi_family(k["name"])
            fams[fam] = fams.get(fam, 0.0) + k["dur"] / R / 1e3
            mt = re.search(r"\b(k_\w+|at::native::\w+|\w*[Kk]ernel\w*)", k["name"])
            nm = mt.group(1) if mt else k["name"][:60]
            cnt, ms = names.get(nm, (0, 0.0))
            names[nm] = (cnt + 1, ms + k["dur"] / R / 1e3)
        conv = [k for k in ks if CONV_KERNEL.search(k["name"]) and "k_textcnn" not in k["name"]]
        conv_us = sum(k["dur"] for k in conv) / R
        ach = conv_flops / (conv_us * 1e-6) / 1e12 if conv_us else None
        roof.update({"achieved": round(ach, 3) if ach else None,
                     "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4) if ach else None,
                     "conv_ms_per_step": round(conv_us / 1e3, 4), "conv_launches_per_step": len(conv) / R,
                     "kernels_per_step": len(ks) / R, "kernel_ms_per_step": round(sum(k["dur"] for k in ks) / R / 1e3, 4),
                     "kernel_ms_per_step_by_family": {k: round(v, 4) for k, v in sorted(fams.items())},
                     "kernels_by_name": {k: [round(v[0] / R, 2), round(v[1], 4)] for k, v in
                                         sorted(names.items(), key=lambda kv: -kv[1][1])},
                     "timing": f"device kernel durations (torch.profiler = rocprofiler timestamps) of {R} graph "
                               "replays after the timed region (one stream)"})
    name = ("MOSEI UTT-Fusion (configs/mosei/centralised/utt_fusion_train_mosei.yaml: maxpool LSTMs, BN classifier)"
            if args.mosei else "MOSI UTT-Fusion (LSTM audio/video + TextCNN text + FcClassifier)")
    res = {"metric": f"samples/sec {name} train step" + ("" if args.mosei else " (BASELINE.json configs[4])"),
           "value": round(value, 2), "unit": "samples/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(el / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "fp32",
           "data": f"synthetic {'MOSEI' if args.mosei else 'MOSI'}-shaped ragged corpus of {args.mosi_corpus} samples "
                   f"(audio {cfg.audio_dim}-d, video {cfg.video_dim}-d, text 768-d, lengths U[20,50]) resident in HBM, "
                   "padded to 50 and gathered on device each step; random-init weights (seed 0)",
           "config": {"workload": f"{'mosei' if args.mosei else 'mosi'}_utt_fusion_train_step(lstm x2 "
                                  f"[{cfg.embd_method}], textcnn, fc classifier{' +bn' if cfg.use_bn else ''}, CE, "
                                  f"clip {cfg.clip}, Adam)",
                      "per_rank_batch": B, "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                      "params": sum(p.numel() for p in model.parameters())},
           "roofline": roof, "final_loss": round(st.eng.loss.item(), 5), "process_group": process_group_info()}
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        from oracle import mosi_ref as mref
        from oracle.avmnist_ref import OracleAdam
        threads, hcpu = cpu_threads()
        torch.set_num_threads(threads)
        ocfg = mref.MOSEI if args.mosei else mref.MOSI
        ref = mref.build_oracle_utt(0, cfg=ocfg)
        ropt = OracleAdam(list(ref.parameters()), lr=cfg.lr, weight_decay=cfg.weight_decay)
        A, V, X, y = mref.synthetic_batch(B, T, seed=1234, cfg=ocfg)
        mref.train_step(ref, ropt, A, V, X, y)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and n < 500:
            mref.train_step(ref, ropt, A, V, X, y)
            n += 1
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(n * B / el, 1), "unit": "samples/sec", "cores": threads,
                               "cpu_model": hcpu["model"], "host_cpus": hcpu, "kind": "port",
                               "sample": f"{n} oracle UTT-Fusion train steps (fwd+CE+bwd+clip+Adam, fp32; bit-identical "
                                         f"to the reference on CPU) at batch {B}, T={T}, {el:.1f}s, "
                                         f"torch.set_num_threads({threads})"}
    if rank == 0:
        emit(res)
    if world > 1:
        dist.destroy_process_group()


def process_group_info():
    """Backend and world size as the initialised process group reports them (None at N=1 without one)."""
    if not dist.is_initialized():
        return None
    return {"backend": str(dist.get_backend()), "world_size": dist.get_world_size(), "rank": dist.get_rank()}


_JSON_FD = None


def quiet_stdout() -> None:
    """Route everything written to fd 1 (RCCL's init banner, library prints, Python prints) to stderr,
    keeping a private duplicate of the real stdout for the ONE JSON result line (emit)."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(obj) -> None:
    """Write the bench's one JSON line to the real stdout."""
    line = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """``--gpus N`` (N > 1) started as a plain process: this parent makes NO GPU call (it only counts
    nothing, binds a port and waits) and starts N child processes of this same script, one per GPU, with
    the torchrun-style env (RANK = LOCAL_RANK = r, WORLD_SIZE = N, MASTER_ADDR 127.0.0.1, a free
    MASTER_PORT) — children, not an exec of this process.  It forwards rank 0's ONE JSON line (with
    ``launch`` added) and exits non-zero, after stopping the others, as soon as any child fails."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        # rank 0's stdout carries the JSON line; the other ranks' stdout joins this process's stderr
        out = subprocess.PIPE if r == 0 else sys.stderr.fileno()
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=out))
    failed = None
    while failed is None and any(p.poll() is None for p in procs):
        for r, p in enumerate(procs):
            if p.poll() not in (None, 0):
                failed = (r, p.returncode)
                break
        time.sleep(0.2)
    if failed is None:
        bad = [(r, p.returncode) for r, p in enumerate(procs) if p.returncode != 0]
        failed = bad[0] if bad else None
    if failed is not None:
        for p in procs:  # the exact PIDs this process started
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        print(f"bench.py: rank {failed[0]} exited with status {failed[1]}", file=sys.stderr)
        return failed[1] or 1
    lines = [ln for ln in procs[0].stdout.read().decode().splitlines() if ln.strip().startswith("{")]
    if len(lines) != 1:
        print(f"bench.py: rank 0 printed {len(lines)} JSON lines, expected 1", file=sys.stderr)
        return 1
    res = json.loads(lines[0])
    res["launch"] = {"mode": "spawned by bench.py --gpus (one child process per GPU)", "ranks": n}
    emit(res)
    return 0


def check_world(gpus: int) -> None:
    """Refuse a launch whose torchrun world disagrees with --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (launch one rank per GPU)")


def dry_run(args) -> None:
    """--dry-run: the multi-rank plumbing without a GPU — the same launch (torchrun env or spawn_ranks),
    process group (gloo), barrier-bracketed timed region, max over ranks and rank-0 JSON line as the
    real bench, with an empty step; then the post-timed-region legs with the real line's keys: an
    ``exchange`` block from a phased gloo all-reduce of a small flat buffer (host-timed), a ``roofline``
    placeholder (no kernels ran) and — rank 0 only, every N, the other ranks waiting in a gloo barrier — the
    oracle's CPU train step for ``--cpu-budget`` seconds.  Every rank reports (rank, pid, world size)."""
    from tspm_amd import ddp
    rank, world, _ = ddp.init_from_env("gloo")
    B = args.batch_per_rank
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    if world > 1:
        dist.barrier()
    el = max(time.perf_counter() - t0, 1e-9)
    me = torch.tensor([rank, os.getpid(), dist.get_world_size() if dist.is_initialized() else 1, el],
                      dtype=torch.float64)
    allr = [torch.zeros_like(me) for _ in range(world)]
    if world > 1:
        dist.all_gather(allr, me)
    else:
        allr = [me]
    el = max(float(t[3]) for t in allr)
    ms_per_step = el / max(args.steps, 1) * 1e3
    exchange = None
    if world > 1 and args.exchange_steps > 0:
        flat = torch.ones(3 * 1024)
        ar = ddp.PhasedGradAllReduce([[flat[:1024]], [flat[1024:2048]], [flat[2048:]]], bucket_mb=0.002)
        tails = []
        for _ in range(args.exchange_steps):
            t1 = time.perf_counter()
            for k in range(3):
                ar.wait(ar.launch(k))
            tails.append((time.perf_counter() - t1) * 1e3)
        vals = torch.tensor([0.0, sum(tails) / len(tails), max(tails), 0.0, 0.0, 0.0, 0.0], dtype=torch.float64)
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        exchange = exchange_summary(vals.tolist(), [v.numel() * 4 for ph in ar.phases for v in ph[:1]],
                                    [len(ph) for ph in ar.phases], world, ms_per_step, args.exchange_steps)
        exchange["dry_run"] = "gloo all-reduce of a 12 KB flat buffer in 3 phases, host-timed; no step ran"
    res = None
    if rank == 0:
        res = {"metric": METRIC, "value": round(world * B * args.steps / el, 2), "unit": "samples/sec",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "dry_run": True,
               "process_group_world_size": int(allr[0][2]),
               "ranks": [{"rank": int(t[0]), "pid": int(t[1]), "pg_world_size": int(t[2])} for t in allr],
               "config": {"per_rank_batch": B, "global_batch": B * world, "parallelism": f"dp{world}"},
               "roofline": {"bound": "mfma", "achieved": None, "frac": None, "r34_3x3": None,
                            "dry_run": "no kernels ran (the GPU bench's rank 0 profiles its local step here)"},
               "exchange": exchange}
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(B, args.cpu_budget)
    if world > 1:
        dist.barrier()  # gloo: the other ranks sleep here while rank 0 times the CPU baseline
    if rank == 0:
        emit(res)
    if dist.is_initialized():
        dist.destroy_process_group()


def main() -> None:
    quiet_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-rank", type=int, default=PER_RANK_BATCH)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--corpus", type=int, default=16384, help="samples in the HBM-resident synthetic corpus")
    ap.add_argument("--phased", action="store_true",
                    help="at N=1, run the DP step path anyway (1-rank RCCL group, all-reduce = identity)")
    ap.add_argument("--input-stage", action="store_true", help="benchmark the input stage alone (one JSON line)")
    ap.add_argument("--corpus-input", type=int, default=60000, help="--input-stage corpus size (AVMNIST train: 60k)")
    ap.add_argument("--cpu-input-samples", type=int, default=16384)
    ap.add_argument("--eval", action="store_true", help="benchmark the evaluation path / epoch harness (one JSON line)")
    ap.add_argument("--eval-corpus", type=int, default=10000, help="--eval validation corpus (x3 patterns)")
    ap.add_argument("--mono", action="store_true",
                    help="benchmark the monomodal ResNet18 audio pre-training step (BASELINE.json configs[1])")
    ap.add_argument("--mono-batch", type=int, default=256)
    ap.add_argument("--mmimdb", action="store_true", help="BASELINE configs[3]: MMIMDb late-fusion step (one JSON line)")
    ap.add_argument("--mmimdb-batch", type=int, default=256)
    ap.add_argument("--mmimdb-pooling", default=None, choices=["max", "avg", "sum", "attention", "gated"],
                    help="--mmimdb with multimodal_pooling fusion instead of the GMU")
    ap.add_argument("--mosi", action="store_true", help="BASELINE configs[4]: MOSI UTT-Fusion step (one JSON line)")
    ap.add_argument("--mosi-batch", type=int, default=0, help="default 128 (MOSI YAML) / 256 (--mosei YAML)")
    ap.add_argument("--mosei", action="store_true",
                    help="--mosi with the MOSEI UTT-Fusion config (maxpool LSTM embeddings, BN classifier, clip 0.5)")
    ap.add_argument("--mosi-corpus", type=int, default=4096, help="samples in the HBM-resident MOSI corpus")
    ap.add_argument("--profile-steps", type=int, default=10,
                    help="step replays profiled after the timed region for the roofline (0: skip)")
    ap.add_argument("--exchange-steps", type=int, default=20,
                    help="DP exchange probe: phased steps probed + local steps timed after the timed region (0: skip)")
    ap.add_argument("--pcie-steps", type=int, default=20,
                    help="steps of the secondary PCIe-inclusive measurement (0: skip)")
    ap.add_argument("--kernel-table", default=None, help="write the per-launch conv durations (JSON) here")
    ap.add_argument("--dry-run", action="store_true",
                    help="multi-rank plumbing only (gloo, no GPU, empty step): launch, barriers, max over ranks")
    args = ap.parse_args()
    check_world(args.gpus)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.input_stage or args.eval or args.mono:
            raise SystemExit("bench.py: --input-stage / --eval / --mono are single-GPU benches")
        sys.exit(spawn_ranks(args.gpus))
    if args.dry_run:
        dry_run(args)
        return
    if args.input_stage:
        input_stage_bench(args)
        return
    if args.mono:
        mono_bench(args)
        return
    if args.mmimdb:
        mmimdb_bench(args)
        return
    if args.mosi:
        mosi_bench(args)
        return
    if args.eval:
        eval_bench(args)
        return

    import tspm_amd
    from tspm_amd import ddp
    from tspm_amd.roofline import FP32_MFMA_PEAK_TFLOPS, step_flops_per_sample

    rank, world, local = ddp.init_from_env("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    B = args.batch_per_rank

    torch.manual_seed(0)
    model = tspm_amd.AVMNIST(tspm_amd.ResNet18(1, 64), tspm_amd.ResNet34(1, 128), 128, dropout=0.5).to(dev)
    opt = tspm_amd.FusedAdam(model.parameters(), lr=5e-4, weight_decay=1e-4, grad_scale=1.0 / world)
    step = tspm_amd.FusedTrainStep(model, opt, None, B, use_graph=not args.no_graph)
    if world > 1:
        for fg in opt.flat_groups():
            dist.broadcast(fg.param, src=0)
        # RCCL gradient all-reduce overlapped with the second backward phase (ddp.PhasedGradAllReduce)
        step.allreduce = step.phased_allreduce()
    elif args.phased:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        step.allreduce = step.phased_allreduce(force=os.environ.get("TSPM_PHASED_FORCE", "1") == "1")
    feed = corpus_loader(step, B, 1234 + rank, dev, args.corpus)

    def one(i):
        next(feed)  # gathers the next shuffled batch into step.A / step.I / step.labels
        step.run()

    for i in range(args.warmup):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        one(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed

    # ---- after the timed region: how much of the DP exchange the step hides (every rank) -----------
    exchange = None
    if isinstance(step.allreduce, ddp.PhasedGradAllReduce) and step.use_graph and args.exchange_steps > 0:
        exchange = exchange_block(step, one, args, world, ms_per_step)
    # from here on every rank runs the LOCAL step (same kernels, no collective), so rank 0 can profile and
    # time the CPU baseline alone; the other ranks wait on a CPU (gloo) barrier, which sleeps in a socket read
    # instead of spinning on the GPU or a host core
    if step.allreduce is not None:
        step.allreduce, step.graph, step.graph_opt = None, None, None
    cpu_group = dist.new_group(backend="gloo") if world > 1 else None

    # ---- roofline: device kernel durations of further step replays (outside the timed region) ----
    R = args.profile_steps
    roof = None
    if R > 0 and rank == 0 and step.use_graph:
        seq = []
        concurrent = lambda: one(0)  # noqa: E731  (the benched graph)
        step.graph, step.serial = None, True  # re-capture on ONE stream, recording the launch order
        # with the optimizer's own Adam launches: the conv kernels' device time is then conv work alone (the benched
        # step carries the finished blocks' Adam updates inside later backward launches, step.AdamCarry)
        carry, step.adam_carry = step.adam_carry, "none"
        step.eng_a.conv_timer, step.eng_i.conv_timer = _EngineRecorder("audio", seq), _EngineRecorder("image", seq)
        one(0)
        step.eng_a.conv_timer = step.eng_i.conv_timer = None
        roof = conv_roofline(seq, lambda: one(0), R)
        step.graph, step.serial, step.adam_carry = None, False, carry
        one(0)  # back to the benched two-stream graph
        roof["concurrent"] = conv_roofline(seq, concurrent, R)["families"]
    nominal, valid = step_flops_per_sample()
    step_tflops = valid * B * world / (elapsed / args.steps) / 1e12 / world

    # ---- secondary: the PCIe-inclusive step (a pinned host batch copied H2D each step) -----------
    pcie = None
    if args.pcie_steps > 0 and rank == 0:
        import numpy as np
        from tspm_amd.data import default_lut, synthetic_corpus
        hc = synthetic_corpus(B, seed=4321 + rank)  # a host batch in the collated layout (input data, untimed)
        lut = default_lut().astype(np.float32) * np.float32(1.0 / 255.0)
        ha = torch.from_numpy(hc.audio).pin_memory()
        hi = torch.from_numpy(lut[hc.image.astype(np.int64)]).reshape(B, 1, 28, 28).pin_memory()
        hl = torch.from_numpy(hc.labels).pin_memory()

        def one_h2d():
            step.A.copy_(ha, non_blocking=True)
            step.I.copy_(hi, non_blocking=True)
            step.labels.copy_(hl, non_blocking=True)
            step.run()
        one_h2d()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.pcie_steps):
            one_h2d()
        torch.cuda.synchronize()
        el = time.perf_counter() - t1
        pcie = {"samples_per_s": round(B * args.pcie_steps / el, 1), "ms_per_step": round(el / args.pcie_steps * 1e3, 4),
                "h2d_bytes_per_step": int(ha.numel() * 4 + hi.numel() * 4 + hl.numel() * 8),
                "what": "pinned host batch (audio f32 [B,32,94], image f32 [B,1,28,28], labels i64) copied with "
                        "hipMemcpyAsync into the step's inputs each step, then the same captured step (not value)"}

    traffic, traffic_launches, traffic_src = pmc_traffic("conv")
    loss = step.loss.item()
    result = None
    if rank == 0:
        rl = {"bound": "mfma", "kernel": "conv implicit-GEMM family (k_fwd_lds, k_fwd_pair_lds = a downsampling "
                                         "block's conv1 + 1x1 downsample, k_bwd_lds = dgrad+wgrad, k_bwd_quad_lds = "
                                         "conv2 + downsample dgrad+wgrad, k_dgrad_lds, k_wgrad_lds, stem k_stem_* / "
                                         "k_conv_*; the variant-4 builds k_*_x9 form each fp32 product from an exact "
                                         "3-piece bf16 split, 9 bf16 MFMA 32x32x16 per 16-deep step), fp32 MFMA "
                                         "32x32x2; peak = the fp32 MFMA peak for the whole family",
              "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "traffic": traffic,
              "traffic_unit": "HBM bytes per step of the conv family (PMC: 2 x FETCH_SIZE + WRITE_SIZE)",
              "traffic_per_launch": round(traffic / traffic_launches) if traffic else None,
              "traffic_source": traffic_src,
              "step_valid_tflops_per_gpu": round(step_tflops, 3),
              "step_frac_of_peak": round(step_tflops / FP32_MFMA_PEAK_TFLOPS, 4),
              "which_is_which": "frac / achieved / r34_3x3: conv kernels' device time in a ONE-stream re-capture of "
                                "the step (carried Adam and the audio LDS floor off, each kernel alone on the chip; "
                                "reads ~2 % above a rocprofv3 recompute of the same schedule, r*_roofline_from_trace"
                                ".txt); step_frac_of_peak: valid FLOPs of the TIMED two-stream step / ms_per_step",
              "timing": f"device kernel durations (torch.profiler: the rocprofiler timestamps) of {R} replays of the "
                        "step captured on ONE stream after the timed region (each kernel alone on the chip, as "
                        "under rocprofv3 kernel tracing); conv_ms_per_step = summed conv-kernel durations per step; "
                        "r34_3x3 = the ResNet34 3x3 launches of the same replays (single stream: exact launch "
                        "attribution)"}
        if roof is not None:
            ach = roof["achieved"]
            rl.update({"achieved": round(ach, 3), "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                       "conv_ms_per_step": round(roof["conv_kernel_ms_per_step"], 4),
                       "x9_conv_ms_per_step": round(roof["x9_conv_ms_per_step"], 4),
                       # the variant-4 kernels' own ceiling in fp32 products: dense bf16 MFMA 2.5 PF / 9 piece
                       # products per fp32 product (frac above keeps the f32 MFMA peak for the whole family)
                       "x9_fp32_product_peak_tflops": round(2500.0 / 9, 1),
                       "valid_tap_flop_per_step": roof["valid_tap_flop_per_step"],
                       "launches_per_step": roof["conv_launches_per_step"],
                       "kernels_per_step": roof["kernels_per_step"],
                       "kernel_ms_per_step_by_family": {k: round(v, 4) for k, v in roof["families"].items()},
                       "benched_two_stream_graph_kernel_ms_per_step_by_family":
                           {k: round(v, 4) for k, v in roof["concurrent"].items()}})
            r34 = subset_roofline(roof["per_launch"], lambda name, op: name == "image" and op.shape.r == 3,
                                  FP32_MFMA_PEAK_TFLOPS)
            if r34 is not None:
                r34["what"] = ("ResNet34 (image encoder) 3x3 convs: fwd + dgrad + wgrad launches, valid-tap FLOPs / "
                               "their device time (north_star target >= 0.70)")
            rl["r34_3x3"] = r34
            rl["mfma_counters"] = {f"b{b}": mfma_counters(b) for b in sorted({B, 128, 1024})}
            # the HBM-bound families: algorithmic bytes per step, PMC HBM bytes per step and the
            # achieved rate over their device time (same replays as above)
            bn_elems = 217728 * B  # BN(+ReLU/+add) elements per step (both encoders)
            n_par = sum(p.numel() for p in model.parameters())
            algo = {"bn": (8 + 12) * bn_elems, "pool": int(0.30e6 * B), "adam": 28 * n_par}
            hbm = {}
            for fam, abytes in algo.items():
                ms = roof["families"].get(fam)
                pb, _, psrc = pmc_traffic(fam)
                if not ms:
                    continue
                hbm[fam] = {"algorithmic_bytes": abytes, "pmc_bytes": pb,
                            "device_ms": round(ms, 4),
                            "algorithmic_GBps": round(abytes / (ms * 1e-3) / 1e9, 1),
                            "pmc_GBps": round(pb / (ms * 1e-3) / 1e9, 1) if pb else None,
                            "frac_of_8TBps": round(abytes / (ms * 1e-3) / 8e12, 4)}
            if hbm:
                hbm["what"] = ("BN: 8 B/elem fwd + 12 B/elem bwd x 217,728 elems/sample; pool: 0.30 MB/sample; Adam: "
                               "28 B/param; pmc_bytes from the same PMC summary as traffic_source")
                rl["hbm_families"] = hbm
            rl["profiled_steps"] = roof["profiled_steps"]
            rl["incomplete_steps_dropped"] = roof["incomplete_steps_dropped"]
            if roof.get("attribution_failed"):
                rl["attribution_failed"] = roof["attribution_failed"]
            if args.kernel_table and roof["per_launch"]:
                from tspm_amd.roofline import launch_flops
                rows = []
                for name, op, kind, us in roof["per_launch"]:
                    s_ = op.shape
                    rows.append({"engine": name, "kind": kind,
                                 "shape": [s_.n, s_.h, s_.w, s_.c, s_.k, s_.r, s_.s, s_.stride],
                                 "us": round(us, 3), "gflop": round(launch_flops(op, kind) / 1e9, 4),
                                 "tflops": round(launch_flops(op, kind) / (us * 1e-6) / 1e12, 2) if us else None})
                with open(args.kernel_table, "w") as f:
                    json.dump({"batch": B, "rows": rows}, f, indent=1)
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "dtype_note": "fp32 storage, fp32 products, fp32 accumulation; the variant-4 conv kernels (k_*_x9) form each "
                          "fp32 product exactly from a three-piece bf16 split on the bf16 MFMA (DESIGN 3.1; "
                          "tests/test_gpu_split.py: single products bit-exact, error vs fp64 at the f32 MFMA's level)",
            "data": f"synthetic AVMNIST-shaped corpus of {args.corpus} samples resident in HBM (audio f32 [32,94] "
                    "log-normal-ish, image uint8 [28,28]); each step gathers a shuffled batch on device "
                    "(colormap LUT, 1/255, masks) into the step's inputs; random-init weights (seed 0)",
            "config": {"workload": "avmnist_late_fusion_train_step(resnet18_audio+resnet34_image+mlp_head, CE, Adam)",
                       "per_rank_batch": B, "global_batch": B * world, "parallelism": f"dp{world}",
                       "graph": not args.no_graph},
            "roofline": rl,
            "exchange": exchange,
            "pcie_inclusive": pcie,
            "final_loss": round(loss, 5),
            "process_group": process_group_info(),
        }
        if world > 1:
            rl["timing"] += ("; at N > 1 rank 0 profiles its local step (the same conv launches without the "
                             "collective) after the timed region while the other ranks wait")
    if rank == 0 and not args.no_cpu_baseline:
        # the reference CPU train step on this host (rank 0 only, every N: north_star's 'alongside the reference
        # CPU train step'); the other ranks sleep in the gloo barrier below meanwhile
        result["cpu_baseline"] = cpu_baseline(B, args.cpu_budget)
        if world > 1:
            result["cpu_baseline"]["note"] = (f"timed on rank 0's host after the timed region, the other {world - 1} "
                                              "ranks idle in a gloo barrier")
    if rank == 0:
        emit(result)
    if cpu_group is not None:
        dist.barrier(group=cpu_group)
    # explicit teardown order: every stream idle, graphs and step flags released, THEN the
    # process group
    step.close()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
