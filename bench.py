"""Benchmark: samples/sec (node) of the AVMNIST late-fusion train step on 1..8 MI355X.

One rank per GPU (torchrun env).  Per rank: batch 128 (BASELINE.json configs[2]: global 1024 on 8
GPUs), synthetic AVMNIST-shaped inputs already resident in HBM, random-init weights (seed 0).  A
"step" = one fused train step: H2D-free batch copy into the static buffers → ResNet18(audio) ‖
ResNet34(image) forward → fusion head → cross-entropy → backward → [RCCL all-reduce] → Adam,
all in fp32 on the libtspm HIP kernels (graph-replayed).

Prints ONE JSON line on rank 0 (contract in the task statement), including:
  roofline     — the conv implicit-GEMM kernel family (dominant: ~90 % of step FLOPs): valid-tap
                 FLOPs of every conv launch of one step ÷ the summed device time of those launches,
                 timed with HIP events in an instrumented eager step run right after the timed
                 region with every launch on one stream (no concurrent kernels inside a bracket); peak = fp32 MFMA 157.3 TF/s.
  cpu_baseline — the oracle (CPU fp32 restatement of the reference train step, bit-identical to it
                 on CPU) timed on this host at batch 128, rank 0 / N=1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "samples/sec (node) AVMNIST late-fusion train step at 1/2/4/8 MI355X"
PER_RANK_BATCH = 128


def synthetic_device_batches(k: int, batch: int, seed: int, dev):
    """k distinct synthetic batches (BASELINE.md 'Synthetic inputs'), resident in HBM."""
    sys.path.insert(0, REPO)
    from oracle.avmnist_ref import synthetic_batch  # same generator the parity tests use (data only)
    import numpy as np
    lut = torch.from_numpy(np.frombuffer(open(os.path.join(REPO, "tests/golden/lut_gist_earth_L.bin"), "rb").read(),
                                         dtype=np.uint8).copy())
    out = []
    for i in range(k):
        a, im, lab, _ = synthetic_batch(batch, seed=seed + 7919 * i, lut=lut)
        out.append((a.to(dev), im.to(dev), lab.to(dev)))
    return out


class ConvTimer:
    """Records HIP events around every conv launch (fwd/dgrad/wgrad) on the launching stream."""

    def __init__(self):
        self.events = []

    def begin(self, op, kind):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        self.events.append([op, kind, e0, None])

    def end(self):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.events[-1][3] = e1

    def summarize(self):
        from tspm_amd.roofline import conv_macs
        tot_ms = 0.0
        flops = 0
        for op, kind, e0, e1 in self.events:
            s = op.shape
            _, valid = conv_macs(s.n, s.h, s.w, s.c, s.k, s.r, s.s, s.stride, s.pad)
            flops += 2 * valid
            tot_ms += e0.elapsed_time(e1)
        return len(self.events), flops, tot_ms


def cpu_baseline(batch: int, budget_s: float = 15.0):
    """Time the oracle's CPU train step (reference-equivalent) on this host's cores."""
    from oracle import avmnist_ref as orc
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
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
    return {"value": n * batch / el, "unit": "samples/sec", "cores": threads, "kind": "port",
            "sample": f"{n} oracle train steps (fwd+CE+bwd+Adam, fp32) at batch {batch} on CPU, "
                      f"{el:.1f}s, torch.set_num_threads({threads})"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-per-rank", type=int, default=PER_RANK_BATCH)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--phased", action="store_true",
                    help="at N=1, run the DP step path anyway (1-rank RCCL group, all-reduce = identity)")
    args = ap.parse_args()

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
    batches = synthetic_device_batches(4, B, 1234 + rank, dev)

    def one(i):
        a, im, lab = batches[i % len(batches)]
        step.load_batch(a, im, lab)
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

    # ---- roofline: instrumented eager step (same inputs), conv launches timed with HIP events --
    timer = ConvTimer()
    for eng in (step.eng_a, step.eng_i):
        eng.conv_timer = timer
    saved = step.use_graph
    step.use_graph = False
    saved_serial = step.serial
    saved_ar = step.allreduce
    step.serial = True  # one stream: each conv's event pair brackets that kernel alone
    step.allreduce = None  # (the instrumented step is not part of the timed region)
    a, im, lab = batches[0]
    step.load_batch(a, im, lab)
    step.run()
    step.use_graph = saved
    step.serial = saved_serial
    step.allreduce = saved_ar
    torch.cuda.synchronize()
    for eng in (step.eng_a, step.eng_i):
        eng.conv_timer = None
    n_launch, conv_flops, conv_ms = timer.summarize()
    achieved = conv_flops / (conv_ms * 1e-3) / 1e12
    nominal, valid = step_flops_per_sample()
    step_tflops = valid * B * world / (elapsed / args.steps) / 1e12 / world

    loss = step.loss.item()
    result = None
    if rank == 0:
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "samples/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "synthetic AVMNIST-shaped batches resident in HBM (audio [B,32,94] log-uniform-ish, "
                    "image uint8->LUT [B,1,28,28]), random-init weights (seed 0)",
            "config": {"workload": "avmnist_late_fusion_train_step(resnet18_audio+resnet34_image+mlp_head, CE, Adam)",
                       "per_rank_batch": B, "global_batch": B * world, "parallelism": f"dp{world}",
                       "graph": not args.no_graph},
            "roofline": {"bound": "mfma", "kernel": "conv implicit-GEMM family (k_conv_fwd_vec/gather, k_conv_dgrad, "
                                                    "k_conv_wgrad), fp32 MFMA 32x32x2",
                         "achieved": round(achieved, 3), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                         "launches_per_step": n_launch, "conv_ms_per_step": round(conv_ms, 4),
                         "valid_tap_flop_per_step": conv_flops,
                         "step_valid_tflops_per_gpu": round(step_tflops, 3),
                         "step_frac_of_peak": round(step_tflops / FP32_MFMA_PEAK_TFLOPS, 4)},
            "final_loss": round(loss, 5),
        }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(B, args.cpu_budget)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
