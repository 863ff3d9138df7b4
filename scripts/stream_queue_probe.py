"""Build several FusedTrainSteps in one process and time each alone (graph replays, batch 128).  Each step
takes three streams from PyTorch's pool, and HIP spreads streams over GPU_MAX_HW_QUEUES (4) hardware queues
round-robin: a step whose two encoder streams share a queue loses the audio/image overlap.  Prints the
per-step time with the streams' ids.

    python scripts/stream_queue_probe.py --steps 8
"""
import argparse
import gc
import os
import statistics
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), HERE]
from tune_in_step import build, time_steps  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--delete", action="store_true", help="free each step before building the next (the tuner's pattern)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    steps = []
    for i in range(a.steps):
        st = build({**__import__("tspm_amd").engine.tuned_table()}, dev)
        ids = [s.stream_id for s in (st.side, st.aux_a, st.aux_i)]
        t = statistics.median(time_steps(st, 30) for _ in range(3))
        print(f"step {i}: {t:8.1f} us/step  streams side/aux_a/aux_i {ids}", flush=True)
        if a.delete:
            del st
            gc.collect()
            torch.cuda.empty_cache()
        else:
            steps.append(st)
    if steps:
        print("re-timed, all alive:", [round(statistics.median(time_steps(st, 30) for _ in range(3)), 1) for st in steps],
              flush=True)
    del steps
    gc.collect()


if __name__ == "__main__":
    main()
