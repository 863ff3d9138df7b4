"""Run scripts/accuracy_parity.py for many seeds as concurrent single-seed processes on ONE GPU.

One ATen reference run keeps the MI355X mostly idle (batch-128 ResNet kernels, host-bound launches), so
several seeds share the card.  Each child runs one seed under its own time limit; a progress line is
printed every 30 s; the first failing child stops the launch of new ones (no retries).

  python scripts/acc_par.py --jobs 8 --limit 1000 -- reference --device cuda --epochs 20 --seeds 0-47
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "gpurun_out")


def _seeds(spec: str):
    out = []
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--limit", type=int, default=900, help="seconds per child")
    ap.add_argument("--deadline", type=int, default=0, help="stop launching new seeds after this many seconds")
    ap.add_argument("--script", default="accuracy_parity.py", help="the per-seed script under scripts/")
    ap.add_argument("rest", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    rest = a.rest[1:] if a.rest and a.rest[0] == "--" else a.rest
    i = rest.index("--seeds")
    seeds, base = _seeds(rest[i + 1]), rest[:i] + rest[i + 2:]
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ, OMP_NUM_THREADS="2")
    pending, running, done, failed = list(seeds), {}, [], []
    t0 = time.time()
    last = 0.0
    while pending or running:
        while pending and len(running) < a.jobs and not failed and not (a.deadline and time.time() - t0 > a.deadline):
            s = pending.pop(0)
            log = open(os.path.join(OUT, f"accpar_{a.script[:-3]}_{base[0]}_s{s}.log"), "w")
            cmd = ["timeout", "-k", "10", str(a.limit), sys.executable, "-u", os.path.join(HERE, a.script)]
            running[s] = (subprocess.Popen(cmd + base + ["--seeds", str(s)], stdout=log, stderr=subprocess.STDOUT,
                                           env=env), log)
        if a.deadline and time.time() - t0 > a.deadline:
            pending = []
        for s, (p, log) in list(running.items()):
            rc = p.poll()
            if rc is not None:
                log.close()
                del running[s]
                (done if rc == 0 else failed).append((s, rc))
        if failed:
            pending = []
        if time.time() - last > 30:
            last = time.time()
            print(f"[{time.time() - t0:6.0f}s] done {len(done)} running {sorted(running)} pending {len(pending)} "
                  f"failed {failed}", flush=True)
        time.sleep(1)
    print(f"finished in {time.time() - t0:.0f}s: done {sorted(s for s, _ in done)} failed {failed}", flush=True)
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
