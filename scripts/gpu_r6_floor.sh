#!/bin/bash
# Round 6: the audio LDS floor re-measured on the round-6 step (in-process A/B, alternating rounds).
set -e
mkdir -p gpurun_out
T=${1:-r6j}
timeout -k 10 600 python -u scripts/ab_step.py --rounds 8 --k 50 --variants 'f82k:{}' 'f0:{"_floor":0}' \
  'f60k:{"_floor":60000}' 'f100k:{"_floor":100000}' > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab.json')); print({k: v['median'] for k, v in d['ms_per_step'].items()})"
timeout -k 10 200 python -u scripts/overlap_probe.py --dump gpurun_out/${T}_step_dump.txt > gpurun_out/${T}_overlap.json 2> gpurun_out/${T}_overlap.err
