#!/bin/bash
# Round-4: the stem band kernel (variant 3) — its tests, an in-step A/B against the tuned gather stems, and the
# head kernel's phase stamps (diagnostic library).  usage: bash scripts/gpu_r4_g.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -k "stem" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python3 -u scripts/ab_step.py --variants 'gather:{}' 'band:{"_stem":[0,0,0,0,0,3]}' --rounds 8 --k 50 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
timeout -k 10 200 python3 -u scripts/head_bench.py --stamps > gpurun_out/${T}_head_stamps.txt 2> gpurun_out/${T}_head_stamps.err
