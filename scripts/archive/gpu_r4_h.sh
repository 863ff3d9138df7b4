#!/bin/bash
# Round-4: stem band kernels (forward + weight gradient, variant 3) and the head staging / CE changes — their
# tests, the head's phase stamps, and an in-step A/B of the stems.  usage: bash scripts/gpu_r4_h.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_head.py tests/test_gpu_ops.py -k "stem or head" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 200 python3 -u scripts/head_bench.py --stamps > gpurun_out/${T}_head_stamps.txt 2> gpurun_out/${T}_head_stamps.err
timeout -k 10 300 python3 -u scripts/ab_step.py --variants 'gather:{}' 'band:{"_stem":[0,0,0,0,0,3]}' 'band2:{"_stem":[0,0,0,0,0,3],"_stemw":[0,0,0,0,0,3]}' --rounds 8 --k 50 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_mtA$i.json 2> gpurun_out/${T}_mtA$i.err
  TSPM_LIB=$GRAFT_REPO_ROOT/task-specific-pretraining-multimodal_amd/libtspm_mt128.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_mtB$i.json 2> gpurun_out/${T}_mtB$i.err
done
