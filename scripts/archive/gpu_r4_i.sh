#!/bin/bash
# Round-4: stem band kernels in the tables + 128 BN merge tiles: the BN / stem / model tests, the stems in
# isolation, the step with 128 (default) vs 64 merge tiles (two libraries, alternating), a one-stream rocprofv3 trace.
# usage: bash scripts/gpu_r4_i.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ops.py -k "bn or stem" tests/test_gpu_model.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 200 python3 -u scripts/stem_bench.py > gpurun_out/${T}_stem_bench.json 2> gpurun_out/${T}_stem_bench.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_mtA$i.json 2> gpurun_out/${T}_mtA$i.err
  TSPM_LIB=$GRAFT_REPO_ROOT/task-specific-pretraining-multimodal_amd/libtspm_mt64.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_mtB$i.json 2> gpurun_out/${T}_mtB$i.err
done
cd /tmp && export TMPDIR=/tmp
TSPM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_serial.log 2>&1
