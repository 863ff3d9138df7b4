#!/bin/bash
# Round-4: head weight-gradient launch on the image stream (ABI 17 parts), early head staging, 16-row BN partial
# batches for long tiles — their tests, two bench lines and a one-stream rocprofv3 trace.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_head.py tests/test_gpu_model.py tests/test_abi.py tests/test_gpu_ops.py -k "bn or stem or head or model or abi or adam" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err
done
timeout -k 10 200 python3 -u scripts/head_bench.py > gpurun_out/${T}_head.txt 2> gpurun_out/${T}_head.err
cd /tmp && export TMPDIR=/tmp
TSPM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_serial.log 2>&1
