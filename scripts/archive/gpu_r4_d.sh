#!/bin/bash
# Round-4 measurement call: the changed kernels' tests, the adam_split A/B, layer4's span in the benched graph,
# two bench lines, the kineto overlap probe and a one-stream rocprofv3 kernel trace.  Each GPU step under its
# own limit; the first failure ends the call.   usage: bash scripts/gpu_r4_d.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_head.py tests/test_gpu_ops.py "tests/test_gpu_model.py::test_adam_split_schedules_equal_plain_step" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 240 python3 -u scripts/ab_step.py --variants 'plain:{}' 'split:{"adam_split":true}' 'phase:{"adam_split":"phase"}' --rounds 8 --k 50 > gpurun_out/${T}_ab_split.json 2> gpurun_out/${T}_ab_split.err
timeout -k 10 200 python3 -u scripts/layer_span.py --replays 20 > gpurun_out/${T}_layer_span.json 2> gpurun_out/${T}_layer_span.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err
done
timeout -k 10 200 python3 -u scripts/overlap_probe.py > gpurun_out/${T}_overlap.json 2> gpurun_out/${T}_overlap.err
cd /tmp && export TMPDIR=/tmp
TSPM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_serial.log 2>&1
