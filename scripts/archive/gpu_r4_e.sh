#!/bin/bash
# Round-4 A/B call: Adam schedules (plain / per encoder / balanced) and the audio chain on a high-priority
# stream, with the split-schedule equality tests and two bench lines.  usage: bash scripts/gpu_r4_e.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python3 -u -m pytest "tests/test_gpu_model.py::test_adam_split_schedule_equals_plain_step" "tests/test_gpu_model.py::test_graph_replay_equals_eager" "tests/test_gpu_model.py::test_fused_step_vs_oracle" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python3 -u scripts/ab_step.py --variants 'plain:{"adam_split":false}' 'encoder:{"adam_split":"encoder"}' 'balanced:{}' --rounds 8 --k 50 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err
done
timeout -k 10 200 python3 -u scripts/overlap_probe.py > gpurun_out/${T}_overlap.json 2> gpurun_out/${T}_overlap.err
timeout -k 10 200 python3 -u scripts/layer_span.py --replays 20 > gpurun_out/${T}_layer_span.json 2> gpurun_out/${T}_layer_span.err
cd /tmp && export TMPDIR=/tmp
TSPM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $GRAFT_REPO_ROOT/gpurun_out/${T}_serial.log 2>&1
