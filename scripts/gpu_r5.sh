#!/bin/bash
# Round-5 GPU calls.  Every GPU step runs under its own time limit; the script stops at the first failure.
#   bash scripts/gpu_r5.sh check TAG    smoke, the whole GPU suite (-s: an abort's own message reaches the log),
#                                       the default bench line, --phased (exchange block), loop-clock stamps
#   bash scripts/gpu_r5.sh suite TAG    smoke + the whole GPU suite
#   bash scripts/gpu_r5.sh bench TAG    two default bench lines (no CPU baseline) + --phased
#   bash scripts/gpu_r5.sh stamps TAG [--only ...]   loop-clock stamps of single conv launches
#   bash scripts/gpu_r5.sh dp TAG       the capture / phased / DP tests (-s), --phased bench line, loop stamps
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MODE=$1
T=$2
shift 2
STAMP_SHAPES="fwd:8,24,64,64,3,1;dgrad:8,24,64,64,3,1;wgrad:8,24,64,64,3,1;fwd:4,12,128,128,3,1;dgrad:4,12,128,128,3,1;fwd:2,2,256,256,3,1;fwd:1,1,512,512,3,1"
smoke() { timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1; }
suite() { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1; }
stamps() { timeout -k 10 240 python -u scripts/stamp_conv.py --only "${1:-$STAMP_SHAPES}" > gpurun_out/${T}_stamps.txt 2> gpurun_out/${T}_stamps.err; }
bench1() { timeout -k 10 300 python -u bench.py "$@"; }
case $MODE in
  check)
    smoke
    suite
    bench1 --kernel-table gpurun_out/${T}_kernel_table.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
    bench1 --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_phased.json 2> gpurun_out/${T}_phased.err
    stamps
    ;;
  suite)
    smoke
    suite
    ;;
  bench)
    bench1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench1.json 2> gpurun_out/${T}_bench1.err
    bench1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench2.json 2> gpurun_out/${T}_bench2.err
    bench1 --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_phased.json 2> gpurun_out/${T}_phased.err
    ;;
  stamps)
    stamps "$1"
    ;;
  dp)  # the DP / capture tests with their output visible (-s), the phased bench line, then loop stamps
    timeout -k 10 400 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_phased.py tests/test_gpu_ddp.py "tests/test_gpu_model.py::test_phased_allreduce_step_equals_plain_step" -x -q -s --timeout 300 --timeout-method thread > gpurun_out/${T}_dp_tests.log 2>&1
    bench1 --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_phased.json 2> gpurun_out/${T}_phased.err
    stamps
    ;;
esac
