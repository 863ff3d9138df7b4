#!/bin/bash
# Quick GPU check used while iterating: selected GPU tests, two bench lines, and a rocprofv3 kernel
# trace of the step on one stream (TSPM_SERIAL=1).  usage: scripts/gpu_quick.sh TAG "test files" [bench args]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; TESTS=$2; shift 2
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
fi
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 "$@" > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err
done
cd /tmp && export TMPDIR=/tmp
TSPM_SERIAL=1 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 "$@" > $GRAFT_REPO_ROOT/gpurun_out/${T}_serial.log 2>&1
