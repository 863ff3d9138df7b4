#!/bin/bash
# Round-4: stem kernels without integer divisions — stem tests, stamps, and two bench lines.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -k "stem" "tests/test_gpu_model.py::test_fused_step_vs_oracle" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 200 python3 -u scripts/stem_bench.py --stamps > gpurun_out/${T}_stem_bench.json 2> gpurun_out/${T}_stem_bench.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench$i.json 2> gpurun_out/${T}_bench$i.err
done
