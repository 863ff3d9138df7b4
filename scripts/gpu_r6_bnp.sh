#!/bin/bash
# Round 6: dgrad-epilogue BN backward partial sums — kernel tests, the step against the oracle, and an in-process A/B.
set -e
mkdir -p gpurun_out
T=${1:-r6b}
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bn_dgrad_part.py \
  "tests/test_gpu_model.py::test_fused_step_vs_oracle" > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u scripts/ab_step.py --rounds 8 --k 50 --variants 'on:{"_bnp":"ai"}' 'off:{"_bnp":""}' \
  'img:{"_bnp":"i"}' > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
cat gpurun_out/${T}_ab.json
