#!/bin/bash
# Round 6: the stem BN partial sums gathered through the max pool — kernel test, step tests, A/B.
set -e
mkdir -p gpurun_out
T=${1:-r6f}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_dgrad_part.py \
  "tests/test_gpu_model.py::test_fused_step_vs_oracle" "tests/test_gpu_model.py::test_graph_replay_equals_eager" \
  > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u scripts/ab_step.py --rounds 8 --k 50 --variants 'on:{}' 'off:{"_bnps":0}' \
  > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab.json')); print({k: v['median'] for k, v in d['ms_per_step'].items()})"
