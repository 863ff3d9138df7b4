#!/bin/bash
# Round 6: the whole BN backward in the dgrad epilogue for short maps — kernel tests, step tests, A/B.
set -e
mkdir -p gpurun_out
T=${1:-r6g}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_dgrad_part.py -k whole \
  \
  \
  > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u scripts/ab_step.py --rounds 8 --k 50 --variants 'off:{}' 'r128:{"_bnx":128}' 'r512:{"_bnx":512}' \
  > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab.json')); print({k: v['median'] for k, v in d['ms_per_step'].items()})"
