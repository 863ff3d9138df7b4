#!/bin/bash
# Variant-4 sign alternation: bias + split tests + step-vs-oracle, then an alternating-process A/B of the product
# build against libtspm_alt.so (built with ALT_FLAGS, e.g. the round's previous per-stage form).
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6g}
timeout -k 10 200 python -u scripts/split_bias.py > gpurun_out/${T}_bias.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_split_tests.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread -k "oracle" > gpurun_out/${T}_model.log 2>&1
P=task-specific-pretraining-multimodal_amd
if [ -f $P/libtspm_alt.so ]; then
  timeout -k 10 700 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm_alt.so --b $P/libtspm.so -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
fi
