#!/bin/bash
# Round 6: finalize with 16-deep tile batches + apply_merge with batched row loads (both bitwise the old arithmetic):
# the affected kernel tests, then an alternating-process A/B of the two builds in the captured step.
set -e
mkdir -p gpurun_out
T=${1:-r6k}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bn_apply_merge.py tests/test_gpu_ops.py -k "bn or merge" > gpurun_out/${T}_tests.log 2>&1
P=task-specific-pretraining-multimodal_amd
timeout -k 10 900 python -u scripts/ab_lib.py --rounds 6 --a $P/libtspm_alt.so --b $P/libtspm.so -- --steps 200 > gpurun_out/${T}_ab.json 2> gpurun_out/${T}_ab.err
tail -c 600 gpurun_out/${T}_ab.json
