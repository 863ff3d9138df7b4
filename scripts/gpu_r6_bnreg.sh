#!/bin/bash
# Round 6: the BN backward apply kernel's register use (rolled coefficient reduction, per-G merge batches) — tests,
# then library A/Bs: the default build vs the prefetching build, and vs the previous commit's library.
set -e
mkdir -p gpurun_out
T=${1:-r6i}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_dgrad_part.py \
  tests/test_gpu_bn_src.py "tests/test_gpu_model.py::test_fused_step_vs_oracle" > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --b $P/libtspm_alt.so -- --steps 200 > gpurun_out/${T}_ab_prefetch.json 2> gpurun_out/${T}_ab_prefetch.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab_prefetch.json')); print('A=default B=prefetch', d['ms_per_step'])"
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --b $P/libtspm_head.so -- --steps 200 > gpurun_out/${T}_ab_head.json 2> gpurun_out/${T}_ab_head.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab_head.json')); print('A=default B=head', d['ms_per_step'])"
