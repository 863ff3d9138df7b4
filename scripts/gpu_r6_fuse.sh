#!/bin/bash
# Round 6: the paired forward / quad backward launches and the >128-tile BN partials — kernel tests, step tests, A/B.
set -e
mkdir -p gpurun_out
T=${1:-r6c}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fwd_pair.py \
  tests/test_gpu_bwd_quad.py tests/test_gpu_bn_dgrad_part.py "tests/test_gpu_model.py::test_fused_step_vs_oracle" \
  "tests/test_gpu_model.py::test_graph_replay_equals_eager" > gpurun_out/${T}_tests.log 2>&1
tail -2 gpurun_out/${T}_tests.log
TSPM_FWD_PAIR=0 TSPM_BWD_QUAD=0 timeout -k 10 500 python -u scripts/ab_step.py --rounds 8 --k 50 --variants \
  'base:{}' 'bnp1024:{"_bnpt":1024}' 'bnp256:{"_bnpt":256}' > gpurun_out/${T}_ab_tiles.json 2> gpurun_out/${T}_ab_tiles.err
cat gpurun_out/${T}_ab_tiles.json | python -c "import json,sys; d=json.load(sys.stdin); print({k: v['median'] for k, v in d['ms_per_step'].items()})"
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --b task-specific-pretraining-multimodal_amd/libtspm.so \
  --env-b TSPM_FWD_PAIR=0,TSPM_BWD_QUAD=0 -- --steps 200 > gpurun_out/${T}_ab_fuse.json 2> gpurun_out/${T}_ab_fuse.err
python -c "import json; d=json.load(open('gpurun_out/${T}_ab_fuse.json')); print(d['ms_per_step'])"
