#!/bin/bash
# fused last-block apply + average pool (ABI 17): its kernel test, A/B against the separate pool launch,
# then the evidence set on this tree (smoke, GPU suite, headline line + rocprofv3 + PMC, secondary lines)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_bn_pool.py -x -q --timeout 100 --timeout-method thread > gpurun_out/r4s_pool_test.log 2>&1
timeout -k 10 300 python -u scripts/ab_step.py --rounds 10 --variants 'pool:{}' 'nopool:{"_pool":false}' > gpurun_out/r4s_ab_pool.json 2> gpurun_out/r4s_ab_pool.err
bash scripts/gpu_r4_final.sh suite r4_v2
bash scripts/gpu_r4_final.sh prof r4_v2
