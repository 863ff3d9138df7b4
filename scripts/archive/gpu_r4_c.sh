#!/bin/bash
# Round-4 check of the pruned tree: the whole GPU suite, the adam_split A/B, layer4's span in the benched
# graph and the kineto overlap probe.  Every GPU step under its own limit; the first failure ends the call.
# usage: bash scripts/gpu_r4_c.sh TAG [pytest selection]
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1; SEL=${2:-tests}
timeout -k 10 900 python3 -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_suite.log 2>&1
timeout -k 10 240 python3 -u scripts/ab_step.py --variants 'plain:{}' 'split:{"adam_split":true}' 'phase:{"adam_split":"phase"}' --rounds 8 --k 50 > gpurun_out/${T}_ab_split.json 2> gpurun_out/${T}_ab_split.err
timeout -k 10 200 python3 -u scripts/layer_span.py --replays 20 > gpurun_out/${T}_layer_span.json 2> gpurun_out/${T}_layer_span.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
