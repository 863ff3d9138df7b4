#!/bin/bash
# Host-side switches re-measured on the final tables (A = defaults, B = the switch), bench.py alternating processes.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r6env}
P=task-specific-pretraining-multimodal_amd
for kv in TSPM_ADAM_CARRY=image TSPM_ADAM_CARRY_BLOCKS=256 TSPM_FC_SPLITS=4 TSPM_BN_TWO_LEVEL=1 TSPM_BN_BWD_EPI_ROWS=0; do
  n=${kv%%=*}
  timeout -k 10 400 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b $kv -- --steps 200 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/${T}_${n}.json 2> gpurun_out/${T}_${n}.err
done
