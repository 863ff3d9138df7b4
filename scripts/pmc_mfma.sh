#!/bin/bash
# MFMA utilisation and stall counters of the train step's kernels (verdict r3 item 3; north_star's
# "rocprof reports ... MFMA utilisation on the conv kernels against gfx950 peak").  Two SQ passes, each
# its own run (MI355X_MICROARCH.md "rocprofv3 PMC slots": at most 8 SQ + 2 GRBM counters per pass):
#   issue:  where wave time goes (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY) + MFMA busy
#   lds:    LDS issue stalls, bank conflicts, LDS-array cycles
# Summarise with: python scripts/pmc_mfma.py gpurun_out/<TAG>_issue gpurun_out/<TAG>_lds > profiles/<TAG>_mfma_busy.json
# The profiled runs use the optimizer's own Adam launches (TSPM_ADAM_CARRY=none; see prof_bench.sh).
# usage: scripts/pmc_mfma.sh TAG [extra bench args]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
ARGS="--steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0"
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $O/${TAG}_issue -o run -- python3 $R/bench.py $ARGS "$@" > $O/${TAG}_issue.log 2>&1 || exit $?
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/${TAG}_lds -o run -- python3 $R/bench.py $ARGS "$@" > $O/${TAG}_lds.log 2>&1
