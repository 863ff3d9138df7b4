#!/bin/bash
# Round 5: the profiled passes of the evidence set again, with the optimizer's own Adam launches (see prof_bench.sh)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
T=$1
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- python3 $R/bench.py --no-cpu-baseline > $O/${T}_prof.json 2> $O/${T}_prof.err
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${T}_pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${T}_pmc_fetch.log 2>&1
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${T}_pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${T}_pmc_write.log 2>&1
cd $R
bash scripts/pmc_mfma.sh ${T}_b128
bash scripts/pmc_mfma.sh ${T}_b1024 --batch-per-rank 1024
