#!/bin/bash
# Kernel-trace statistics of the main bench step and of the monomodal step (rocprofv3 --kernel-trace
# --stats, no counters), then the PMC HBM-traffic passes (scripts/pmc_traffic.sh).  Each step under
# its own time limit; stops at the first failure.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_main -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_main.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_mono -o run -- python3 $R/bench.py --mono --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_mono.log 2>&1 || exit $?
bash $R/scripts/pmc_traffic.sh
