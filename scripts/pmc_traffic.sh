#!/bin/bash
# HBM traffic of the train step from PMC counters (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and
# WRITE_SIZE in separate passes (they cannot share the 4 TCC slots), each over a short bench run.
# Summarise with: python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
ARGS="--steps 3 --warmup 2 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_write.log 2>&1
