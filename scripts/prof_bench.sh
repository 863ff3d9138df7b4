#!/bin/bash
# The committed evidence for bench.py's roofline line: (1) the default bench line, (2) rocprofv3
# --kernel-trace --stats over the same bench command (CPU baseline off: it launches no kernels),
# (3) PMC FETCH_SIZE / WRITE_SIZE passes (separate runs).  Each step under its own time limit; the
# script stops at the first failure.  usage: scripts/prof_bench.sh TAG [extra bench args]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 $R/bench.py "$@" --kernel-table $O/${TAG}_kernel_table.json > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/${TAG}_prof.json 2> $O/${TAG}_prof.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_pmc_fetch -o run -- python3 $R/bench.py "$@" --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${TAG}_pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_pmc_write -o run -- python3 $R/bench.py "$@" --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${TAG}_pmc_write.log 2>&1
