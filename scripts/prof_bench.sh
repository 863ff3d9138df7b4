#!/bin/bash
# The committed evidence for bench.py's roofline line: (1) the default bench line, (2) rocprofv3
# --kernel-trace --stats over the same bench command (CPU baseline off: it launches no kernels),
# (3) PMC FETCH_SIZE / WRITE_SIZE passes (separate runs).  Each step under its own time limit; the
# script stops at the first failure.  The profiled runs (2, 3) use the optimizer's own Adam launches
# (TSPM_ADAM_CARRY=none) and no audio LDS floor (TSPM_SLACK_LDS_FLOOR=0), as bench.py's one-stream roofline
# re-capture does: rocprofv3's kernel tracing serialises the two streams, so the floor (there to leave CU room to
# the concurrent image chain) would only slow the audio convs, and the conv kernels hold conv work alone (the
# benched step carries finished blocks' Adam updates inside later backward launches, step.AdamCarry).
# usage: scripts/prof_bench.sh TAG [extra bench args]
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python3 $R/bench.py "$@" --kernel-table $O/${TAG}_kernel_table.json > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit $?
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python3 $R/bench.py "$@" --no-cpu-baseline > $O/${TAG}_prof.json 2> $O/${TAG}_prof.err || exit $?
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/${TAG}_pmc_fetch -o run -- python3 $R/bench.py "$@" --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${TAG}_pmc_fetch.log 2>&1 || exit $?
TSPM_ADAM_CARRY=none TSPM_SLACK_LDS_FLOOR=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/${TAG}_pmc_write -o run -- python3 $R/bench.py "$@" --steps 3 --warmup 2 --no-cpu-baseline --profile-steps 0 --pcie-steps 0 > $O/${TAG}_pmc_write.log 2>&1
