# MMIMDb kernel stats (compare the BatchNorm1d launches with round 1's r1_v11 profile) + two bench lines.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 200 python3 $R/bench.py --mmimdb --no-cpu-baseline > $O/r2_v7_mmimdb_a.json 2> $O/r2_v7_mmimdb_a.err
timeout -k 10 200 python3 $R/bench.py --mmimdb --no-cpu-baseline > $O/r2_v7_mmimdb_b.json 2> $O/r2_v7_mmimdb_b.err
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r2_v7_mmimdb_prof -o run -- python3 $R/bench.py --mmimdb --no-cpu-baseline > $O/r2_v7_mmimdb_prof.json 2> $O/r2_v7_mmimdb_prof.err
