# Current bench lines of every workload (r2_v6): headline (with the HBM-bound family entries), per-rank
# batch 1024, monomodal, MMIMDb, MOSI, MOSEI; MOSEI rocprofv3 kernel stats.
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline > $O/r2_v6_bench_nocpu.json 2> $O/r2_v6_bench_nocpu.err
timeout -k 10 300 python3 $R/bench.py --batch-per-rank 1024 --steps 20 --warmup 5 --no-cpu-baseline --pcie-steps 0 --kernel-table $O/r2_v6_kernel_table_b1024.json > $O/r2_v6_bench_b1024.json 2> $O/r2_v6_bench_b1024.err
timeout -k 10 300 python3 $R/bench.py --mono > $O/r2_v6_mono.json 2> $O/r2_v6_mono.err
timeout -k 10 300 python3 $R/bench.py --mmimdb > $O/r2_v6_mmimdb_bench.json 2> $O/r2_v6_mmimdb_bench.err
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r2_v6_mosei_prof -o run -- python3 $R/bench.py --mosi --mosei --no-cpu-baseline > $O/r2_v6_mosei_prof.json 2> $O/r2_v6_mosei_prof.err
