# Round-3 baseline check of the tree: smoke, full GPU suite, headline bench line.
set -e
mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_t.log 2>&1
timeout -k 10 300 python -u bench.py --kernel-table gpurun_out/r3_v0_kernel_table_b128.json > gpurun_out/r3_v0_bench.json 2> gpurun_out/r3_v0_bench.err
