# End-of-session check of the committed tree: smoke, full GPU suite, headline bench line (with CPU baseline).
set -e
mkdir -p gpurun_out
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_end.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_end.log 2>&1
timeout -k 10 400 python -u bench.py --kernel-table gpurun_out/r2_v8_kernel_table_b128.json > gpurun_out/r2_v8_bench.json 2> gpurun_out/r2_v8_bench.err
