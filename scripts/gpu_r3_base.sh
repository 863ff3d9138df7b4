# Round-3 session-2 baseline of the restored tree: smoke, full GPU suite, headline bench line with the
# per-launch table, and the stream/queue probe (24 steps built and freed in turn: verdict r2 item 8).
set -e
mkdir -p gpurun_out
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3b_smoke.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b_t.log 2>&1
timeout -k 10 300 python -u bench.py --kernel-table gpurun_out/r3b_kernel_table_b128.json > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err
timeout -k 10 300 python -u scripts/stream_queue_probe.py --steps 24 --delete > gpurun_out/r3b_stream_probe_delete.log 2>&1
