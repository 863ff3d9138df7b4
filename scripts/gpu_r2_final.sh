# End-of-round evidence: full GPU suite, smoke, then the headline bench line + rocprofv3 stats + PMC passes.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_final.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
bash scripts/prof_bench.sh r2_v5
