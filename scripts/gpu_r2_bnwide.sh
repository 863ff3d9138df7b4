# BN "wide" launch shapes: full GPU suite, then alternating A/B bench runs of the headline step (TSPM_BN_WIDE=0/1).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1
for i in 1 2; do
  for w in 0 1; do
    TSPM_BN_WIDE=$w timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bnwide${w}_$i.json 2> gpurun_out/bnwide${w}_$i.err
  done
done
