# 1,024-thread BN backward partial pass for the 64-channel layers: BN op tests, then alternating A/B bench
# (TSPM_BN_PART_RG64=0/1), then the full GPU suite.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "bn" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bnrg_ops.log 2>&1
for i in 1 2; do
  for w in 0 1; do
    TSPM_BN_PART_RG64=$w timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --pcie-steps 0 > gpurun_out/bnrg${w}_$i.json 2> gpurun_out/bnrg${w}_$i.err
  done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bnrg.log 2>&1
