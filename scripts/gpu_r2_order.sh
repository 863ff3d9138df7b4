# A/B of the two encoder branches' capture order in the step graph (TSPM_ENC_ORDER=ia / ai), 3 alternating pairs.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_order.log 2>&1
for i in 1 2 3; do
  for o in ia ai; do
    TSPM_ENC_ORDER=$o timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/order_${o}_$i.json 2> gpurun_out/order_${o}_$i.err
  done
done
timeout -k 10 200 python -u scripts/encoder_timing.py > gpurun_out/encoder_timing_r2.log 2>&1
