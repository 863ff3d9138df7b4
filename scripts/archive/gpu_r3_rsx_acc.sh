# Two register stages for the low-VGPR dgrad / wgrad kernels (three elsewhere): conv/model tests, two bench
# lines with kernel tables; then an accuracy batch (scripts/gpu_r3_acc_c.sh).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rx_t.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/rx_kt$i.json > gpurun_out/rx_$i.json 2> gpurun_out/rx_$i.err
done
bash scripts/gpu_r3_acc_c.sh "$@"
