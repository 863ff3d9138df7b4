# Fragment prefetch (3 LDS slots; libtspm_nofp.so = two slots, the committed loop): conv/model tests with a
# per-test time limit (a barrier-count mismatch would hang), then A/B bench lines.
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_bnfold.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fp_t.log 2>&1
L=$PWD/task-specific-pretraining-multimodal_amd
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/fp_on_kt$i.json > gpurun_out/fp_on_$i.json 2> gpurun_out/fp_on_$i.err
  TSPM_LIB=$L/libtspm_nofp.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/fp_off_kt$i.json > gpurun_out/fp_off_$i.json 2> gpurun_out/fp_off_$i.err
done
