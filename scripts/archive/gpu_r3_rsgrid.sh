# Register stages chosen per launch by grid size (TSPM_RS3_MAX_BLOCKS: default 1024, 0 = always two, 1e9 =
# always three): conv/model tests, then the batch-128 / batch-1024 / monomodal / MOSEI lines for each bound.
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_model.py tests/test_gpu_mono.py -x -q --timeout 200 --timeout-method thread > gpurun_out/rg_t.log 2>&1
for lim in 1024 0 1000000000; do
  TSPM_RS3_MAX_BLOCKS=$lim timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/rg_b128_${lim}_kt.json > gpurun_out/rg_b128_$lim.json 2> gpurun_out/rg_b128_$lim.err
  TSPM_RS3_MAX_BLOCKS=$lim timeout -k 10 300 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 1024 --steps 15 --profile-steps 3 > gpurun_out/rg_b1024_$lim.json 2> gpurun_out/rg_b1024_$lim.err
  TSPM_RS3_MAX_BLOCKS=$lim timeout -k 10 200 python -u bench.py --mono --no-cpu-baseline > gpurun_out/rg_mono_$lim.json 2> gpurun_out/rg_mono_$lim.err
  TSPM_RS3_MAX_BLOCKS=$lim timeout -k 10 200 python -u bench.py --mosi --mosei --no-cpu-baseline > gpurun_out/rg_mosei_$lim.json 2> gpurun_out/rg_mosei_$lim.err
done
