# A/B of two libtspm builds on one box: conv/model GPU tests on the new build, then alternating bench lines.
# usage: bash scripts/gpu_r3_ab.sh <tag> <alt_lib>
set -e
mkdir -p gpurun_out
TAG=$1; ALT=$2
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --kernel-table gpurun_out/${TAG}_new_kt$i.json > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err
  TSPM_LIB=$ALT timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --kernel-table gpurun_out/${TAG}_old_kt$i.json > gpurun_out/${TAG}_old_$i.json 2> gpurun_out/${TAG}_old_$i.err
done
