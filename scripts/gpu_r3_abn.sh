# Alternating bench lines for several libtspm builds on one box (no CPU baseline), kernel tables kept.
# usage: bash scripts/gpu_r3_abn.sh <tag> <rounds> <name=lib> [<name=lib> ...]; optional TESTLIB=<lib> runs the
# conv/model GPU tests against that build first.
set -e
mkdir -p gpurun_out
TAG=$1; R=$2; shift 2
if [ -n "$TESTLIB" ]; then
  TSPM_LIB=$TESTLIB timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
fi
for i in $(seq 1 $R); do
  for nl in "$@"; do
    n=${nl%%=*}; l=${nl#*=}
    TSPM_LIB=$l timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 50 --kernel-table gpurun_out/${TAG}_${n}_kt$i.json > gpurun_out/${TAG}_${n}_$i.json 2> gpurun_out/${TAG}_${n}_$i.err
  done
done
