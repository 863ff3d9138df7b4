# Slab reduction parallel over slabs: full GPU suite, A/B bench (TSPM_SLAB_WIDE=0/1), stem config sweep.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full2.log 2>&1
for i in 1 2; do
  for w in 0 1; do
    TSPM_SLAB_WIDE=$w timeout -k 10 240 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline --pcie-steps 0 > gpurun_out/slab${w}_$i.json 2> gpurun_out/slab${w}_$i.err
  done
done
timeout -k 10 300 python -u scripts/tune_stem.py --batch 128 --out gpurun_out/stem_tuning_b128.json > gpurun_out/stem_tuning_b128.log 2>&1
