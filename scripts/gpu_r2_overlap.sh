# Re-measure the Adam-overlap options on the final tree (TSPM_OVERLAP_OPT = 0 / main / stream), 2 rounds.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  for o in 0 main stream; do
    TSPM_OVERLAP_OPT=$o timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/ovl_${o}_$i.json 2> gpurun_out/ovl_${o}_$i.err
  done
done
