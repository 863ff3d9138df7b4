# Hybrid batch-128 table (variant 2 for the launches that were >3 % faster with it single-stream) vs the committed one.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  TSPM_TUNED_FILE=$PWD/scripts/tables/b128_hybrid.json timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 > gpurun_out/hy_h_$i.json 2> gpurun_out/hy_h_$i.err
  TSPM_TUNED_FILE=$PWD/task-specific-pretraining-multimodal_amd/tuned/mi355x_b128.json timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 > gpurun_out/hy_v1_$i.json 2> gpurun_out/hy_v1_$i.err
done
