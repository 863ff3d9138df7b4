# Per-launch variant choice at batch 128: the committed table (variant 1) vs every LDS entry as variant 2,
# each with the single-stream per-launch table (bench --kernel-table), two runs each.
set -e
mkdir -p gpurun_out
for i in 1 2; do
  TSPM_TUNED_FILE=$PWD/task-specific-pretraining-multimodal_amd/tuned/mi355x_b128.json timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/mx_v1_kt$i.json > gpurun_out/mx_v1_$i.json 2> gpurun_out/mx_v1_$i.err
  TSPM_TUNED_FILE=$PWD/scripts/tables/b128_all_v2.json timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/mx_v2_kt$i.json > gpurun_out/mx_v2_$i.json 2> gpurun_out/mx_v2_$i.err
done
