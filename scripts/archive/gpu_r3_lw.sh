# Loader variants at three batch sizes: register-staged loader waves (default), LDS-DMA loader waves
# (libtspm_lw1.so: round 2's late default), single-role LDS-DMA (libtspm_lw0.so).
set -e
mkdir -p gpurun_out
L=$PWD/task-specific-pretraining-multimodal_amd
for v in main lw1 lw0; do
  if [ $v = main ]; then lib=$L/libtspm.so; else lib=$L/libtspm_$v.so; fi
  TSPM_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 > gpurun_out/lw_b128_$v.json 2> gpurun_out/lw_b128_$v.err
  TSPM_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 1024 --steps 15 --profile-steps 3 > gpurun_out/lw_b1024_$v.json 2> gpurun_out/lw_b1024_$v.err
  TSPM_LIB=$lib timeout -k 10 200 python -u bench.py --mono --no-cpu-baseline > gpurun_out/lw_mono_$v.json 2> gpurun_out/lw_mono_$v.err
done
