# Fragment prefetch: timing only (the model test fails at audio-128: debugging only if it pays)
set -e
mkdir -p gpurun_out
L=$PWD/task-specific-pretraining-multimodal_amd
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/fp_on_kt$i.json > gpurun_out/fp_on_$i.json 2> gpurun_out/fp_on_$i.err
  TSPM_LIB=$L/libtspm_nofp.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/fp_off_kt$i.json > gpurun_out/fp_off_$i.json 2> gpurun_out/fp_off_$i.err
done
