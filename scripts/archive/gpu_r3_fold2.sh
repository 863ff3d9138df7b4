# bn1 fold v2 (compile-time BNIN kernels, table reads hoisted to load time, prologue loads ahead of the
# stage loads) + phased DP structure: tests, then A/B bench lines.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bnfold.py tests/test_gpu_phased.py tests/test_gpu_model.py tests/test_gpu_mono.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/f2_t.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 100 --kernel-table gpurun_out/f2_fold_kt$i.json > gpurun_out/f2_fold_$i.json 2> gpurun_out/f2_fold_$i.err
  TSPM_BN_FOLD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 100 --kernel-table gpurun_out/f2_nofold_kt$i.json > gpurun_out/f2_nofold_$i.json 2> gpurun_out/f2_nofold_$i.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/f2_ph_one.json 2> gpurun_out/f2_ph_one.err
TSPM_PHASED_FORCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/f2_ph_noar.json 2> gpurun_out/f2_ph_noar.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/f2_plain.json 2> gpurun_out/f2_plain.err
