# Register-staged loader: RS stages in flight with a straight-line full-trip loop (default RS 4/3,
# libtspm_rs3 = 3, libtspm_rs2n = 2 with the new loop, libtspm_rs2 = the previous loop) — conv/model
# tests on the default, A/B bench lines (fold off everywhere, fold on for the default), phased diagnostics.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_bnfold.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/rs_t.log 2>&1
L=$PWD/task-specific-pretraining-multimodal_amd
for i in 1 2; do
  for v in main rs3 rs2n rs2; do
    if [ $v = main ]; then lib=$L/libtspm.so; else lib=$L/libtspm_$v.so; fi
    TSPM_BN_FOLD=0 TSPM_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/rs_${v}_kt$i.json > gpurun_out/rs_${v}_$i.json 2> gpurun_out/rs_${v}_$i.err
  done
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/rs_fold_kt$i.json > gpurun_out/rs_fold_$i.json 2> gpurun_out/rs_fold_$i.err
done
for d in wait nowait inline; do
  TSPM_PHASED_DIAG=$d TSPM_PHASED_FORCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/fe_ph_$d.json 2> gpurun_out/fe_ph_$d.err
done
