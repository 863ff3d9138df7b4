# bn1 fold into conv2's loader (ABI 15) + one-graph phased DP step: new tests, full GPU suite, A/B bench
# lines (fold on / off, phased one / split), and a probe of the ATen reference's speed (accuracy runs).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bnfold.py tests/test_gpu_phased.py -x -q --timeout 200 --timeout-method thread > gpurun_out/f1_new.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f1_t.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 100 --kernel-table gpurun_out/f1_fold_kt$i.json > gpurun_out/f1_fold_$i.json 2> gpurun_out/f1_fold_$i.err
  TSPM_BN_FOLD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 100 > gpurun_out/f1_nofold_$i.json 2> gpurun_out/f1_nofold_$i.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/f1_ph_one.json 2> gpurun_out/f1_ph_one.err
TSPM_PHASED=split timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/f1_ph_split.json 2> gpurun_out/f1_ph_split.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/f1_plain_np.json 2> gpurun_out/f1_plain_np.err
