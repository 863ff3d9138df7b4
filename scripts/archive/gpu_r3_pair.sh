# Stage pairs per barrier (libtspm_nopair.so = one barrier per stage), both with 3 register stages:
# conv/model/DP tests on the default, A/B bench lines, phased lines; then an accuracy batch (reference side).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_bnfold.py tests/test_gpu_model.py tests/test_gpu_phased.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pr_t.log 2>&1
L=$PWD/task-specific-pretraining-multimodal_amd
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/pr_pair_kt$i.json > gpurun_out/pr_pair_$i.json 2> gpurun_out/pr_pair_$i.err
  TSPM_LIB=$L/libtspm_nopair.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 --kernel-table gpurun_out/pr_nopair_kt$i.json > gpurun_out/pr_nopair_$i.json 2> gpurun_out/pr_nopair_$i.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/pr_ph_one.json 2> gpurun_out/pr_ph_one.err
TSPM_PHASED_FORCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/pr_ph_noar.json 2> gpurun_out/pr_ph_noar.err
export MIOPEN_FIND_MODE=FAST
timeout -k 10 800 python -u scripts/acc_par.py --jobs 4 --limit 760 --deadline 30 -- reference --device cuda --epochs 20 --seeds 8-11 > gpurun_out/accb_ref.log 2>&1 &
P1=$!
timeout -k 10 800 python -u scripts/acc_par.py --jobs 3 --limit 760 --deadline 30 -- pt_reference --device cuda --mono-epochs 10 --epochs 20 --seeds 6-8 > gpurun_out/accb_ptref.log 2>&1 &
P2=$!
wait $P1
wait $P2
