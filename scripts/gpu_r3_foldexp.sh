# Diagnostic: which part of the conv2 BN-input hook costs (TSPM_FOLD_EXP builds: 1 = no x_out store,
# 2 = no transform either, 3 = prologue only) — forward per-launch tables only.
set -e
mkdir -p gpurun_out
for n in fx1 fx2 fx3; do
  TSPM_LIB=$PWD/task-specific-pretraining-multimodal_amd/libtspm_$n.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 30 --kernel-table gpurun_out/fe_${n}_kt.json > gpurun_out/fe_$n.json 2> gpurun_out/fe_$n.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 30 --kernel-table gpurun_out/fe_fold_kt.json > gpurun_out/fe_fold.json 2> gpurun_out/fe_fold.err
TSPM_BN_FOLD=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 30 --kernel-table gpurun_out/fe_nofold_kt.json > gpurun_out/fe_nofold.json 2> gpurun_out/fe_nofold.err
for d in "" nowait inline; do
  TSPM_PHASED_DIAG=$d TSPM_PHASED_FORCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/fe_ph_$d.json 2> gpurun_out/fe_ph_$d.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/fe_plain.json 2> gpurun_out/fe_plain.err
