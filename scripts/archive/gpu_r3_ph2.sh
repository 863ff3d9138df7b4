# Host-polled step flags for the one-graph phased DP step; RS = 3 default: full GPU suite, then bench lines
# (plain x2, phased forced 1-rank RCCL, phased without exchange, split schedule).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_phased.py tests/test_gpu_ddp.py -x -q --timeout 250 --timeout-method thread > gpurun_out/p2_new.log 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/p2_t.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 100 --kernel-table gpurun_out/p2_plain_kt$i.json > gpurun_out/p2_plain_$i.json 2> gpurun_out/p2_plain_$i.err
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/p2_ph_one.json 2> gpurun_out/p2_ph_one.err
TSPM_PHASED_FORCE=0 timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/p2_ph_noar.json 2> gpurun_out/p2_ph_noar.err
TSPM_PHASED=split timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/p2_ph_split.json 2> gpurun_out/p2_ph_split.err
