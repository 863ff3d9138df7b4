# One-graph phased DP step: mechanism + DP tests, then bench --phased vs plain A/B.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_phased.py tests/test_gpu_ddp.py "tests/test_gpu_model.py::test_phased_allreduce_step_equals_plain_step" -x -v --timeout 300 --timeout-method thread > gpurun_out/ph_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/ph_plain_$i.json 2> gpurun_out/ph_plain_$i.err
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/ph_one_$i.json 2> gpurun_out/ph_one_$i.err
  TSPM_PHASED=split timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 --phased > gpurun_out/ph_split_$i.json 2> gpurun_out/ph_split_$i.err
done
