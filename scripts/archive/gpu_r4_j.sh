#!/bin/bash
# Round-4: DP tests (phase Adam behind each exchange), the stem kernels (tests, stamps, batch 1024), layer4's span in the benched graph, the step with 4 vs 8 waves per small-GEMM tile (two libraries,
# alternating), and the phased DP step at N=1 against the plain step.  usage: bash scripts/gpu_r4_j.sh TAG
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=$1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ddp.py tests/test_gpu_phased.py "tests/test_gpu_model.py::test_phased_allreduce_step_equals_plain_step" -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -k "stem" -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_stem_tests.log 2>&1
timeout -k 10 200 python3 -u scripts/stem_bench.py --stamps > gpurun_out/${T}_stem_bench.json 2> gpurun_out/${T}_stem_bench.err
timeout -k 10 200 python3 -u scripts/stem_bench.py --batch 1024 > gpurun_out/${T}_stem_bench_b1024.json 2> gpurun_out/${T}_stem_bench_b1024.err
timeout -k 10 200 python3 -u scripts/layer_span.py --replays 20 > gpurun_out/${T}_layer_span.json 2> gpurun_out/${T}_layer_span.err
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_wkA$i.json 2> gpurun_out/${T}_wkA$i.err
  TSPM_LIB=$GRAFT_REPO_ROOT/task-specific-pretraining-multimodal_amd/libtspm_wk8.so timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 > gpurun_out/${T}_wkB$i.json 2> gpurun_out/${T}_wkB$i.err
done
timeout -k 10 200 python3 -u bench.py --phased --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_phased.json 2> gpurun_out/${T}_phased.err
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --pcie-steps 0 --profile-steps 0 --steps 100 > gpurun_out/${T}_plain.json 2> gpurun_out/${T}_plain.err
