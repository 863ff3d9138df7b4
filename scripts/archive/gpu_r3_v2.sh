# Two LDS-kernel builds (variant 1 register-staged loader waves, variant 2 single-role LDS-DMA — the batch-256 /
# 1024 tables): conv/model/mono tests, then the batch-128, batch-1024 and monomodal lines.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_conv_bwd.py tests/test_gpu_model.py tests/test_gpu_mono.py tests/test_gpu_bnfold.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v2_t.log 2>&1
timeout -k 10 200 python -u bench.py --no-cpu-baseline --pcie-steps 0 --steps 60 > gpurun_out/v2_b128.json 2> gpurun_out/v2_b128.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 1024 --steps 15 --profile-steps 3 > gpurun_out/v2_b1024.json 2> gpurun_out/v2_b1024.err
timeout -k 10 200 python -u bench.py --mono --no-cpu-baseline > gpurun_out/v2_mono.json 2> gpurun_out/v2_mono.err
