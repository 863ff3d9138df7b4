# MOSEI UTT-Fusion widening: GPU parity (MOSI + MOSEI + the BatchNorm1d kernels' MMIMDb users), bench lines,
# then 8 more paired accuracy-parity seeds (AVMNIST, real data).
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_mosi.py tests/test_gpu_mmimdb.py tests/test_abi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_mosei.log 2>&1
timeout -k 10 240 python -u bench.py --mosi --mosei --steps 50 --warmup 10 > gpurun_out/r2_v5_mosei_bench.json 2> gpurun_out/r2_v5_mosei_bench.err
timeout -k 10 240 python -u bench.py --mosi --steps 50 --warmup 10 > gpurun_out/r2_v5_mosi_bench.json 2> gpurun_out/r2_v5_mosi_bench.err
timeout -k 10 400 python -u scripts/accuracy_parity.py ours --epochs 20 --seeds 8,9,10,11,12,13,14,15 > gpurun_out/acc_ours2.log 2>&1
timeout -k 10 650 python -u scripts/accuracy_parity.py reference --device cuda --epochs 20 --seeds 8,9,10,11,12,13,14,15 > gpurun_out/acc_refgpu2.log 2>&1
