# Pretrained-encoder accuracy parity (AVMNIST real data): quick check, then 8 paired seeds per side;
# GPU tests touched since the last full run (harness NaN test, MOSI).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pt.log 2>&1
timeout -k 10 120 python -u scripts/accuracy_parity.py pt_ours --mono-epochs 1 --epochs 1 --seeds 99 > gpurun_out/pt_quick.log 2>&1
timeout -k 10 400 python -u scripts/accuracy_parity.py pt_ours --mono-epochs 10 --epochs 15 --seeds 0,1,2,3,4,5,6,7 > gpurun_out/pt_ours.log 2>&1
timeout -k 10 720 python -u scripts/accuracy_parity.py pt_reference --device cuda --mono-epochs 10 --epochs 15 --seeds 0,1,2,3,4,5,6,7 > gpurun_out/pt_ref.log 2>&1
