# Accuracy parity batch: a probe of MIOpen kernel selection speed for the ATen reference (1 epoch each),
# then scratch reference seeds and pretrained reference seeds concurrently (no refills: one wave of runs).
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
timeout -k 10 150 python -u scripts/accuracy_parity.py reference --device cuda --epochs 1 --seeds 900 > gpurun_out/accb_probe_fast.log 2>&1
MIOPEN_FIND_MODE=NORMAL ACC_CUDNN_BENCHMARK=1 timeout -k 10 200 python -u scripts/accuracy_parity.py reference --device cuda --epochs 2 --seeds 901 > gpurun_out/accb_probe_bench.log 2>&1
timeout -k 10 1000 python -u scripts/acc_par.py --jobs 4 --limit 950 --deadline 30 -- reference --device cuda --epochs 20 --seeds 8-11 > gpurun_out/accb_ref.log 2>&1 &
P1=$!
timeout -k 10 1000 python -u scripts/acc_par.py --jobs 3 --limit 950 --deadline 30 -- pt_reference --device cuda --mono-epochs 10 --epochs 20 --seeds 6-8 > gpurun_out/accb_ptref.log 2>&1 &
P2=$!
wait $P1
wait $P2
