# Accuracy parity batch: reference-side seeds (scratch and pretrained) and our seeds concurrently.
# usage: bash scripts/gpu_r3_acc_c.sh <scratch ref seeds> <pretrained ref seeds> <our scratch seeds> <tag> [<our pretrained seeds>]
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
TAG=${4:-c}
python scripts/acc_pack.py unpack
timeout -k 10 900 python -u scripts/acc_par.py --jobs 6 --limit 860 --deadline 30 -- reference --device cuda --epochs 20 --seeds $1 > gpurun_out/acc${TAG}_ref.log 2>&1 &
P1=$!
timeout -k 10 900 python -u scripts/acc_par.py --jobs 4 --limit 860 --deadline 30 -- pt_reference --device cuda --mono-epochs 10 --epochs 20 --seeds $2 > gpurun_out/acc${TAG}_ptref.log 2>&1 &
P2=$!
timeout -k 10 900 python -u scripts/acc_par.py --jobs 1 --limit 400 --deadline 600 -- ours --epochs 20 --seeds $3 > gpurun_out/acc${TAG}_ours.log 2>&1 &
P3=$!
if [ -n "$5" ]; then
  timeout -k 10 900 python -u scripts/acc_par.py --jobs 1 --limit 400 --deadline 600 -- pt_ours --mono-epochs 10 --epochs 20 --seeds $5 > gpurun_out/acc${TAG}_ptours.log 2>&1 &
  P4=$!
fi
wait $P1
wait $P2
wait $P3
if [ -n "$5" ]; then wait $P4; fi
