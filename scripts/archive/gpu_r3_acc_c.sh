# Accuracy parity batch: reference-side seeds (scratch and pretrained) and our seeds concurrently.
# usage: bash scripts/gpu_r3_acc_c.sh <scratch ref seeds> <pretrained ref seeds> <our scratch seeds> <tag> [<our pretrained seeds>]
# (a seed list of '-' skips that side)
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
TAG=${4:-c}
python scripts/acc_pack.py unpack
PIDS=""
if [ "$1" != "-" ]; then
  timeout -k 10 900 python -u scripts/acc_par.py --jobs 12 --limit 860 --deadline 30 -- reference --device cuda --epochs 20 --seeds $1 > gpurun_out/acc${TAG}_ref.log 2>&1 &
  PIDS="$PIDS $!"
fi
if [ "$2" != "-" ]; then
  timeout -k 10 900 python -u scripts/acc_par.py --jobs 12 --limit 860 --deadline 30 -- pt_reference --device cuda --mono-epochs 10 --epochs 20 --seeds $2 > gpurun_out/acc${TAG}_ptref.log 2>&1 &
  PIDS="$PIDS $!"
fi
if [ "$3" != "-" ]; then
  timeout -k 10 900 python -u scripts/acc_par.py --jobs 1 --limit 400 --deadline 600 -- ours --epochs 20 --seeds $3 > gpurun_out/acc${TAG}_ours.log 2>&1 &
  PIDS="$PIDS $!"
fi
if [ -n "$5" ]; then
  timeout -k 10 900 python -u scripts/acc_par.py --jobs 1 --limit 400 --deadline 600 -- pt_ours --mono-epochs 10 --epochs 20 --seeds $5 > gpurun_out/acc${TAG}_ptours.log 2>&1 &
  PIDS="$PIDS $!"
fi
for p in $PIDS; do wait $p; done
