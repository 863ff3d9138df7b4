#!/bin/bash
# Round 5 (pre-registered pretrained extension): accuracy parity on the reference's protocol (scripts/accuracy_protocol.py): one batch of paired seeds,
# reference side (ATen on the MI355X) and ours concurrently on one GPU (at most 8 + 5 + 1 + 1 = 15 GPU processes: the
# box allows 16).  usage:
#   bash scripts/gpu_r5_acc.sh <ref seeds|-> <ours seeds|-> <pt ref seeds|-> <pt ours seeds|-> <tag> [limit s]
set -e
export MIOPEN_FIND_MODE=FAST
mkdir -p gpurun_out
TAG=$5; LIM=${6:-1000}
python scripts/acc_pack.py unpack
PIDS=""
run() {  # cmd seeds jobs log
  timeout -k 10 $((LIM + 60)) python -u scripts/acc_par.py --script accuracy_protocol.py --jobs $3 --limit $LIM --deadline $((LIM / 2)) -- $1 --seeds $2 > gpurun_out/accproto_${TAG}_$4.log 2>&1 &
  PIDS="$PIDS $!"
}
# concurrent processes per side (env REFJ / PTRJ / OURJ / PTOJ; their sum must stay <= 15)
[ "$1" != "-" ] && run "reference --device cuda" $1 ${REFJ:-8} ref
[ "$3" != "-" ] && run "pt_reference --device cuda" $3 ${PTRJ:-5} ptref
[ "$2" != "-" ] && run ours $2 ${OURJ:-1} ours
[ "$4" != "-" ] && run pt_ours $4 ${PTOJ:-1} ptours
for p in $PIDS; do wait $p; done
