#!/bin/bash
# MOSI / MOSEI TextCNN convs: tile search over variants 1 and 4 at batch 128 (MOSI) and 256 (MOSEI), then bench
# A/Bs of the merged tables against the current ones.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out ab_old
T=${1:-r6t}
P=task-specific-pretraining-multimodal_amd
timeout -k 10 400 python -u scripts/tune_textcnn.py --batch 128 --variants 1,4 --out gpurun_out/${T}_text_b128.json > gpurun_out/${T}_text_b128.log 2>&1
timeout -k 10 400 python -u scripts/tune_textcnn.py --batch 256 --variants 1,4 --out gpurun_out/${T}_text_b256.json > gpurun_out/${T}_text_b256.log 2>&1
python - <<PY
import json
a = json.load(open("gpurun_out/${T}_text_b128.json")); b = json.load(open("gpurun_out/${T}_text_b256.json"))
a["entries"] += b["entries"]
json.dump(a, open("gpurun_out/${T}_text_both.json", "w"), indent=1)
PY
python scripts/merge_tuned.py ab_old/tuned_text.json gpurun_out/${T}_text_both.json > gpurun_out/${T}_merge.log
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_text.json -- --mosi --steps 100 > gpurun_out/${T}_ab_mosi.json 2> gpurun_out/${T}_ab_mosi.err
timeout -k 10 500 python -u scripts/ab_lib.py --rounds 4 --a $P/libtspm.so --b $P/libtspm.so --env-b TSPM_TUNED_FILE=$GRAFT_REPO_ROOT/ab_old/tuned_text.json -- --mosi --mosei --steps 100 > gpurun_out/${T}_ab_mosei.json 2> gpurun_out/${T}_ab_mosei.err
