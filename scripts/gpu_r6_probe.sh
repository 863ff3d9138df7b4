#!/bin/bash
# Round 6: the headline line on the current tree, the per-kernel dump of one replayed two-stream step, batch 1024.
set -e
mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 300 python -u bench.py --kernel-table gpurun_out/${T}_kernel_table.json > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('frac'), (r.get('r34_3x3') or {}).get('frac'), r.get('kernel_ms_per_step_by_family'))"
timeout -k 10 200 python -u scripts/overlap_probe.py --dump gpurun_out/${T}_step_dump.txt > gpurun_out/${T}_overlap.json 2> gpurun_out/${T}_overlap.err
timeout -k 10 300 python -u bench.py --no-cpu-baseline --pcie-steps 0 --batch-per-rank 1024 --steps 20 > gpurun_out/${T}_bench_b1024.json 2> gpurun_out/${T}_b1024.err
python -c "import json; d=json.load(open('gpurun_out/${T}_bench_b1024.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r.get('frac'))"
