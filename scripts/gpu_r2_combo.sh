# encoder capture order A/B + encoder chain timing, then the current bench line of every workload.
set -e
bash scripts/gpu_r2_order.sh
bash scripts/gpu_r2_lines.sh
