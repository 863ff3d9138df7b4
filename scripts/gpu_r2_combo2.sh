set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/encoder_timing.py > gpurun_out/encoder_timing_r2.log 2>&1
timeout -k 10 300 python3 bench.py --mosi > gpurun_out/r2_v6_mosi_bench.json 2> gpurun_out/r2_v6_mosi_bench.err
bash scripts/gpu_r2_lines.sh
