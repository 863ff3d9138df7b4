# encoder capture order A/B + encoder chain timing, MOSI/MOSEI parity after the LSTM change, then the current
# bench line of every workload.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_mosi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_mosi_lstm.log 2>&1
bash scripts/gpu_r2_order.sh
bash scripts/gpu_r2_lines.sh
timeout -k 10 300 python3 bench.py --mosi > gpurun_out/r2_v6_mosi_bench.json 2> gpurun_out/r2_v6_mosi_bench.err
