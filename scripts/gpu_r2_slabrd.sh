# Split-K slab read with each slab's loads issued together: stamps of the small forward launches, the headline
# bench (2 runs), then the full GPU suite.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/stamp_conv.py --only "fwd:4,4,128,128,3,1;fwd:2,2,256,256,3,1;dgrad:2,2,256,256,3,1" > gpurun_out/stamps_r2_slabrd.log 2>&1
for i in 1 2; do
  timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --pcie-steps 0 > gpurun_out/slabrd_$i.json 2> gpurun_out/slabrd_$i.err
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_slabrd.log 2>&1
