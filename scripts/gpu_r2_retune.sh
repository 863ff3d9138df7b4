# Re-tune the batch-128 forward convs after the slab-read change, then A/B the merged table vs the current one.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/tune_convs.py --batch 128 --only-kind fwd --no-bwd --out gpurun_out/fwd_r2.json > gpurun_out/fwd_r2.log 2>&1
python scripts/merge_tuned.py gpurun_out/tab_old.json > gpurun_out/merge.log
python scripts/merge_tuned.py gpurun_out/tab_new.json gpurun_out/fwd_r2.json >> gpurun_out/merge.log
for i in 1 2; do
  for t in old new; do
    TSPM_TUNED_FILE=gpurun_out/tab_$t.json timeout -k 10 240 python -u bench.py --steps 100 --warmup 10 --no-cpu-baseline --pcie-steps 0 --profile-steps 0 > gpurun_out/tun_${t}_$i.json 2> gpurun_out/tun_${t}_$i.err
  done
done
