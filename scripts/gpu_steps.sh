#!/bin/bash
# Run GPU steps in sequence; each under its own time limit.  A test failure (rc 1..123) lets the
# next step run; a timeout / abort / crash (rc >= 124) ends the call so nothing more touches the GPU.
# usage: scripts/gpu_steps.sh LOGPREFIX "SECONDS|command" ["SECONDS|command" ...]
prefix=$1; shift
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  secs=${spec%%|*}; cmd=${spec#*|}
  log=gpurun_out/${prefix}_$i.log
  echo "### $cmd" > "$log"
  timeout -k 10 "$secs" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "### rc=$rc" >> "$log"
  echo "step $i rc=$rc ($cmd)"
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  i=$((i+1))
done
