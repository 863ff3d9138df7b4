cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ONLY="dgrad:2,2,256,256,3,1;fwd:8,24,64,64,3,1;wgrad:8,24,64,64,3,1;fwd:1,1,512,512,3,1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc1 -o run -- python3 $R/scripts/conv_bench.py --only "$ONLY" --reps 5 --iters 2 > $R/gpurun_out/pmc1.log 2>&1
echo rc=$?
