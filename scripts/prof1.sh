set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- $B > gpurun_out/prof_trace.log 2>&1 || { tail -20 gpurun_out/prof_trace.log; exit 1; }
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "knn_packet|leaf_key2|rs_scatter" -d gpurun_out/prof_pmc$i -o run --output-format csv -- $B > gpurun_out/prof_pmc$i.log 2>&1 || { tail -20 gpurun_out/prof_pmc$i.log; exit 1; }
done
ls -R gpurun_out | head -40
