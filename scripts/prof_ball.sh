# PMC passes over the radius-count kernel (1e8, r=0.01, one pass), each in its own run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pb}
mkdir -p $O
B="python3 scripts/ball_ab.py --n 1e8 --steps 1"
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "ball_count2" -d $O/pmc$i -o run --output-format csv -- $B > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1
python3 scripts/pmc_summary.py $O
