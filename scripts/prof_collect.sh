# PMC passes over the collect/select kernels (one bench step), each in its own run
#   TAG=x [KRX=regex] [PASSES="sq1 sq2 sq3 tcc fetch write"] bash scripts/prof_collect.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pc}
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-parity ${BENCH_ARGS}"
declare -A P
P[sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P[sq2]="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P[sq3]="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_FLAT SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_SENDMSG"
P[tcc]="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
P[fetch]="FETCH_SIZE"
P[write]="WRITE_SIZE"
for name in ${PASSES:-sq1 sq2 sq3 tcc fetch write}; do
  timeout -k 10 300 rocprofv3 --pmc ${P[$name]} --kernel-include-regex "${KRX:-knn_collect|knn_select}" -d $O/pmc_$name -o run --output-format csv -- $B > $O/pmc_$name.log 2>&1 || { tail -20 $O/pmc_$name.log; exit 1; }
done
ls $O
