# rocprofv3 kernel stats + PMC passes over the deposit kernels (one pass per run).
# PASSES="SETS" selects passes by name: sq1 sq2 tcc fetch write (default: all of sq1 sq2 fetch write)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-dp}
mkdir -p $O
B="python3 scripts/bench_deposit.py --no-cpu --reps 1 ${DEP_ARGS}"
declare -A SETS
SETS[sq1]="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
SETS[sq2]="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
SETS[tcc]="TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"
SETS[fetch]="FETCH_SIZE"
SETS[write]="WRITE_SIZE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/stats -o run --output-format csv -- $B > $O/stats.log 2>&1 || { tail -20 $O/stats.log; exit 1; }
for name in ${PASSES:-sq1 sq2 fetch write}; do
  timeout -k 10 300 rocprofv3 --pmc ${SETS[$name]} --kernel-include-regex "${KRX:-deposit}" -d $O/pmc_$name -o run --output-format csv -- $B > $O/pmc_$name.log 2>&1 || { tail -20 $O/pmc_$name.log; exit 1; }
done
ls $O
