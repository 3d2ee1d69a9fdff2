# Profiles of one build (round 4): the bench line with the suite, the rocprofv3
# kernel trace + stats of the plain bench, HBM PMC passes (FETCH_SIZE, WRITE_SIZE:
# separate runs) of the collect / select kernels and of the C3 radius count, and
# SQ / TCC breakdowns of both; lib.sha256 ties them to the library (bench.py
# reports roofline.traffic only for the same build).
# usage (on the box): TAG=r04b bash scripts/prof_r04.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
BR="python3 scripts/ball_run.py"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
pmc() { # name counters regex command...
  local name=$1 ctr=$2 rx=$3; shift 3
  echo "[prof] $name"
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" -d $O/$name -o run --output-format csv -- "$@" > $O/$name.log 2>&1
}
echo "[prof] suite"; date
timeout -k 10 900 python3 bench.py --suite > $O/suite.json 2> $O/suite.err \
 && echo "[prof] trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 \
 && pmc fetch FETCH_SIZE "knn_collect|knn_select" $B \
 && pmc write WRITE_SIZE "knn_collect|knn_select" $B \
 && pmc ball_fetch FETCH_SIZE ball_packet $BR \
 && pmc ball_write WRITE_SIZE ball_packet $BR \
 && pmc pmc_sq1 "$SQ1" "knn_collect|knn_select" $B \
 && pmc pmc_sq2 "$SQ2" "knn_collect|knn_select" $B \
 && pmc pmc_tcc "$TCC" "knn_collect|knn_select" $B \
 && pmc ball_sq1 "$SQ1" ball_packet $BR \
 && pmc ball_sq2 "$SQ2" ball_packet $BR \
 && cp $O/suite.json $O/bench.json
rc=$?
date
tail -c 3000 $O/suite.json
exit $rc
