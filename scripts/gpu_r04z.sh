# knob A/Bs with the experiments build: candidate-column budget (fewer, larger
# collect/select batches) on uniform 1e8; density anchor and seed margin on
# log-normal 1e8.  usage (on the box): TAG=r04z bash scripts/gpu_r04z.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04z}
O=gpurun_out/$TAG
mkdir -p $O
echo "[$TAG] budget"; date
timeout -k 10 900 python3 -u scripts/lib_ab.py --libs "exp,exp@NBKD_CAND_BYTES=51539607552,exp@NBKD_CAND_BYTES=85899345920" --rounds 3 -- --n 1e8 > $O/budget.log 2>&1 \
 && echo "[$TAG] lognormal" && timeout -k 10 900 python3 -u scripts/lib_ab.py --libs "exp,exp@NBKD_KNN_ANCHOR=64,exp@NBKD_KNN_ANCHOR=256,exp@NBKD_KNN_SEED=4.5" --rounds 2 -- --n 1e8 --lognormal > $O/lognormal.log 2>&1
rc=$?
date
tail -4 $O/budget.log; tail -5 $O/lognormal.log
exit $rc
