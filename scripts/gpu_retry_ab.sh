# GPU tests, then log-normal kNN with the adaptive retry off / on (separate processes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-retry}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for A in 0 1; do
  NBKD_RETRY_ADAPT=$A timeout -k 10 300 python -u scripts/variants.py --n ${N:-1e8} --dist lognormal --variants 0 --stats > $O/ab$A.log 2>&1 || { tail -5 $O/ab$A.log; exit 1; }
  echo "ADAPT=$A"; tail -4 $O/ab$A.log
done
