# GPU tests, then uniform 1e8 kNN with the LDS top levels of the bucketing descent off / on
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-keyab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for A in 0 1; do
  NBKD_KEY_LDS=$A timeout -k 10 300 python -u scripts/variants.py --n ${N:-1e8} --variants 0 > $O/ab$A.log 2>&1 || { tail -5 $O/ab$A.log; exit 1; }
  echo "KEY_LDS=$A"; tail -1 $O/ab$A.log | cut -c1-420
done
