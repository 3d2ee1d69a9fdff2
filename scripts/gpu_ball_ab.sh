# ball-count parity tests, then the transposed-count threshold A/B at 1e8
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ballab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ball" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for T in ${TS:-0 9}; do
  NBKD_BALL_T=$T timeout -k 10 300 python -u scripts/ball_ab.py --n ${N:-1e8} $EXTRA >> $O/ab.log 2>&1 || exit $?
done
cat $O/ab.log
