# ball-count parity tests, then radius-count A/B runs at 1e8 (one process per setting)
# usage (on the box): TAG=x ENVS="NBKD_BALL_GROUPS=0 NBKD_BALL_GROUPS=1" LEAVES="32 64" bash scripts/gpu_ball_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ballab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ball" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for L in ${LEAVES:-32}; do
  for E in ${ENVS:-NONE=0}; do
    env $E timeout -k 10 300 python -u scripts/ball_ab.py --n ${N:-1e8} --leaf $L $EXTRA >> $O/ab.log 2>&1 || exit $?
  done
done
cat $O/ab.log
