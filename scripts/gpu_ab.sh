# A/B of library builds on the box (lib_ab.py over knn_time.py):
#   TAG=x LIBS=prod,v1 [ROUNDS=3] [ARGS="--n 1e8"] [BALL_LIBS=prod,v2] bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 ${TMO:-900} python3 -u scripts/lib_ab.py --libs ${LIBS:-prod} --rounds ${ROUNDS:-3} -- ${ARGS:---n 1e8} > $O/ab.log 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -n "$BALL_LIBS" ]; then
  timeout -k 10 600 python3 -u scripts/lib_ab.py --libs $BALL_LIBS --rounds ${ROUNDS:-3} -- --n 1e8 --ball 0.01 > $O/ball.log 2>&1
  rc=$?
fi
tail -8 $O/ab.log; [ -f $O/ball.log ] && tail -4 $O/ball.log; exit $rc
