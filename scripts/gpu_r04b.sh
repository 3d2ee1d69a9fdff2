# round 4: GPU tests, then the A/B of the collect walk-ahead and of the radius
# count's plain-d2 loop (experiments build, interleaved runs, same output SHA)
# usage: TAG=r04b bash scripts/gpu_r04b.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04b}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
echo "[r04b] gpu tests"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r04b] ab" && TAG=$TAG/ab ROUNDS=${ROUNDS:-3} LIBS="exp@NBKD_COLLECT_AHEAD=0,exp@NBKD_COLLECT_AHEAD=1" ARGS="--n 1e8" TMO=900 BALL_LIBS="exp@NBKD_BALL_PLAIN=0,exp@NBKD_BALL_PLAIN=1" bash scripts/gpu_ab.sh
rc=$?
date
tail -5 $O/tests.log
exit $rc
