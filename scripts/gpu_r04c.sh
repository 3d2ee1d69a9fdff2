# round 4 combined call: GPU tests, the default bench line, the N = 2 launcher
# rehearsal on the one GPU, then the A/B of the collect walk-ahead and of the
# radius count's plain-d2 loop.  usage: TAG=r04c bash scripts/gpu_r04c.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04c}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
echo "[r04c] gpu tests"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r04c] bench" && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err \
 && echo "[r04c] bench n2 launcher" && NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --particles 2e7 --steps 3 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err \
 && echo "[r04c] ab" && TAG=$TAG/ab ROUNDS=${ROUNDS:-2} LIBS="exp@NBKD_COLLECT_AHEAD=0,exp@NBKD_COLLECT_AHEAD=1" ARGS="--n 1e8" TMO=900 BALL_LIBS="exp@NBKD_BALL_PLAIN=0,exp@NBKD_BALL_PLAIN=1" bash scripts/gpu_ab.sh
rc=$?
date
tail -5 $O/tests.log
cat $O/bench.json $O/bench_n2.json 2>/dev/null | cut -c1-600
exit $rc
