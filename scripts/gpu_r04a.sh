# round 4, first call: calibration, GPU tests, the default bench line and the
# N = 2 launcher rehearsal on the one GPU.  usage: TAG=r04a bash scripts/gpu_r04a.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04a}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
TAG=$TAG bash scripts/gpu_calib.sh \
 && echo "[r04a] gpu tests" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r04a] bench" && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err \
 && echo "[r04a] bench n2 launcher" && NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 bench.py --gpus 2 --particles 2e7 --steps 3 --warmup 1 > $O/bench_n2.json 2> $O/bench_n2.err \
 && echo "[r04a] ab walk-ahead" && TAG=$TAG/ab ROUNDS=2 LIBS="exp@NBKD_COLLECT_AHEAD=0,exp@NBKD_COLLECT_AHEAD=1" ARGS="--n 1e8" TMO=600 bash scripts/gpu_ab.sh
rc=$?
date
tail -5 $O/tests.log
cat $O/bench.json $O/bench_n2.json
exit $rc
