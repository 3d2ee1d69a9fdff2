# fused outside-box listing + per-piece select reads: GPU tests, then A/B
# against the packed-points build (lib/exp/packed)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04i}
O=gpurun_out/$TAG
mkdir -p $O
echo "[r04i] gpu tests"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r04i] ab" && TAG=$TAG/ab ROUNDS=3 LIBS="packed,prod" ARGS="--n 1e8" TMO=900 bash scripts/gpu_ab.sh
rc=$?
date
tail -5 $O/tests.log
exit $rc
