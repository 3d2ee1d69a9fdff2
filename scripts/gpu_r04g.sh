# packed points (x, y, z, id) + id-carrying candidates: GPU tests, then A/B
# against the previous production build (lib/exp/base) for kNN and the C3 count
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04g}
O=gpurun_out/$TAG
mkdir -p $O
echo "[r04g] gpu tests"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r04g] ab" && TAG=$TAG/ab ROUNDS=3 LIBS="base,prod" ARGS="--n 1e8" TMO=900 BALL_LIBS="base,prod" bash scripts/gpu_ab.sh
rc=$?
date
tail -5 $O/tests.log
exit $rc
