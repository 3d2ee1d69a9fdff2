# segmented slot assignment in the collect kernel's pair loop (lib/exp/seg) and the
# two-level node blocks of the packet walk (lib/exp/wide): kNN parity tests against the
# combined build, then the A/B against the round-4 head (lib/exp/base), kNN and radius count.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04s}
O=gpurun_out/$TAG
mkdir -p $O
V=${VARIANT:-segwide}
echo "[$TAG] parity tests with lib/exp/$V"; date
NBKD_LIB=$PWD/nbodyhpc_amd/lib/exp/$V/libnbkd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests_$V.log 2>&1 \
 && echo "[$TAG] ab" && TAG=$TAG/ab ROUNDS=${ROUNDS:-3} LIBS="${LIBS:-base,seg,wide,$V}" BALL_LIBS="${BALL_LIBS:-base,wide}" ARGS="--n 1e8" TMO=1000 bash scripts/gpu_ab.sh
rc=$?
date
tail -3 $O/tests_$V.log
exit $rc
