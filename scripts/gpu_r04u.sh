# round-4 head with the packet-level plain walk: the GPU test suite, then the
# profiles of this build (scripts/prof_r04.sh).  usage: TAG=r04u bash scripts/gpu_r04u.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04u}
O=gpurun_out/$TAG
mkdir -p $O
echo "[$TAG] gpu tests"; date
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[$TAG] profiles" && TAG=$TAG bash scripts/prof_r04.sh
rc=$?
date
tail -3 $O/tests.log
exit $rc
