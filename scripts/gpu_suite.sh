# GPU tests, then the bench with SURVEY §8(d)'s secondary runs (--suite)
# usage (on the box): TAG=r01e bash scripts/gpu_suite.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u bench.py --suite --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/suite.json 2> $O/suite.err
rc=$?
tail -5 $O/suite.err
cat $O/suite.json
exit $rc
