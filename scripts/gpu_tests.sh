set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/t1.log 2>&1
rc=$?
tail -40 gpurun_out/t1.log
exit $rc
