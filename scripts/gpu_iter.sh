# quick iteration on the box: gpu tests then a variant sweep
# usage: VARIANTS="0,1" N=1e8 bash scripts/gpu_iter.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/iter_tests.log 2>&1
rc=$?
tail -15 gpurun_out/iter_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u scripts/variants.py --n ${N:-1e8} --variants ${VARIANTS:-0} --stats > gpurun_out/iter_var.log 2>&1
rc=$?
cat gpurun_out/iter_var.log | tail -20
exit $rc
