# full gpu tests + smoke + the profiling script of the same build
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && bash scripts/prof_r03.sh
rc=$?; tail -3 $O/tests.log; exit $rc
