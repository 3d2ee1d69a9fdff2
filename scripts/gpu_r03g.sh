set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && timeout -k 10 600 python3 scripts/knn_ks.py --ks 32,100 > $O/ks.log 2>&1 \
 && timeout -k 10 600 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; tail -3 $O/tests.log; cat $O/ks.log; cut -c1-600 $O/bench.json; exit $rc
