set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "knn_vs_oracle or squared or seed_retry or kth_distance" > $O/tests.log 2>&1 \
 && timeout -k 10 600 python3 scripts/knn_ks.py --ks 32,64,100,200 > $O/ks.log 2>&1
rc=$?; tail -3 $O/tests.log; cat $O/ks.log; exit $rc
