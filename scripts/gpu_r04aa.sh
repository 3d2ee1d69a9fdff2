# next-leaf L2 prefetch in the collect kernel (lib/exp/pf): parity tests, then
# A/B against the head on uniform and log-normal 1e8, with the density anchor
# at the leaf (exp@NBKD_KNN_ANCHOR=64) beside it.  usage: TAG=r04aa bash scripts/gpu_r04aa.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04aa}
O=gpurun_out/$TAG
mkdir -p $O
NBKD_LIB=$PWD/nbodyhpc_amd/lib/exp/pf/libnbkd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests_pf.log 2>&1 \
 && echo "[$TAG] uniform" && timeout -k 10 900 python3 -u scripts/lib_ab.py --libs "prod,pf,exp,exp@NBKD_KNN_ANCHOR=64" --rounds 3 -- --n 1e8 > $O/uniform.log 2>&1 \
 && echo "[$TAG] lognormal" && timeout -k 10 600 python3 -u scripts/lib_ab.py --libs "prod,pf,exp@NBKD_KNN_ANCHOR=64" --rounds 2 -- --n 1e8 --lognormal > $O/lognormal.log 2>&1
rc=$?
tail -3 $O/tests_pf.log; tail -5 $O/uniform.log; tail -4 $O/lognormal.log
exit $rc
