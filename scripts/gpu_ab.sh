# A/B of library builds on the box: TAG=x LIBS=base,v1 ROUNDS=3 ARGS="--n 1e8" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 ${TMO:-900} python3 -u scripts/lib_ab.py --libs ${LIBS:-prod} --rounds ${ROUNDS:-3} -- ${ARGS:---n 1e8} > $O/ab.log 2>&1
rc=$?; tail -12 $O/ab.log; exit $rc
