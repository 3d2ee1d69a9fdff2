# Profiles of one build: the bench line with the suite, the rocprofv3 kernel
# trace + stats of the plain bench, and the HBM PMC passes (FETCH_SIZE and
# WRITE_SIZE in separate runs) of the collect kernel; lib.sha256 ties them to
# the library (bench.py reports roofline.traffic only for the same build).
# usage (on the box): TAG=r03d bash scripts/prof_r03.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
echo "[prof] suite"; date
timeout -k 10 900 python3 bench.py --suite > $O/suite.json 2> $O/suite.err \
 && echo "[prof] trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 \
 && echo "[prof] fetch" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_collect -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1 \
 && echo "[prof] write" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn_collect -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1 \
 && echo "[prof] ball fetch" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ball_packet -d $O/ball_fetch -o run --output-format csv -- python3 scripts/ball_run.py > $O/ball_fetch.log 2>&1 \
 && echo "[prof] ball write" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex ball_packet -d $O/ball_write -o run --output-format csv -- python3 scripts/ball_run.py > $O/ball_write.log 2>&1 \
 && cp $O/suite.json $O/bench.json
rc=$?
date
tail -c 3000 $O/suite.json
exit $rc
