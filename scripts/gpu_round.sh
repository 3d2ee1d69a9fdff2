# One GPU call: gpu tests, smoke, default bench line, rocprofv3 kernel stats and
# the HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) of the same command.
# usage (on the box): TAG=r01 bash scripts/gpu_round.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
echo "[round] gpu tests"; date
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[round] smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && echo "[round] bench" && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err \
 && echo "[round] trace" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B > $O/trace.log 2>&1 \
 && echo "[round] fetch" && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn_collect -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1 \
 && echo "[round] write" && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn_collect -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1
rc=$?
date
tail -5 $O/tests.log
cat $O/bench.json
exit $rc
