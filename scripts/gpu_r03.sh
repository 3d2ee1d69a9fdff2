# Round-3 GPU call: all gpu tests (incl. the full-size slow ones), smoke, the
# default bench line, then an N=2 strong-scaling rehearsal with both ranks on
# the box's one GPU (gloo-staged halo and second round).
# usage (on the box): TAG=r03b bash scripts/gpu_r03.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
echo "[r03] gpu tests"; date
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
 && echo "[r03] smoke" && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
 && echo "[r03] bench" && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err \
 && echo "[r03] n2" && NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/bench_n2.json 2> $O/bench_n2.err
rc=$?
date
tail -5 $O/tests.log
cat $O/bench.json $O/bench_n2.json
exit $rc
