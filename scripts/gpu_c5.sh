# Config C5 lines: one GPU at 1e8, then an N=2 rehearsal with both ranks on
# the box's one GPU (gloo-staged halo).  usage (on the box): TAG=r01j bash scripts/gpu_c5.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > $O/slab_tests.log 2>&1
rc=$?; tail -3 $O/slab_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --workload c5 --particles ${N1:-1e8} --steps 3 --warmup 1 > $O/c5_n1.json 2> $O/c5_n1.err
rc=$?; tail -3 $O/c5_n1.err; cat $O/c5_n1.json; [ $rc -ne 0 ] && exit $rc
NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --workload c5 --gpus 2 --particles ${N2:-2e7} --steps 3 --warmup 1 > $O/c5_n2.json 2> $O/c5_n2.err
rc=$?; tail -3 $O/c5_n2.err; cat $O/c5_n2.json; exit $rc
