# N=2 rehearsal on a one-GPU box of bench --input FILE --redistribute (both ranks
# on device 0, gloo transport), then the C5 line at N=1 (1e8)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-redist}
mkdir -p $O
python -c "
from nbodyhpc_amd import io, synth
io.write_positions('/tmp/p2e7.f32', synth.uniform(20_000_000, 5, 1.0))
" || exit 1
NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 2 --steps 2 --warmup 1 --input /tmp/p2e7.f32 --redistribute > $O/n2.json 2> $O/n2.err
rc=$?; tail -3 $O/n2.err; cat $O/n2.json; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 -u bench.py --workload c5 --steps 3 --warmup 1 > $O/c5_n1.json 2> $O/c5_n1.err
rc=$?; tail -2 $O/c5_n1.err; cat $O/c5_n1.json; exit $rc
