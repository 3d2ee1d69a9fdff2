# The N > 1 bench paths other than the headline, rehearsed with both ranks on
# the box's one GPU (gloo-staged halo): --input FILE --redistribute, weak
# scaling, and a Gadget-2 snapshot streamed per slab.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-paths}
mkdir -p $O
export NBKD_BENCH_SAME_DEVICE=1
python -c "
from nbodyhpc_amd import io, synth
pts = synth.uniform(20_000_000, 5, 1.0)
io.write_positions('/tmp/p2e7.f32', pts)
io.write_gadget('/tmp/snap2e7', pts[:4_000_000], box=1.0)
" || exit 1
R="timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
$R --master-port 29514 bench.py --gpus 2 --steps 2 --warmup 1 --input /tmp/p2e7.f32 --redistribute > $O/redist.json 2> $O/redist.err \
 && $R --master-port 29515 bench.py --gpus 2 --steps 2 --warmup 1 --scaling weak --particles 2e7 > $O/weak.json 2> $O/weak.err \
 && $R --master-port 29516 bench.py --gpus 2 --steps 2 --warmup 1 --input /tmp/snap2e7 --input-format gadget > $O/gadget.json 2> $O/gadget.err
rc=$?
for f in redist weak gadget; do echo "== $f"; tail -2 $O/$f.err; grep '^{' $O/$f.json | cut -c1-400; done
exit $rc
