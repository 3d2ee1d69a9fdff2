# ball-count XCD A/B (old library variant vs current) + an N=2 gadget-slab bench rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-misc}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ball" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for E in "NBKD_LIB=nbodyhpc_amd/lib/exp/ballold/libnbkd.so" "NONE=1" "NBKD_LIB=nbodyhpc_amd/lib/exp/ballold/libnbkd.so" "NONE=2"; do
  env $E timeout -k 10 300 python -u scripts/ball_ab.py --n 1e8 --leaf 64 >> $O/ball_ab.log 2>&1 || { tail -5 $O/ball_ab.log; exit 1; }
done
cat $O/ball_ab.log
timeout -k 10 120 python -c "
import numpy as np, sys
sys.path.insert(0, '.')
from nbodyhpc_amd import io, synth
io.write_gadget('/tmp/snap', synth.uniform(4_000_000, box=1.0), 1.0, fmt=2, num_files=3)
" && export NBKD_BENCH_SAME_DEVICE=1 && timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 --input /tmp/snap --input-format gadget > $O/gadget_n2.json 2> $O/gadget_n2.err || { tail -20 $O/gadget_n2.err; exit 1; }
tail -1 $O/gadget_n2.json | cut -c1-600
