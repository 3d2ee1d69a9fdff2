# Round 4: C5 at 1e8 on the one GPU, then the N > 1 bench paths with every
# rank on the box's one GPU (gloo-staged halo; bench.py starts its own ranks):
# headline strong scaling at N = 2 and 4 (1e8 total), C5 at N = 2, weak
# scaling, --input --redistribute and a Gadget-2 snapshot streamed per slab.
# usage (on the box): TAG=r04r bash scripts/gpu_r04_rehearse.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04r}
mkdir -p $O
B="timeout -k 10 600 python3 -u bench.py"
echo "[rehearse] suite"; date
timeout -k 10 900 python3 -u bench.py --suite > $O/suite.json 2> $O/suite.err \
 && echo "[rehearse] c5 n1" && $B --workload c5 --steps 3 --warmup 1 > $O/c5_n1.json 2> $O/c5_n1.err \
 && echo "[rehearse] n2 strong" && NBKD_BENCH_SAME_DEVICE=1 $B --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/n2_strong.json 2> $O/n2_strong.err \
 && echo "[rehearse] n4 strong" && NBKD_BENCH_SAME_DEVICE=1 $B --gpus 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/n4_strong.json 2> $O/n4_strong.err \
 && echo "[rehearse] c5 n2" && NBKD_BENCH_SAME_DEVICE=1 $B --workload c5 --gpus 2 --particles 2e7 --steps 3 --warmup 1 > $O/c5_n2.json 2> $O/c5_n2.err \
 && python3 -c "
from nbodyhpc_amd import io, synth
pts = synth.uniform(20_000_000, 5, 1.0)
io.write_positions('/tmp/p2e7.f32', pts)
io.write_gadget('/tmp/snap2e7', pts[:4_000_000], box=1.0, num_files=2)
" \
 && echo "[rehearse] redistribute" && NBKD_BENCH_SAME_DEVICE=1 $B --gpus 2 --steps 2 --warmup 1 --input /tmp/p2e7.f32 --redistribute > $O/redist.json 2> $O/redist.err \
 && echo "[rehearse] weak" && NBKD_BENCH_SAME_DEVICE=1 $B --gpus 2 --steps 2 --warmup 1 --scaling weak --particles 2e7 > $O/weak.json 2> $O/weak.err \
 && echo "[rehearse] gadget" && NBKD_BENCH_SAME_DEVICE=1 $B --gpus 2 --steps 2 --warmup 1 --input /tmp/snap2e7 --input-format gadget > $O/gadget.json 2> $O/gadget.err
rc=$?
rm -f /tmp/p2e7.f32 /tmp/snap2e7.*
date
for f in suite c5_n1 n2_strong n4_strong c5_n2 redist weak gadget; do echo "== $f"; grep '^{' $O/$f.json 2>/dev/null | cut -c1-300; done
# (appended) seed-margin A/B at the round-4 head (experiments build knob)
if [ $rc -eq 0 ] && [ -n "$SEED_AB" ]; then
  timeout -k 10 900 python3 -u scripts/lib_ab.py --libs "exp@NBKD_KNN_SEED=3.0,exp@NBKD_KNN_SEED=3.5,exp@NBKD_KNN_SEED=4.0" --rounds 2 -- --n 1e8 > $O/seed_ab.log 2>&1
  rc=$?
  tail -4 $O/seed_ab.log
fi
exit $rc
