set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t2.log 2>&1; rc=$?; tail -3 gpurun_out/t2.log; [ $rc -eq 0 ] || exit $rc
for LEAF in 32 16 64; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --leafsize $LEAF --no-cpu-baseline --cpu-sample 100000 > gpurun_out/b_v2_l$LEAF.json 2> gpurun_out/b_v2_l$LEAF.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/b_v2_l$LEAF.json'));print('v2 leaf',$LEAF,'%.3e'%d['value'],'knn ms',round(d['roofline']['kernel_ms_per_launch'],1),d['breakdown_ms_per_step'],d['traversal_per_query'],d['traversal_per_packet'],d['build_ms'],d['parity_vs_cpu'])"
done
