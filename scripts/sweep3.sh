set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/t4.log 2>&1; rc=$?; tail -3 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
for V in 0 1 3 4; do
  NBKD_KNN_VARIANT=$V timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/b4_var$V.json 2> gpurun_out/b4_var$V.err || { tail gpurun_out/b4_var$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b4_var$V.json'));print('variant',$V,'%.3e'%d['value'],'knn ms',round(d['roofline']['kernel_ms_per_launch'],1),d['breakdown_ms_per_step'],d['traversal_per_query'],d['traversal_per_packet'])"
done
