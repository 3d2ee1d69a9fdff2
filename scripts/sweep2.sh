set -o pipefail
cd $GRAFT_REPO_ROOT
for V in 0 1 2 3 4; do
  NBKD_KNN_VARIANT=$V timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/b_var$V.json 2> gpurun_out/b_var$V.err || { tail gpurun_out/b_var$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_var$V.json'));print('variant',$V,'%.3e'%d['value'],'knn ms',round(d['roofline']['kernel_ms_per_launch'],1),d['traversal_per_query'],d['traversal_per_packet'])"
done
