set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity $BENCH_ARGS > gpurun_out/one.json 2> gpurun_out/one.err || { tail gpurun_out/one.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/one.json'));print('%.3e'%d['value'],'knn ms',round(d['roofline']['kernel_ms_per_launch'],1),d['breakdown_ms_per_step'],d['traversal_per_query'],d['traversal_per_packet'],d['build_ms'])"
