set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --n 1e7 --steps 3 --warmup 1 --cpu-sample 200000 > gpurun_out/bench_1e7.json 2> gpurun_out/bench_1e7.err
rc=$?; tail -5 gpurun_out/bench_1e7.err; cat gpurun_out/bench_1e7.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_1e8.json 2> gpurun_out/bench_1e8.err
rc=$?; tail -5 gpurun_out/bench_1e8.err; cat gpurun_out/bench_1e8.json; exit $rc
