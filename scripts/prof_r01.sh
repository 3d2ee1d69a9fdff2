# Round-1 measurement: default bench line, rocprofv3 kernel stats, HBM PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
timeout -k 10 900 python3 bench.py > gpurun_out/r01_bench.json 2> gpurun_out/r01_bench.err \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r01_trace -o run --output-format csv -- $B > gpurun_out/r01_trace.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex knn4 -d gpurun_out/r01_fetch -o run --output-format csv -- $B > gpurun_out/r01_fetch.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex knn4 -d gpurun_out/r01_write -o run --output-format csv -- $B > gpurun_out/r01_write.log 2>&1
rc=$?
cat gpurun_out/r01_bench.json
exit $rc
