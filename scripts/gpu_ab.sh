# GPU tests (optional) + short bench lines per setting.
# usage (on the box): TAG=r02d TESTS=1 LEAVES="32 64" ENVS="NBKD_GROUPS=0 NBKD_GROUPS=1" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-ab}
mkdir -p $O
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for R in $(seq 1 ${REPEAT:-1}); do
for L in ${LEAVES:-32}; do
  for E in ${ENVS:-NONE=0}; do
    F=$(echo "$E" | tr '/' '_')_$R
    env $E timeout -k 10 300 python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --no-parity --leafsize $L ${BENCH_ARGS} > $O/b_${L}_${F}.json 2> $O/b_${L}_${F}.err || { cat $O/b_${L}_${F}.err | tail -20; exit 1; }
  done
done
done
