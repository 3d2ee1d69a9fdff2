# One parametrised GPU-box runner (round 5; replaces round 4's single-use
# gpu_r04*.sh recipes).  Run through gpurun, from the repo root:
#
#   TAG=r05a STEPS="tests bench" bash scripts/gpu_run.sh
#
# Steps run in the order given; the first that fails ends the call (every GPU
# step has its own time limit).  Everything lands under gpurun_out/$TAG/.
#   tests     pytest -m gpu, then smoke()
#   bench     the default bench line (N = 1, the driver's command)
#   suite     bench.py --suite (SURVEY §8(d)'s secondary runs)
#   trace     rocprofv3 --kernel-trace --stats of a short bench
#   pmc       FETCH_SIZE / WRITE_SIZE passes (separate runs) of collect / select
#             and of the C3 radius count, and the SQ / TCC sets of both
#   step      whole-step HBM bytes: FETCH / WRITE over 1- and 3-step knn_time runs
#   slab      the same per rank for SLABS (default "2:strong 4:strong 8:strong
#             8:weak:1.25e8"): rank 0's slab of the N-GPU bench alone on this GPU
#   rehearse  N > 1 bench lines with every rank on this GPU (NBKD_BENCH_SAME_DEVICE=1)
#   ab        scripts/gpu_ab.sh with LIBS / BALL_LIBS / ARGS / ROUNDS
#   final     smoke() + the default bench line
#   probe     each command of PROBE ("cmd1; cmd2; ..."), 600 s each, into probe.log
#   summarize summarize_prof.py / summarize_step.py on the box (profiles/<tag>_*,
#             copied to $O/profiles), so a later bench / suite step matches them
# Afterwards, in the build container:
#   python scripts/summarize_prof.py gpurun_out/$TAG $TAG     (trace, pmc)
#   python scripts/summarize_step.py gpurun_out/$TAG $TAG     (step)
#   python scripts/summarize_slab.py gpurun_out/$TAG $TAG     (slab)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-run}
O=gpurun_out/$TAG
mkdir -p $O
sha256sum nbodyhpc_amd/lib/libnbkd.so > $O/lib.sha256
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity"
BR="python3 scripts/ball_run.py"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
TCC="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"

say() { echo "[$TAG] $*"; date; }
pmc() { # dir counters regex command...
  local name=$1 ctr=$2 rx=$3; shift 3
  say "pmc $name"
  timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" -d $O/$name -o run \
    --output-format csv -- "$@" > $O/$name.log 2>&1
}
pass() { # dir counter knn_time args...  (every kernel, no regex)
  local name=$1 ctr=$2; shift 2
  say "pass $name"
  timeout -s KILL 400 rocprofv3 --pmc $ctr -d $O/$name -o run --output-format csv -- \
    python3 scripts/knn_time.py "$@" > $O/$name.log 2>&1
}
steps4() { # dir knn_time args...: the 1- and 3-step FETCH / WRITE passes
  local d=$1; shift
  mkdir -p $O/$d
  pass $d/f1 FETCH_SIZE "$@" --steps 1 && pass $d/f3 FETCH_SIZE "$@" --steps 3 \
    && pass $d/w1 WRITE_SIZE "$@" --steps 1 && pass $d/w3 WRITE_SIZE "$@" --steps 3
}

step_tests() {
  say tests
  NBKD_TEST_REPORT_DIR=$O timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > $O/tests.log 2>&1
  local rc=$?
  tail -3 $O/tests.log
  [ $rc -eq 0 ] || return $rc
  say smoke
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $O/smoke.log 2>&1
}
step_bench() {
  say bench
  timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
  local rc=$?
  tail -c 1500 $O/bench.json
  return $rc
}
step_suite() {
  say suite
  timeout -k 10 900 python3 bench.py --suite > $O/suite.json 2> $O/suite.err
}
step_trace() {
  say trace
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B \
    > $O/trace.log 2>&1
}
step_pmc() {
  pmc fetch FETCH_SIZE "knn_collect|knn_select" $B \
    && pmc write WRITE_SIZE "knn_collect|knn_select" $B \
    && pmc ball_fetch FETCH_SIZE ball_count2 $BR \
    && pmc ball_write WRITE_SIZE ball_count2 $BR \
    && pmc pmc_sq1 "$SQ1" "knn_collect|knn_select" $B \
    && pmc pmc_sq2 "$SQ2" "knn_collect|knn_select" $B \
    && pmc pmc_tcc "$TCC" "knn_collect|knn_select" $B \
    && pmc ball_sq1 "$SQ1" ball_count2 $BR \
    && pmc ball_sq2 "$SQ2" ball_count2 $BR
}
step_step() {
  steps4 step --n 1e8 --k 32
}
# summarise trace / pmc / step on the box too (so a later bench step of this
# call finds this build's profiles); the summaries are copied back under $O
step_summarize() {
  say summarize
  python3 scripts/summarize_prof.py $O $TAG > $O/summarize.log 2>&1 && \
  { [ ! -d $O/step ] || python3 scripts/summarize_step.py $O/step $TAG >> $O/summarize.log 2>&1; } && \
  mkdir -p $O/profiles && cp profiles/${TAG}_* $O/profiles/
}
step_slab() {
  local s w sc n
  for s in ${SLABS:-2:strong 4:strong 8:strong 8:weak:1.25e8}; do
    IFS=: read w sc n <<< "$s"
    steps4 slab_${w}_${sc} --n ${n:-1e8} --k 32 --slab-world $w --slab-rank 0 --scaling $sc || return $?
  done
  # summarised on the box too, so a later `rehearse` step of this call finds
  # the profile of this very build (profiles/ is not merged back: copy it)
  python3 scripts/summarize_slab.py $O $TAG && cp profiles/${TAG}_pmc_slab.json $O/
}
step_rehearse() {
  local w
  for w in ${REHEARSE:-2 4}; do
    say "rehearse n$w"
    NBKD_BENCH_SAME_DEVICE=1 timeout -k 10 900 python3 bench.py --gpus $w --steps 3 --warmup 1 \
      --no-cpu-baseline > $O/rehearse_n$w.json 2> $O/rehearse_n$w.err || return $?
    tail -c 2500 $O/rehearse_n$w.json
  done
}
step_ab() {
  say ab
  TAG=$TAG/ab bash scripts/gpu_ab.sh
}
step_final() {
  say final
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > $O/final_smoke.log 2>&1 \
    && timeout -k 10 600 python3 bench.py > $O/final_bench.json 2> $O/final_bench.err
  local rc=$?
  tail -2 $O/final_smoke.log; tail -c 1500 $O/final_bench.json
  return $rc
}

step_probe() {
  local c
  IFS=';' read -ra cmds <<< "$PROBE"
  for c in "${cmds[@]}"; do
    say "probe: $c"
    echo "### $c" >> $O/probe.log
    timeout -k 10 600 $c >> $O/probe.log 2>&1 || return $?
  done
  tail -c 3000 $O/probe.log
}

rc=0
for st in ${STEPS:-tests bench}; do
  step_$st || { rc=$?; echo "[$TAG] step $st failed: $rc"; break; }
done
date
exit $rc
