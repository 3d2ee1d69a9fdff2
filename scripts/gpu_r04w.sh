# GPU tests + profiles of the head (scripts/gpu_r04u.sh), then two diagnostics:
# the k = 100 phase split and a PMC pass over the bucketing kernels.
# usage (on the box): TAG=r04w bash scripts/gpu_r04w.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04w}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash scripts/gpu_r04u.sh \
 && echo "[$TAG] k100 phases" && timeout -k 10 300 python3 scripts/knn_time.py --n 1e8 --k 100 --steps 2 > $O/k100.json 2> $O/k100.err \
 && echo "[$TAG] leaf_key pmc" && timeout -s KILL 300 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "leaf_key3|os_pass" -d $O/lk -o run --output-format csv -- python3 scripts/knn_time.py --n 1e8 --steps 1 > $O/lk.log 2>&1
rc=$?
tail -2 $O/k100.json
exit $rc
