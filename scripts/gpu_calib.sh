# PMC calibration of this code's store / load shapes (scripts/calib/pmc_calib.hip):
# one plain run for the known byte counts, then WRITE_SIZE and FETCH_SIZE in
# separate rocprofv3 passes.  usage (on the box): TAG=r04a bash scripts/gpu_calib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG/calib
mkdir -p $O
echo "[calib] known"; date
timeout -k 10 120 scripts/calib/pmc_calib > $O/known.json \
 && echo "[calib] write" && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- scripts/calib/pmc_calib > $O/write.log 2>&1 \
 && echo "[calib] fetch" && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- scripts/calib/pmc_calib > $O/fetch.log 2>&1
rc=$?
cat $O/known.json
exit $rc
