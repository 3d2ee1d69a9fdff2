# the driver's own round-end commands on the head: smoke(), then the default
# bench line (N = 1), whose roofline must carry the PMC traffic of this build.
# usage (on the box): TAG=r04final bash scripts/gpu_final_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r04final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
 && timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
rc=$?
tail -2 $O/smoke.log; tail -c 1500 $O/bench.json
exit $rc
