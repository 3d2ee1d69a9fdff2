# A/B of the radius count's walk-ahead (experiments build, interleaved runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04f}
mkdir -p $O
timeout -k 10 900 python3 -u scripts/lib_ab.py --libs "exp@NBKD_BALL_AHEAD=0,exp@NBKD_BALL_AHEAD=1,prod" --rounds 3 -- --n 1e8 --ball 0.01 > $O/ball_ahead.log 2>&1
rc=$?
tail -6 $O/ball_ahead.log
exit $rc
