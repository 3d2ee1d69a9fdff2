set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dbg}
mkdir -p $O
EXP=$GRAFT_REPO_ROOT/nbodyhpc_amd/lib/exp/libnbkd.so
NBKD_LIB=$EXP NBKD_COLLECT_AHEAD=0 timeout -k 10 300 python3 scripts/debug_ahead.py dump /tmp/a0.npy \
 && NBKD_LIB=$EXP NBKD_COLLECT_AHEAD=1 timeout -k 10 300 python3 scripts/debug_ahead.py dump /tmp/a1.npy \
 && timeout -k 10 300 python3 scripts/debug_ahead.py compare /tmp/a0.npy /tmp/a1.npy $O/ahead.json
rc=$?
rm -f /tmp/a0.npy /tmp/a1.npy
exit $rc
