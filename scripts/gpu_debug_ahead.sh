set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dbg}
mkdir -p $O
NBKD_LIB=$GRAFT_REPO_ROOT/nbodyhpc_amd/lib/exp/libnbkd.so timeout -k 10 600 python3 scripts/debug_ahead.py $O/ahead.json
