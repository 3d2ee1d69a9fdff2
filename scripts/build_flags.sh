# Build libnbkd.so with extra compile flags on some sources (A/B experiments):
#   bash scripts/build_flags.sh <name> "<flags>" <source-basename>...
# -> nbodyhpc_amd/lib/exp/<name>/libnbkd.so (objects of the other sources reused
#    from nbodyhpc_amd/lib/obj, so build the production library first)
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; shift 2
OUT=nbodyhpc_amd/lib/exp/$NAME
mkdir -p $OUT
for SRC in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off $FLAGS \
    -c nbodyhpc_amd/csrc/$SRC -o $OUT/$SRC.o &
done
wait
OBJS=""
for o in nbodyhpc_amd/lib/obj/*.o; do
  b=$(basename $o .o)
  if [ -f $OUT/$b.o ]; then OBJS="$OBJS $OUT/$b.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnbkd.so $OBJS -ldl
echo $OUT/libnbkd.so
