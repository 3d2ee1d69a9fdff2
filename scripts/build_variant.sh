# Build libnbkd.so with one source file replaced (A/B experiments):
#   bash scripts/build_variant.sh <name> <replacement.hip> <original-basename>
# -> nbodyhpc_amd/lib/exp/<name>/libnbkd.so (objects of the other sources reused)
set -e
cd "$(dirname "$0")/.."
NAME=$1; SRC=$2; ORIG=$3
OUT=nbodyhpc_amd/lib/exp/$NAME
mkdir -p $OUT
cp "$SRC" nbodyhpc_amd/csrc/_variant_$ORIG
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c nbodyhpc_amd/csrc/_variant_$ORIG -o $OUT/$ORIG.o
rm -f nbodyhpc_amd/csrc/_variant_$ORIG
OBJS=""
for o in nbodyhpc_amd/lib/obj/*.o; do
  b=$(basename $o .o)
  if [ "$b" = "$ORIG" ]; then OBJS="$OBJS $OUT/$ORIG.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libnbkd.so $OBJS -ldl
echo $OUT/libnbkd.so
