set -o pipefail
mkdir -p gpurun_out/r02c
for L in 24 32 48 64; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --leafsize $L > gpurun_out/r02c/leaf$L.json 2> gpurun_out/r02c/leaf$L.err || exit 1
done
