set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/deep0p; mkdir -p $out
for v in 0 1; do
SALZ_DEEP0=$v timeout -k 10 200 rocprofv3 --kernel-trace -d $out/p$v -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --steps 1 --warmup 0 > $out/b$v.json 2> $out/b$v.err || exit 1
done
