set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r02r; mkdir -p $out
for a in 0 1; do
SALZ_ALPHA=$a timeout -k 10 300 rocprofv3 --kernel-trace -d $out/prof_a$a -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --steps 2 --warmup 0 > $out/a$a.json 2> $out/a$a.err || exit 1
done
