# Mixed 100 MB kernel trace of the current build (per-pass parse breakdown).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-r03t}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_mixed -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 1 --warmup 1 > $out/mixed.json 2> $out/mixed.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_text -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 1 --warmup 1 > $out/text.json 2> $out/text.err
