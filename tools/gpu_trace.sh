#!/bin/bash
# One GPU call: rocprofv3 kernel traces of one encode of the mixed 100 MB block and of the
# Silesia-sized workload, with the parse's per-pass log; read them with tools/trace_rounds.py
# (suffix-sort rounds) and tools/parse_passes.py (parse passes).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-trace}; mkdir -p $out
SALZ_DEBUG=parse timeout -k 10 200 rocprofv3 --kernel-trace -d $out/mixed -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 1 --warmup 0 > $out/mixed.json 2> $out/mixed.err &&
SALZ_DEBUG=parse timeout -k 10 200 rocprofv3 --kernel-trace -d $out/sil -o prof --output-format csv -- python3 bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --steps 1 --warmup 0 > $out/sil.json 2> $out/sil.err
