set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r02l; mkdir -p $out
for v in "split 20" "stage 20" "stage 18" "stage 16"; do set -- $v
  SALZ_RANK_MODE=$1 SALZ_RANK_RLOG=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --workload fib256 --steps 2 > $out/fib_$1_$2.json 2>$out/fib.err || exit 1
  SALZ_RANK_MODE=$1 SALZ_RANK_RLOG=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 > $out/text_$1_$2.json 2>$out/text.err || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 > $out/text_default.json 2>$out/text.err || exit 1
for f in $out/*.json; do python -c "
import json; d=json.load(open('$f')); print('$f', d['value'], d['stages_ms_last_block']['ms_sa'])"; done
