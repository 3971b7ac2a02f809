# Env-variant A/B on one box: bash tools/gpu_envab.sh OUT "VAR=a VAR2=b" "VAR=c" ... (R rounds)
set -o pipefail
out=$1; shift
mkdir -p $out
for r in 1 2; do
  k=0
  for v in "$@"; do
    k=$((k+1))
    env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 5 > $out/v$k.$r.json 2> $out/v$k.$r.err || exit 1
    python -c "import json;d=json.load(open('$out/v$k.$r.json'));s=d['stages_ms_last_block'];print('$v', d['value'], ' '.join(f'{k[3:]}={v:.2f}' for k,v in s.items()), d['roundtrip_ok'], d['parity_vs_cpu_port'])"
  done
done
