# radix-scatter workgroup variants (A/B on one box, with parity tests), C3 encoder slots,
# mixed-data pair finishing, and a kernel trace of C3
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/rxab
mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_batch.py -k "suffix_sort_modes or appendix_c or batch" > $o/pytest.log 2>&1 || { tail -5 $o/pytest.log; exit 1; }
SALZ_RADIX_WG512=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "suffix_sort_modes or appendix_c" > $o/pytest512.log 2>&1 || { tail -5 $o/pytest512.log; exit 1; }
tail -1 $o/pytest.log $o/pytest512.log
for r in 1 2 3; do
  for v in "cur 0" "rxgen 0" "rxgen 1"; do set -- $v
    SALZ_LIB_PATH=$PWD/ab/$1.so SALZ_RADIX_WG512=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --steps 5 > $o/rx_$1_$2_$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$o/rx_$1_$2_$r.json'));s=d['stages_ms_last_block'];r=d['roofline'];print('$1 wg512=$2', d['value'], 'sa=%.2f'%s['ms_sa'], r['avg_launch_us'], r['frac'])"
  done
done
for r in 1 2; do
  for sl in 4 6 8; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --workload silesia --slots $sl --steps 3 > $o/c3_s$sl.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$o/c3_s$sl.$r.json'));print('silesia slots=$sl', d['value'])"
  done
  for pv in 0 1; do
    SALZ_SA_PAIRS=$pv timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-e2e --kind mixed --steps 3 > $o/mixed_p$pv.$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('$o/mixed_p$pv.$r.json'));print('mixed pairs=$pv', d['value'], d['stages_ms_last_block']['ms_sa'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof_sil -o prof --output-format csv -- python3 bench.py --no-pmc --no-cpu-baseline --no-e2e --workload silesia --steps 2 --warmup 1 > $o/sil_prof.json 2> $o/sil_prof.err
