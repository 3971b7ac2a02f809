set -o pipefail
mkdir -p gpurun_out/dg
export SALZ_CHECK_STAGES=1
timeout -k 10 200 python tools/diag_concurrency.py --threads 4 --iters 30 --device > gpurun_out/dg/c_text.log 2>&1 &&
timeout -k 10 200 python tools/diag_concurrency.py --threads 4 --iters 30 --device --kind mixed --size 2000001 > gpurun_out/dg/c_mixed.log 2>&1 &&
timeout -k 10 200 python tools/diag_concurrency.py --threads 3 --iters 15 --device --kind text --size 9000001 > gpurun_out/dg/c_text9.log 2>&1 &&
timeout -k 10 200 python tools/diag_concurrency.py --threads 4 --iters 40 --kind mixed --size 300001 > gpurun_out/dg/c_small.log 2>&1
rc=$?
for f in c_text c_mixed c_text9 c_small; do echo "== $f"; tail -2 gpurun_out/dg/$f.log; done
exit $rc
