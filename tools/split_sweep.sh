timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -3 gpurun_out/pt.log
SALZ_CHECK_STAGES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/chk.json 2> gpurun_out/chk.err || { tail -3 gpurun_out/chk.err; exit 1; }
SALZ_CHECK_STAGES=1 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --kind mixed > gpurun_out/chkm.json 2> gpurun_out/chkm.err || { tail -3 gpurun_out/chkm.err; exit 1; }
echo checks ok
bash tools/ab.sh 2
bash tools/ab.sh 1 --kind mixed --steps 2
