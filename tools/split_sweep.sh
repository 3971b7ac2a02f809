timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; tail -2 gpurun_out/pt.log
bash tools/ab.sh 2
