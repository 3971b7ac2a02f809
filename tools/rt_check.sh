set -o pipefail
mkdir -p gpurun_out/rt
timeout -k 10 180 python tools/runtime_check.py salz-only > gpurun_out/rt/a.log 2>&1 &&
timeout -k 10 180 python tools/runtime_check.py torch-first > gpurun_out/rt/b.log 2>&1 ;
timeout -k 10 180 python tools/runtime_check.py salz-first > gpurun_out/rt/c.log 2>&1 ;
cat gpurun_out/rt/*.log | grep -v Warning | tail -20
