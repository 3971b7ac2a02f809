#!/bin/bash
# The split suffix array at one rank (no launcher: the env gives rank 0 of 1, so rocprofv3 can take
# the program itself): local path, forced exchange through the library's RCCL communicator, and the
# torch.distributed callbacks; then a kernel trace of the forced-exchange run.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/${TAG:-split1}; mkdir -p $out
export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29555
timeout -k 10 300 python tools/bench_split.py --kind text --steps 3 > $out/local.json 2> $out/local.err &&
SALZ_SA=xchg timeout -k 10 300 python tools/bench_split.py --kind text --steps 3 > $out/xchg_rccl.json 2> $out/xchg_rccl.err &&
SALZ_SA=xchg timeout -k 10 300 python tools/bench_split.py --kind text --steps 3 --callbacks > $out/xchg_cb.json 2> $out/xchg_cb.err &&
SALZ_SA=xchg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o prof --output-format csv -- python3 tools/bench_split.py --kind text --steps 2 > $out/prof.json 2> $out/prof.err &&
python tools/prof_summary.py $out/prof/prof_kernel_stats.csv > $out/kernel_stats.txt 2>&1
rc=$?
cat $out/local.json $out/xchg_rccl.json $out/xchg_cb.json; head -30 $out/kernel_stats.txt
exit $rc
