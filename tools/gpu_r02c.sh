set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r02c; mkdir -p $out
timeout -k 10 200 python bench.py > $out/bench.json 2> $out/bench.err &&
timeout -k 10 200 python bench.py --workload silesia --steps 2 --no-cpu-baseline > $out/silesia.json 2> $out/silesia.err &&
timeout -k 10 300 python bench.py --workload enwik9 --steps 1 --no-cpu-baseline --no-e2e > $out/enwik9.json 2> $out/enwik9.err
rc=$?
cat $out/bench.json $out/silesia.json $out/enwik9.json | cut -c1-400; tail -5 $out/*.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --workload silesia --size 50000000 --no-cpu-baseline --no-e2e > $out/two.json 2> $out/two.err
echo "two-rank rc=$?"; cut -c1-600 $out/two.json; tail -20 $out/two.err
exit 0
