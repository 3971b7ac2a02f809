set -o pipefail
mkdir -p gpurun_out/dg
for k in 1 2 3 4; do
timeout -k 10 200 python bench.py --workload silesia --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dg/s$k.json 2> gpurun_out/dg/s$k.err
echo "plain $k rc=$? $(tail -1 gpurun_out/dg/s$k.err | cut -c1-200)"
SALZ_CHECK_SA=1 timeout -k 10 200 python bench.py --workload silesia --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dg/c$k.json 2> gpurun_out/dg/c$k.err
echo "checked $k rc=$? $(tail -1 gpurun_out/dg/c$k.err | cut -c1-200)"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --kind mixed --steps 2 --warmup 1 > gpurun_out/dg/m.json 2> gpurun_out/dg/m.err
echo "mixed rc=$?"
for k in 5 6; do
timeout -k 10 200 python bench.py --workload silesia --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/dg/s$k.json 2> gpurun_out/dg/s$k.err
echo "plain $k rc=$? $(tail -1 gpurun_out/dg/s$k.err | cut -c1-200)"
done
