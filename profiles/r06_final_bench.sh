# round 6, final build: the default bench line (config 3, with the CPU baseline), the driver's 20-step
# window twice, configs 2 / 4 / 5, the edge hand-off (--edges) and the row-buffer insert (--buffer)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/r06_bench_default.json 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_driver.json 2>&1 || exit $?
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_bench_driver2.json 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/r06_bench_c2.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config 4 --steps 300 --warmup 60 --no-cpu-baseline > gpurun_out/r06_bench_c4.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config 5 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r06_bench_c5.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r06_bench_edges.json 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --buffer > gpurun_out/r06_bench_buffer.json 2>&1
rc=$?; echo "rc=$rc"; exit $rc
