# round 5, final C: bench lines (driver-style, default, config 5, edges), smoke, the full GPU suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_driver.json 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r05_bench_default.json 2>&1 && \
timeout -k 10 300 python -u bench.py --config 2 --no-cpu-baseline > gpurun_out/r05_bench_c2.json 2>&1 && \
timeout -k 10 300 python -u bench.py --config 4 --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/r05_bench_c4.json 2>&1 && \
timeout -k 10 300 python -u bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r05_bench_c5.json 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_bench_edges.json 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests.txt 2>&1
echo rc=$?
