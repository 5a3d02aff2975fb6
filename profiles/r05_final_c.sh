# round 5, final C: the driver's exact command under rocprofv3 (kernel trace -> window attribution),
# bench lines (default, driver-style, config 5, edges), smoke, the full GPU suite
set -o pipefail
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_fdrv -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT"/gpurun_out/r05_driver_bench_prof.json 2>&1) && \
python layered-safe-marl_amd/tools/boundary_trace.py "$(find /tmp/r05_fdrv -name '*kernel_trace.csv' | head -n1)" > gpurun_out/r05_driver_window.txt && \
cp "$(find /tmp/r05_fdrv -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_driver_kernel_stats.csv && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_bench_driver.json 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r05_bench_default.json 2>&1 && \
timeout -k 10 300 python -u bench.py --config 5 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r05_bench_c5.json 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_bench_edges.json 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_gpu_tests.txt 2>&1
echo rc=$?
