# round 5, GPU session 7: stamps across an auto-reset (config 3), the summary kernel tests, the
# driver's exact command under rocprofv3 (window trace), config-2 reward deviation with the identities
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 > ../gpurun_out/r05_v3_stamps_c3_reset.txt 2>&1) && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_metrics.py "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-t4]" "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-64]" \
   -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s7_tests.txt 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_drv3 -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT"/gpurun_out/r05_v3_driver_bench.json 2>&1) && \
python layered-safe-marl_amd/tools/boundary_trace.py "$(find /tmp/r05_drv3 -name '*kernel_trace.csv' | head -n1)" > gpurun_out/r05_v3_driver_window.txt && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05_v3_bench_driver.json 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r05_v3_bench_default.json 2>&1
echo rc=$?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_edges -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > "$GRAFT_REPO_ROOT"/gpurun_out/r05_v3_bench_edges.json 2>&1) && \
cp "$(find /tmp/r05_edges -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_v3_edges_kernel_stats.csv
echo rc=$?
