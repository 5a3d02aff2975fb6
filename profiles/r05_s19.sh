# round 5, GPU session 19: process_adj as count+look-back scan (one kernel) and a prefetching emit with
# the edge count read on the device (one host sync per call): edge tests, bench --edges, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_edges.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s19_tests_edges.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_s19_bench_edges.json 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_s19_edges -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > "$GRAFT_REPO_ROOT"/gpurun_out/r05_s19_bench_edges_prof.json 2>&1) && \
cp "$(find /tmp/r05_s19_edges -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_s19_edges_kernel_stats.csv
echo rc=$?
