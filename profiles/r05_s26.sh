# round 5, GPU session 26: process_adj: round-4 count + hipcub scan + emit kernels, emit reading nnz on the device (one host sync per call);
# repeated-count diagnostic, edge tests, bench --edges, kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u layered-safe-marl_amd/tools/edges_diag.py > gpurun_out/r05_s26_edges_diag.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_edges.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s26_tests_edges.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_s26_bench_edges.json 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_s26_edges -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > "$GRAFT_REPO_ROOT"/gpurun_out/r05_s26_bench_edges_prof.json 2>&1) && \
cp "$(find /tmp/r05_s26_edges -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_s26_edges_kernel_stats.csv
echo rc=$?
