# round 6, GPU session 4: edge tests (counts before the node staging); kernel trace of bench --edges
# (which edge kernel changed); the full GPU suite and smoke on this build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_edges.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s04_tests_edges.txt 2>&1 || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r06_s04_edges -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > "$GRAFT_REPO_ROOT"/gpurun_out/r06_s04_bench_edges_prof.json 2>&1) && \
cp "$(find /tmp/r06_s04_edges -name '*kernel_stats.csv' | head -n1)" gpurun_out/r06_s04_edges_kernel_stats.csv
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_s04_smoke.txt 2>&1 && \
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s04_gpu_tests.txt 2>&1
echo rc=$?
