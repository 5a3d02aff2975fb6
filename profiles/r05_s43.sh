# round 5, GPU session 43: process_adj with its scratch buffers reused across calls (lsm.edges._SCRATCH):
# edge tests, per-call time reuse vs per-call allocation in one process, the bench --edges line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_edges.py -m gpu -x -q --timeout 200 --timeout-method thread \
   -p no:cacheprovider > gpurun_out/r05_s43_tests_edges.txt 2>&1 && \
timeout -k 10 300 python -u layered-safe-marl_amd/tools/edges_host_ab.py > gpurun_out/r05_s43_edges_host_ab.json 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_s43_bench_edges.json 2>&1
echo rc=$?
