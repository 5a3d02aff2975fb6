# round 6, GPU session 1: new edge tests (register-held masks, step-kernel counts, one-pass path),
# the full GPU suite (kernel_select API instead of env knobs; configs 3/4 on the full-shape tables,
# every env vs the oracle), smoke, default bench and bench --edges
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_edges.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s01_tests_edges.txt 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_s01_smoke.txt 2>&1 && \
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s01_gpu_tests.txt 2>&1
echo rc=$?
