# round 5, GPU session 40: the full GPU suite and smoke on the final tree (shipped build 2e6f0d8b)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_s40_smoke.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s40_gpu_tests.txt 2>&1
echo rc=$?
