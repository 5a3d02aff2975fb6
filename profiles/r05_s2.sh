# round 5, GPU session 2: float64 operation costs (tools/fp64_rate.hip) and the PyNum fix's tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 layered-safe-marl_amd/tools/fp64_rate > gpurun_out/r05_fp64_rate.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
   -k "hjf or (multi_env and case10)" > gpurun_out/r05_s2_tests.txt 2>&1
echo rc=$?
