# round 5, GPU session 9: sub-stamps of the agent wave's integration (config 3), the split summary kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s9_tests.txt 2>&1 && \
timeout -k 10 120 python -u layered-safe-marl_amd/tools/summary_time.py > gpurun_out/r05_v4_summary_time.json 2>&1 && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 120 > ../gpurun_out/r05_v4_stamps_c3.txt 2>&1)
echo rc=$?
