# round 5, GPU session 33: the episode summary on 32 workgroups (last-block reduction): its GPU tests,
# the summary-time tool, the driver's command twice
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py tests/test_gpu_sharding.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s33_tests.txt 2>&1 && \
timeout -k 10 200 python -u layered-safe-marl_amd/tools/summary_time.py > gpurun_out/r05_s33_summary_time.json 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s33_driver_1.json 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05_s33_driver_2.json 2>&1
echo rc=$?
