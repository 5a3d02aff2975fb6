# round 6, GPU session 18: the coalesced episode-summary kernel (lsm_metrics.hip) -- its GPU tests, its
# device time (tools/summary_time.py: back to back and right behind a rollout step), and the driver's
# 20-step window three times
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_metrics.py tests/test_dist.py tests/test_bench_cpu.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s18_tests.txt 2>&1 || exit $?
timeout -k 10 200 python -u layered-safe-marl_amd/tools/summary_time.py > gpurun_out/r06_s18_summary_time.json 2>&1 || exit $?
for k in 1 2 3; do timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r06_s18_driver_$k.json 2>&1 || exit $?; done
echo done
