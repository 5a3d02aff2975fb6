# round 4, GPU session d: batched MT word reads in the reset draw: reset parity, reset trace, stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py -k "reset or philox or golden" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04d_reset_tests.txt 2>&1 && \
timeout -k 10 300 bash profiles/r04_reset_ab.sh r04_v9 base > gpurun_out/r04_v9_reset_ab.log 2>&1 && \
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 > ../gpurun_out/r04_v9_stamps_team_g4.txt 2>&1)
echo rc=$?
timeout -k 10 120 python -u layered-safe-marl_amd/tools/host_overhead.py > gpurun_out/r04_host_overhead.json 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_v9_bench_driver.json 2>&1
echo rc=$?
