# round 5, GPU session 34: config-2 reward deviation against the oracle on the final build (the magnetic
# sums now over 26 mirrored segment pairs), one-wave and team kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -s "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-64]" \
   "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-t4]" "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-t2]" \
   -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s34_reward_deviation.txt 2>&1
echo rc=$?
