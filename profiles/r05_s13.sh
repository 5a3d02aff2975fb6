# round 5, GPU session 13: filter-off adjacency in phase C (parity + A/B at config 2), phase-C trims (A/B config 3)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_adjc2.so timeout -k 10 900 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-t2]" "tests/test_gpu_parity.py::test_gpu_matches_reference_golden[di_n8_off_ep2-wave]" \
   "tests/test_gpu_parity.py::test_gpu_matches_reference_golden[di_n8_collab-wave]" "tests/test_gpu_parity.py::test_gpu_matches_reference_golden[di_n4_rw_hj_off-wave]" \
   -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s13_tests_adjc2.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 base: adjc2:LSM_LIB=liblsm_rollout_adjc2.so > gpurun_out/r05_s13_ab_c2.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: > gpurun_out/r05_s13_ab_c3.txt 2>&1
echo rc=$?
