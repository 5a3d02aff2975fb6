# round 5, GPU session 35: action rows in LDS + one-group table loads + unconditional overflow-row
# address (cur) vs the same without the overflow change (vc) vs the shipped build (old):
# parity on cur, then A/B at configs 3 and 4
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 600 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[double_integrator-8-4]" \
   "tests/test_gpu_parity.py::test_gpu_team_kernel_resets_match_oracle[airtaxi-16-4]" \
   "tests/test_gpu_parity.py::test_gpu_separation_chain_unbounded" \
   "tests/test_gpu_parity.py::test_gpu_action_index_out_of_range_is_reported" \
   "tests/test_gpu_parity.py::test_gpu_action_encodings_and_dummy_semantics" \
   -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s35_tests.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 cur: vc:LSM_LIB=liblsm_rollout_vc.so old:LSM_LIB=liblsm_rollout_old.so > gpurun_out/r05_s35_ab_c3.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 cur: vc:LSM_LIB=liblsm_rollout_vc.so old:LSM_LIB=liblsm_rollout_old.so > gpurun_out/r05_s35_ab_c4.txt 2>&1
echo rc=$?
