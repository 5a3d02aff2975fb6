# round 4, GPU session b: wave-parallel reset draw as the default, rsq magnetic sums (GPU suite),
# gather-latency bounds at config 3, magnetic A/B at config 2, stamps, reset-step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04b_gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 2 base: magdiv:LSM_LIB=liblsm_rollout_magdiv.so > gpurun_out/r04_v2_ab_c2_mag.txt 2>&1 && \
timeout -k 10 400 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 2 base: valhot:LSM_LIB=liblsm_rollout_valhot.so gradhot:LSM_LIB=liblsm_rollout_gradhot.so hot2:LSM_LIB=liblsm_rollout_hot2.so noout:LSM_LIB=liblsm_rollout_noout.so > gpurun_out/r04_v2_ab_c3_bounds.txt 2>&1 && \
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 > ../gpurun_out/r04_v2_stamps_team_g4.txt 2>&1) && \
timeout -k 10 500 bash profiles/r04_reset_ab.sh r04_v2 base lanedraw > gpurun_out/r04_v2_reset_ab.log 2>&1
echo rc=$?
