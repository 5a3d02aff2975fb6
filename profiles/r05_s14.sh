# round 5, GPU session 14: phase sensitivity (a ~3000-cycle sleep in one phase at a time) at configs 3 and 2
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: d1:LSM_LIB=liblsm_rollout_d1.so \
   d2:LSM_LIB=liblsm_rollout_d2.so d3:LSM_LIB=liblsm_rollout_d3.so d4:LSM_LIB=liblsm_rollout_d4.so d5:LSM_LIB=liblsm_rollout_d5.so > gpurun_out/r05_s14_ab_c3.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 base: d1:LSM_LIB=liblsm_rollout_d1.so \
   d3:LSM_LIB=liblsm_rollout_d3.so d4:LSM_LIB=liblsm_rollout_d4.so d5:LSM_LIB=liblsm_rollout_d5.so > gpurun_out/r05_s14_ab_c2.txt 2>&1
echo rc=$?
