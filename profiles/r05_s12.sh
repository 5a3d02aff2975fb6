# round 5, GPU session 12: A/B of the checked reciprocal grid division and this round's cumulative change
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 head:LSM_LIB=liblsm_rollout_head.so base: nomdiv:LSM_NO_MDIV=1 > gpurun_out/r05_s11_ab_c3.txt 2>&1 && \
timeout -k 10 900 python -u layered-safe-marl_amd/tools/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 head:LSM_LIB=liblsm_rollout_head.so base: nomdiv:LSM_NO_MDIV=1 > gpurun_out/r05_s11_ab_c4.txt 2>&1
echo rc=$?
