# round 6, GPU session 11: config 4 -- what the lean 13.44 KB layout costs vs what the third wave
# gains: the layout held at 2 workgroups per CU (20 KB of LDS padding, 2 waves per SIMD: lpad2), the
# 3-workgroup build with the landmark-landmark entries recomputed from the landmark positions in LDS
# (llrc) or read from HBM with global loads (llgas; base: flat loads, which LDS waits also wait for),
# and the previous commit's 19.3 KB layout (prev)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 1000 python -u $T/ab_bench.py --config 4 --reps 2 --steps 400 --warmup 40 --allow-old base: lpad2:LSM_LIB=liblsm_rollout_lpad2.so llrc:LSM_LIB=liblsm_rollout_llrc.so llgas:LSM_LIB=liblsm_rollout_llgas.so prev:LSM_LIB=../tools/liblsm_rollout_525928e.so > gpurun_out/r06_s11_ab_c4.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
