# round 6, GPU session 12: config 4 -- the lean 13.44 KB layout with the landmark-landmark entries
# recomputed, at 3 workgroups per CU (llrc) and held at 2 (lrcpad2: 20 KB LDS padding, 2 waves per
# SIMD), against the previous commit's 19.3 KB layout (prev): the third wave alone, same code
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 900 python -u $T/ab_bench.py --config 4 --reps 3 --steps 400 --warmup 40 --allow-old llrc:LSM_LIB=liblsm_rollout_llrc.so lrcpad2:LSM_LIB=liblsm_rollout_lrcpad2.so prev:LSM_LIB=../tools/liblsm_rollout_525928e.so > gpurun_out/r06_s12_ab_c4.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
