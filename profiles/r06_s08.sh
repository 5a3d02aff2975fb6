# round 6, GPU session 8: config 4 -- the REXT = false airtaxi team kernel compiled for at most 2
# waves per SIMD (at22: 224 VGPRs; base: 135 VGPRs, the compiler's 3-wave target, which LDS never
# allows) against base and the REXT = true instance (rext, 213 VGPRs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 600 python -u $T/ab_bench.py --config 4 --reps 4 --steps 400 --warmup 40 --allow-old base: at22:LSM_LIB=liblsm_rollout_at22.so rext:LSM_LIB=liblsm_rollout_rext.so > gpurun_out/r06_s08_ab_c4.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
