# round 6, GPU session 7: the team kernels specialised on the optional-reward block (base: REXT =
# false at configs 2-4, <0, 8, 4> 0 B of scratch instead of 92 B per lane, <1, 16, 4> 135 VGPRs
# instead of 213) against the same build launching the REXT = true instances (rext), and
# nontemporal graph stores at N = 8 (nts8); then the parity suite's team cases on this build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 400 python -u $T/ab_bench.py --config 3 --reps 3 --steps 400 --warmup 50 --allow-old base: rext:LSM_LIB=liblsm_rollout_rext.so nts8:LSM_LIB=liblsm_rollout_nts8.so > gpurun_out/r06_s07_ab_c3.txt 2>&1 && \
timeout -k 10 300 python -u $T/ab_bench.py --config 2 --reps 3 --steps 400 --warmup 50 --allow-old base: rext:LSM_LIB=liblsm_rollout_rext.so > gpurun_out/r06_s07_ab_c2.txt 2>&1 && \
timeout -k 10 400 python -u $T/ab_bench.py --config 4 --reps 2 --steps 60 --warmup 10 --allow-old base: rext:LSM_LIB=liblsm_rollout_rext.so > gpurun_out/r06_s07_ab_c4.txt 2>&1 && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "team or multi_env" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s07_tests.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
