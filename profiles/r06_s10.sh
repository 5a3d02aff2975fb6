# round 6, GPU session 10: the airtaxi team kernel's lean layout at 13.44 KB per env (lmd read from the
# HBM record, landmark rows' agent columns read transposed, aa2 in U2) -> 3 workgroups of 4 envs per CU
# at 3 waves per SIMD: parity (the GPU parity suite and the edge tests) first, then config 4 A/B
# against the 2-workgroup build of the previous commit (525928e) and the 3-wave build with the
# scheduler's upper bound open (wpe38)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_edges.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s10_tests.txt 2>&1 && \
timeout -k 10 600 python -u $T/ab_bench.py --config 4 --reps 3 --steps 400 --warmup 40 --allow-old base: wpe38:LSM_LIB=liblsm_rollout_wpe38.so prev:LSM_LIB=../tools/liblsm_rollout_525928e.so > gpurun_out/r06_s10_ab_c4.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
