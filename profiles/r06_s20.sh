# round 6, GPU session 20: config 3 with the HJ value lookups gathered from the 25 MB node table (16
# scattered 4-B loads per lookup, Infinity-Cache resident) instead of the 400 MB cell-corner table (one
# 64-B cell): parity of the variant on the multi-env cases first, then the A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_nodes.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "multi_env or full_size" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s20_tests_nodes.txt 2>&1 || exit $?
timeout -k 10 500 python -u $T/ab_bench.py --config 3 --reps 3 --steps 400 --warmup 50 --allow-old base: nodes:LSM_LIB=liblsm_rollout_nodes.so > gpurun_out/r06_s20_ab_c3.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
