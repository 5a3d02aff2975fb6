# round 6, GPU session 6: the workgroup kernel's REXT specialisation (config 5 A/B against round 3's
# library) and the one-pass edge call's pinned nnz read (bench --edges), with the block-kernel parity
# cases and the edge tests on this build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=layered-safe-marl_amd/tools
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_edges.py -m gpu -q -k "block or edge" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s06_tests.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r06_s06_bench_edges.json 2>&1 && \
timeout -k 10 600 python -u $T/ab_bench.py --config 5 --reps 3 --steps 300 --warmup 50 --allow-old base: r03:LSM_LIB=../tools/liblsm_rollout_r03.so > gpurun_out/r06_s06_ab_c5.txt 2>&1
rc=$?; echo "rc=$rc"; exit $rc
