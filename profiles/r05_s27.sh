# round 5, GPU session 27: (1) process_adj with the round-4 kernels and the edge count read on the device
# (one host sync per call); (2) magnetic segment sums with one Newton step (parity subset + A/B config 2);
# (3) kernel-parameter lines touched in the scalar cache while the record loads are in flight (A/B 3, 2);
# (4) the magnetic sum over 26 mirrored segment pairs instead of 50 segments (pairs, pn1 = pairs + one Newton step)
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
timeout -k 10 300 python -u layered-safe-marl_amd/tools/edges_diag.py > gpurun_out/r05_s27_edges_diag.txt 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_edges.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s27_tests_edges.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r05_s27_bench_edges.json 2>&1 && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r05_s27_edges -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > "$GRAFT_REPO_ROOT"/gpurun_out/r05_s27_bench_edges_prof.json 2>&1) && \
cp "$(find /tmp/r05_s27_edges -name '*kernel_stats.csv' | head -n1)" gpurun_out/r05_s27_edges_kernel_stats.csv && \
LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_pn1.so timeout -k 10 900 python -u -m pytest $(cat profiles/r05_ab_tests.txt) \
   -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s27_tests_pn1.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 base: n1:LSM_LIB=liblsm_rollout_n1.so pairs:LSM_LIB=liblsm_rollout_pairs.so pn1:LSM_LIB=liblsm_rollout_pn1.so > gpurun_out/r05_s27_ab_c2.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 3 base: kpre2:LSM_LIB=liblsm_rollout_kpre2.so > gpurun_out/r05_s27_ab_c3_kpre2.txt 2>&1 && \
timeout -k 10 600 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 3 base: kpre2:LSM_LIB=liblsm_rollout_kpre2.so > gpurun_out/r05_s27_ab_c2_kpre2.txt 2>&1
echo rc=$?
