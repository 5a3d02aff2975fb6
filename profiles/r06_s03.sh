# round 6, GPU session 3: the v_mov_b64 microtest and the edges check (session 2's, pool busy then);
# edge tests; team-kernel reset tests (two-agents-per-ballot draw chain); gradient speculation
# (LSM_AB_GSPEC) hit rate + config-3 A/B; reset-step stamps; config 4 at the 168-VGPR cap (A/B);
# config 5 across the round-3/4/5 libraries (bisect); bench --edges (count pass vs one pass)
set -o pipefail
mkdir -p gpurun_out
T=layered-safe-marl_amd/tools
timeout -k 10 120 ./$T/movb64_hazard > gpurun_out/r06_s03_movb64.txt 2>&1
timeout -k 10 200 python -u $T/edges_check.py $T/liblsm_rollout_s01.so $T/liblsm_edges_branchy.so $T/liblsm_edges_r05.so > gpurun_out/r06_s03_edges_check.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_edges.py -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s03_tests_edges.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py -m gpu -v -k "team_kernel_resets or philox" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s03_tests_resets.txt 2>&1 || exit 1
cd layered-safe-marl_amd && timeout -k 10 200 python -u -m lsm.diag_stamps --team --config 3 --steps 20 --lib liblsm_rollout_gspecst.so > ../gpurun_out/r06_s03_stamps_gspec.txt 2>&1; \
timeout -k 10 200 python -u -m lsm.diag_stamps --team --config 3 --steps 250 --pick 249 > ../gpurun_out/r06_s03_stamps_reset.txt 2>&1; cd ..
timeout -k 10 600 python -u $T/ab_bench.py --config 3 --reps 3 base: gspec:LSM_LIB=liblsm_rollout_gspec.so > gpurun_out/r06_s03_ab_c3_gspec.txt 2>&1
timeout -k 10 600 python -u $T/ab_bench.py --config 4 --reps 2 --steps 200 --warmup 50 base: atwpe3:LSM_LIB=liblsm_rollout_atwpe3.so > gpurun_out/r06_s03_ab_c4_wpe3.txt 2>&1
timeout -k 10 600 python -u $T/ab_bench.py --config 5 --reps 2 --steps 300 --warmup 50 --allow-old base: r05:LSM_LIB=../tools/liblsm_rollout_r05.so r04:LSM_LIB=../tools/liblsm_rollout_r04.so r03:LSM_LIB=../tools/liblsm_rollout_r03.so > gpurun_out/r06_s03_ab_c5_rounds.txt 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --edges > gpurun_out/r06_s03_bench_edges.json 2>&1
echo rc=$?
