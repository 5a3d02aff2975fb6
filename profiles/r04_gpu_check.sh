set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_gpu_tests_a.txt 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_a.txt 2>&1 && \
{ LSM_LIB=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_wdraw.so LSM_LIB_AB=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_layouts.py -k "team_kernel_resets or philox_reset" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r04_wdraw_tests.txt 2>&1; r=$?; echo wdraw_tests_rc=$r; [ $r -le 1 ]; } && \
timeout -k 10 300 python -u bench.py --steps 1000 --warmup 250 > gpurun_out/r04_bench_a.json 2> gpurun_out/r04_bench_a.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r04_bench_driver_a.json 2>&1 && \
timeout -k 10 400 python -u layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 2 base: pro:LSM_LIB=liblsm_rollout_pro.so nodec:LSM_LIB=liblsm_rollout_nodec.so pronodec:LSM_LIB=liblsm_rollout_pronodec.so nodec0:LSM_LIB=liblsm_rollout_nodec0.so pronodec0:LSM_LIB=liblsm_rollout_pronodec0.so > gpurun_out/r04_v1_ab_c3.txt 2>&1 && \
timeout -k 10 300 python -u layered-safe-marl_amd/tools/ab_bench.py --config 2 --reps 2 base: nodec:LSM_LIB=liblsm_rollout_nodec.so pronodec:LSM_LIB=liblsm_rollout_pronodec.so > gpurun_out/r04_v1_ab_c2.txt 2>&1 && \
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 > ../gpurun_out/r04_stamps_team_g4.txt 2>&1) && \
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --config 2 --steps 60 > ../gpurun_out/r04_stamps_team_g4_c2.txt 2>&1) && \
timeout -k 10 700 bash profiles/r04_reset_ab.sh r04_v1 base wdraw rs_noscen rs_noemit > gpurun_out/r04_reset_ab.log 2>&1
echo rc=$?
