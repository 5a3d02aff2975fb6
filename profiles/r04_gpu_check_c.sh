# round 4, GPU session c: agent-register scenario draw (L = 2), lane-parallel episode summary,
# early MT loads: GPU suite, reset-step trace, stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r04c_gpu_tests.txt 2>&1 && \
timeout -k 10 300 bash profiles/r04_reset_ab.sh r04_v5 base > gpurun_out/r04_v5_reset_ab.log 2>&1 && \
(cd layered-safe-marl_amd && LSM_LIB_AB=1 timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 250 > ../gpurun_out/r04_v5_stamps_team_g4.txt 2>&1)
echo rc=$?
