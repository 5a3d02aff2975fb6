# round 5, GPU session 16: phase-A sub-stamps (pair loop, argmins, gradient) at config 3
set -o pipefail
mkdir -p gpurun_out
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 120 > ../gpurun_out/r05_s16_stamps_c3.txt 2>&1)
echo rc=$?
