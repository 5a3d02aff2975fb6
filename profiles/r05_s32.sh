# round 5, GPU session 32: team-kernel stamps of the step right after the episode boundary (t = 250)
# against an ordinary step (t = 240), config 3
set -o pipefail
mkdir -p gpurun_out
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 245 --pick 250 > ../gpurun_out/r05_s32_stamps_post_reset.txt 2>&1) && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --steps 245 --pick 240 > ../gpurun_out/r05_s32_stamps_t240.txt 2>&1)
echo rc=$?
