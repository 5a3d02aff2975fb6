# round 5, GPU session 4: per-phase dynamic instruction counts of the team kernel (config 3),
# team stamps at config 2 after the magnetic-field change, reward deviations at configs 2/3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
(cd layered-safe-marl_amd && timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVES \
   -d /tmp/pc3 -o run --output-format csv -- python3 -m lsm.diag_phasecount --team --config 3 > $R/gpurun_out/r05_pc3.log 2>&1) && \
(cd layered-safe-marl_amd && python -m lsm.diag_phasecount --team --reduce /tmp/pc3 --config 3 > $R/gpurun_out/r05_phasecount_c3.txt 2>&1) && \
(cd layered-safe-marl_amd && timeout -k 10 300 python -u -m lsm.diag_stamps --team --config 2 --steps 120 > $R/gpurun_out/r05_v1_stamps_c2.txt 2>&1) && \
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[1-t4]" "tests/test_gpu_parity.py::test_gpu_matches_oracle_multi_env[0-t4]" \
   -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s4_rewdev.txt 2>&1
echo rc=$?
