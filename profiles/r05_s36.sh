# round 5, GPU session 36: the separation-chain test on the shipped build (old), vc and cur; a test
# failure (rc 1) goes on to the next library, anything else (timeout, crash) ends the script
set -o pipefail
mkdir -p gpurun_out
export LSM_LIB_AB=1
for V in old vc cur; do
  L=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout_$V.so; [ $V = cur ] && L=$PWD/layered-safe-marl_amd/csrc/liblsm_rollout.so
  LSM_LIB=$L timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_gpu_separation_chain_unbounded" \
     -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_s36_sep_$V.txt 2>&1
  rc=$?; echo "$V rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
