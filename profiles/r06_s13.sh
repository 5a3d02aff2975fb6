# round 6, GPU session 13: the reset draw's acceptance on squared distances and the next MT19937 block
# in three rounds -- the parity suite on this build, then config 3's launch durations over 600 steps
# (3 auto-reset launches) for this build and the previous commit's library (990f7c6 == 525928e)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06_s13_tests.txt 2>&1 || exit $?
for V in new prev; do
  if [ $V = prev ]; then export LSM_LIB=$ROOT/layered-safe-marl_amd/tools/liblsm_rollout_525928e.so; else unset LSM_LIB; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r06_s13_$V -o run --output-format csv \
      -- python3 "$ROOT"/bench.py --config 3 --steps 600 --warmup 20 --no-cpu-baseline > "$ROOT"/gpurun_out/r06_s13_bench_$V.json 2>&1) || exit $?
  (cd "$ROOT/layered-safe-marl_amd" && python -m lsm.pmc launches /tmp/r06_s13_$V --kernel "lsm::rollout") > gpurun_out/r06_s13_launches_$V.json || exit $?
done
echo done
