# round 6, GPU session 15: config 3's auto-reset launch and the two steps after it, with the reset's graph
# outputs as plain (base) or nontemporal stores (rnts): kernel traces over 600 steps (3 boundaries)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
for V in base rnts base2 rnts2; do
  case $V in rnts*) export LSM_LIB=$ROOT/layered-safe-marl_amd/csrc/liblsm_rollout_rnts.so;; *) unset LSM_LIB;; esac
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/r06_s15_$V -o run --output-format csv \
      -- python3 "$ROOT"/bench.py --config 3 --steps 600 --warmup 20 --no-cpu-baseline > "$ROOT"/gpurun_out/r06_s15_bench_$V.json 2>&1) || exit $?
  (cd "$ROOT/layered-safe-marl_amd" && python -m lsm.pmc launches /tmp/r06_s15_$V --kernel "lsm::rollout") > gpurun_out/r06_s15_launches_$V.json || exit $?
done
echo done
