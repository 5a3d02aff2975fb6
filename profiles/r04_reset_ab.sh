#!/bin/bash
# Reset-step A/B (run on the GPU box from the repo root): kernel traces of a 600-step config-3
# bench per library; lsm.pmc launches lists the slowest launches (the auto-reset steps).
#   bash profiles/r04_reset_ab.sh TAG name1 name2 ...   (name = base | a csrc/liblsm_rollout_<name>.so)
set -o pipefail
R=$(pwd); export TMPDIR=/tmp; TAG=$1; shift
for V in "$@"; do
  L=$R/layered-safe-marl_amd/csrc/liblsm_rollout.so
  [ "$V" != base ] && L=$R/layered-safe-marl_amd/csrc/liblsm_rollout_$V.so
  rm -rf /tmp/rc_$V && mkdir -p /tmp/rc_$V
  (cd /tmp && LSM_LIB=$L LSM_LIB_AB=1 timeout -k 10 200 rocprofv3 --kernel-trace -d /tmp/rc_$V -o run --output-format csv \
      -- python3 $R/bench.py --config 3 --steps 600 --warmup 20 --no-cpu-baseline > $R/gpurun_out/${TAG}_rc_$V.json 2>&1) || exit 1
  (cd $R/layered-safe-marl_amd && python -m lsm.pmc launches /tmp/rc_$V --kernel "lsm::rollout") > gpurun_out/${TAG}_reset_$V.json || exit 1
done
echo done
