# round 6, GPU session 22: address translation of config 3's step kernel -- UTCL1 requests, translation
# hits / misses and permission misses per launch (one TCP counter pass, no trace domains)
set -o pipefail
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_PERMISSION_MISS_sum \
   --kernel-include-regex rollout_ -d /tmp/r06_s22 -o run --output-format csv \
   -- python3 $R/bench.py --config 3 --steps 60 --warmup 20 --no-cpu-baseline > $R/gpurun_out/r06_s22_pmc.log 2>&1) || exit 3
cd layered-safe-marl_amd
python -m lsm.pmc counters /tmp/r06_s22 --kernel "lsm::rollout" > $R/gpurun_out/r06_s22_utcl1.txt 2>&1
echo rc=$?
