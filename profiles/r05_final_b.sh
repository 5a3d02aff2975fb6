# round 5, final profiles B: config 5
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 5 > gpurun_out/r05_final_b_c5.log 2>&1
echo rc=$?
