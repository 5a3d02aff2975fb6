# round 5, final profiles A (fifth call; config 3 is in profiles/r05_config3_*): configs 4 and 2, counter
# passes restricted to the step kernel (collect.sh)
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 4 > gpurun_out/r05_final_a_c4.log 2>&1 && \
bash profiles/collect.sh r05 2 > gpurun_out/r05_final_a_c2.log 2>&1
echo rc=$?
