# round 5, final profiles A: rocprofv3 kernel trace + PMC (FETCH_SIZE, WRITE_SIZE) + SQ counters of the
# shipped library (build id recorded in profiles/pmc_traffic.json) at configs 3 and 2
set -o pipefail
mkdir -p gpurun_out
bash profiles/collect.sh r05 3 > gpurun_out/r05_final_a_c3.log 2>&1 && \
bash profiles/collect.sh r05 2 > gpurun_out/r05_final_a_c2.log 2>&1
echo rc=$?
