# round 6, GPU session 16: the driver's 20-step window on the final build, kernel trace + HIP runtime API
# trace (no counters), attributed by tools/window_attrib.py: host time from ev0 to the first launch, the
# launches, the synchronize at the end
set -o pipefail
mkdir -p gpurun_out
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d /tmp/r06_s16 -o run --output-format csv \
    -- python3 "$GRAFT_REPO_ROOT"/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$GRAFT_REPO_ROOT"/gpurun_out/r06_s16_bench_prof.json 2>&1) || exit 1
KT=$(find /tmp/r06_s16 -name '*kernel_trace.csv' | head -n1)
AT=$(find /tmp/r06_s16 -name '*hip_api_trace.csv' | head -n1)
python layered-safe-marl_amd/tools/window_attrib.py "$KT" "$AT" > gpurun_out/r06_s16_window_attrib.txt 2>&1 || exit 2
python - "$AT" > gpurun_out/r06_s16_window_api.txt <<'PY'
import csv, sys
api = list(csv.DictReader(open(sys.argv[1])))
rec = [r for r in api if r["Function"] in ("hipEventRecord", "hipEventRecordWithFlags")]
t0 = int(rec[-2]["Start_Timestamp"])
rows = sorted([r for r in api if int(r["Start_Timestamp"]) >= t0], key=lambda r: int(r["Start_Timestamp"]))[:40]
for r in rows:
    print("%9.1f us  %8.1f us  %s" % ((int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["Function"]))
PY
echo rc=$?
