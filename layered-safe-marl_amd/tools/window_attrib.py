"""Attribute the driver's timed window from a rocprofv3 kernel trace + HIP runtime API trace of
`bench.py --gpus 1 --steps 20 --warmup 5`: the window is bracketed by the last two hipEventRecord
calls of the run (bench.py's ev0 / ev1); reports the host time from ev0's record to the first step
launch, each step kernel's start (relative to ev0's record) and duration, idle gaps, and the time from
the last kernel's end to the return of the synchronize that ends the window.

    python layered-safe-marl_amd/tools/window_attrib.py kernel_trace.csv hip_api_trace.csv
"""
import csv
import sys


def main():
    kt, at = sys.argv[1], sys.argv[2]
    api = [r for r in csv.DictReader(open(at))]
    ker = [r for r in csv.DictReader(open(kt))]
    rec = [r for r in api if r["Function"] in ("hipEventRecord", "hipEventRecordWithFlags")]
    ev0, ev1 = rec[-2], rec[-1]
    t0, t1 = int(ev0["Start_Timestamp"]), int(ev1["End_Timestamp"])
    syncs = [r for r in api if r["Function"] in ("hipDeviceSynchronize", "hipStreamSynchronize", "hipEventSynchronize")
             and int(r["Start_Timestamp"]) >= t1]
    sync_end = int(syncs[0]["End_Timestamp"]) if syncs else None
    launches = [r for r in api if "Launch" in r["Function"] and t0 <= int(r["Start_Timestamp"]) <= t1]
    ks = sorted([r for r in ker if t0 <= int(r["Start_Timestamp"]) and int(r["End_Timestamp"]) <= (sync_end or t1) + 10**9],
                key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in ks if int(r["Start_Timestamp"]) >= t0 and int(r["Start_Timestamp"]) <= (sync_end or t1)]
    us = lambda ns: ns / 1000.0
    print("window: ev0 record -> ev1 record %.1f us; host launch calls in it: %d" % (us(t1 - t0), len(launches)))
    if launches:
        print("first launch call starts %.1f us after ev0's record" % us(int(launches[0]["Start_Timestamp"]) - t0))
    prev_end = None
    busy = 0
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) if prev_end is not None else (s - t0)
        busy += e - s
        print("%8.1f us  start %+9.1f  gap %7.1f  %s" % (us(e - s), us(s - t0), us(gap), r["Kernel_Name"][:60]))
        prev_end = e
    if ks:
        print("kernels busy %.1f us; first kernel starts %.1f us after ev0's record; last ends %.1f us after it"
              % (us(busy), us(int(ks[0]["Start_Timestamp"]) - t0), us(int(ks[-1]["End_Timestamp"]) - t0)))
    if sync_end:
        print("synchronize after ev1 returns %.1f us after the last kernel's end" % us(sync_end - int(ks[-1]["End_Timestamp"])))


if __name__ == "__main__":
    main()
