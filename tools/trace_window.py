"""Timeline of bench.py's timed region from a rocprofv3 kernel trace (csv) of `bench.py --mark-region 1`: every
kernel between the two torch.cuda._sleep markers that bracket the region, start / end in us relative to the first
marker's end, and the gaps -- where the window's wall clock goes besides the kernels.  With a HIP runtime trace
(`--hip-runtime-trace`, *hip_api_trace.csv) also the API calls of the region (graph launch, event records,
synchronize).  Also the back-to-back period of the graph replays that follow (steady_state): rollout start to
rollout start.

usage: python tools/trace_window.py <kernel_trace.csv> [<hip_api_trace.csv>]"""
import csv
import sys


def short(name):
    for k in ("mgx_rollout_kernel", "mgx_refill", "mgx_mt_slide", "mgx_gae_kernel", "mgx_gae_reduce", "spin_kernel", "sleep",
              "random", "distribution", "mgx_step_kernel", "mgx_gather"):
        if k in name:
            return k
    return name[:40]


def main():
    ks = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if "spin_kernel" in k[2] or "sleep" in k[2].lower()]
    if len(marks) < 2:
        sys.exit("no marker pair (bench.py --mark-region 1)")
    # the region: between the first marker pair whose interval holds a rollout or step kernel
    for a, b in zip(marks, marks[1:]):
        inner = ks[a + 1:b]
        if any("mgx_rollout" in k[2] or "mgx_step" in k[2] for k in inner):
            break
    else:
        sys.exit("no region between markers")
    t0 = ks[a][1]
    print("region: %d kernels; first start %+.1f us after the marker; last end %.1f us; next marker %.1f us"
          % (len(inner), (inner[0][0] - t0) / 1e3, (max(k[1] for k in inner) - t0) / 1e3, (ks[b][0] - t0) / 1e3))
    for s, e, n in inner:
        print("  %-22s %8.1f .. %8.1f  (%7.1f us)" % (short(n), (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
    if len(sys.argv) > 2:
        api = []
        with open(sys.argv[2]) as f:
            for r in csv.DictReader(f):
                api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function") or r.get("Kernel_Name", "")))
        api.sort()
        t_lo, t_hi = ks[a][0], ks[b][1]
        print("HIP API calls between the markers' starts:")
        for s, e, n in api:
            if t_lo <= s <= t_hi:
                print("  %-34s %8.1f .. %8.1f  (%6.1f us)" % (n[:34], (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
    # back-to-back replays after the region (steady_state): period between rollout starts
    roll = [k for k in ks[b:] if "mgx_rollout" in k[2]]
    per = [(y[0] - x[0]) / 1e3 for x, y in zip(roll, roll[1:])]
    if per:
        per.sort()
        print("rollout-to-rollout period after the region: %d periods, median %.1f us, p10 %.1f, p90 %.1f"
              % (len(per), per[len(per) // 2], per[len(per) // 10], per[9 * len(per) // 10]))


if __name__ == "__main__":
    main()
