"""Per-epoch kernel timeline of a fused-rollout bench from a rocprofv3 kernel trace (csv): for each epoch
(one mgx_rollout_kernel launch) the rollout and refill durations, when the refill started and ended relative
to the rollout, and the epoch period (rollout start to the next rollout start).  Medians over the last
`--last` epochs (the timed region's steady state).

usage: python tools/epoch_timeline.py <kernel_trace.csv> [--last 48]"""
import csv
import statistics as st
import sys


def main():
    path = sys.argv[1]
    last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 48
    ks = []
    with open(path) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    roll = [k for k in ks if "mgx_rollout_kernel" in k[2]]
    refill = [k for k in ks if "refill" in k[2]]
    slide = [k for k in ks if "mt_slide" in k[2]]
    rows = []
    for i in range(len(roll) - 1):
        r0, r1 = roll[i], roll[i + 1]
        # the refill forked with this rollout: the first refill starting after the previous rollout began
        cand = [k for k in refill if k[0] >= r0[0] - 50_000 and k[0] < r1[0]]
        if not cand:
            continue
        f = cand[0]
        sl = [k for k in slide if k[0] >= f[1] and k[0] < r1[0] + 1_000_000]
        dep = max(r0[1], sl[0][1] if sl else f[1])           # the next rollout's last dependency (join)
        rows.append(dict(start_after_dep=(r1[0] - dep) / 1e3, start_after_rollout=(r1[0] - r0[1]) / 1e3,period=(r1[0] - r0[0]) / 1e3, rollout=(r0[1] - r0[0]) / 1e3, refill=(f[1] - f[0]) / 1e3,
                         refill_start=(f[0] - r0[0]) / 1e3, refill_end=(f[1] - r0[0]) / 1e3,
                         rollout_end=(r0[1] - r0[0]) / 1e3,
                         slide=((sl[0][1] - sl[0][0]) / 1e3) if sl else None,
                         gap_after_refill=(r1[0] - f[1]) / 1e3))
    rows = rows[-last:]
    # every kernel of one steady-state epoch, relative to its rollout's start
    if len(roll) > 4:
        r0, r1 = roll[-4], roll[-3]
        print("epoch sample:", [(k[2].split("(")[0][-40:], round((k[0] - r0[0]) / 1e3, 1), round((k[1] - r0[0]) / 1e3, 1))
                                for k in ks if r0[0] - 20_000 <= k[0] < r1[0] + 5_000])
    out = {k: round(st.median([r[k] for r in rows if r[k] is not None]), 2) for k in rows[0]}
    out["epochs"] = len(rows)
    out["unit"] = "us (median; refill_start / refill_end / rollout_end relative to the rollout's start)"
    print(out)


if __name__ == "__main__":
    main()
