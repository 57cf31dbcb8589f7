"""Every fused-rollout epoch of a rocprofv3 kernel trace (csv), one line each: the rollout launch, the
refill forked with it and the MT slide after that refill, GAE (+ its stat fold) when the epoch ran one,
and the period to the next rollout -- times in us relative to the rollout's start.  For the driver's
`--steps 20` line the timed region is the graph replay whose epoch holds a GAE right after the untimed
replay (bench.py: warm-up epochs, one untimed replay of the graph, the timed replay, then the probe).

usage: python tools/trace_epochs.py <kernel_trace.csv>"""
import csv
import sys


def main():
    ks = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    ks.sort()
    roll = [k for k in ks if "mgx_rollout_kernel" in k[2]]
    for i, r0 in enumerate(roll):
        nxt = roll[i + 1][0] if i + 1 < len(roll) else r0[1] + 2_000_000
        win = [k for k in ks if r0[0] - 20_000 <= k[0] < nxt and k is not r0]
        def span(name):
            c = [k for k in win if name in k[2]]
            return "%s %.1f-%.1f" % (name, (c[0][0] - r0[0]) / 1e3, (c[0][1] - r0[0]) / 1e3) if c else ""
        parts = [span(n) for n in ("refill", "mt_slide", "gae_kernel", "gae_reduce")]
        print("epoch %3d rollout %.1f us | %s | period %.1f" % (i, (r0[1] - r0[0]) / 1e3, " | ".join(p for p in parts if p),
                                                             (nxt - r0[0]) / 1e3))


if __name__ == "__main__":
    main()
