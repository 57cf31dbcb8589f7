"""Per-dispatch durations of the step kernel from a rocprofv3 kernel trace of `bench.py`
(run_kernel_trace.csv): the launches in order are warm-up, the untimed graph replay, the timed
region, the probe (then the same for the SB3 layout).  Prints the average of the compact step
kernel over each phase, given the bench's K (steps), W (warm-up) and P (probe), and how many of the
timed launches ran while a refill launch was executing."""
import csv, sys, json

path, K, W, P = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
rows = list(csv.DictReader(open(path)))
step = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows
        if r["Kernel_Name"].startswith("void (anonymous namespace)::mgx_step_kernel<int, true>")]
refill = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "refill" in r["Kernel_Name"]]
step.sort()
def avg(a):
    return sum(e - s for s, e in a) / len(a) / 1e3 if a else None
warm, replay, timed, probe = step[:W], step[W:W + K], step[W + K:W + 2 * K], step[W + 2 * K:W + 2 * K + P]
def overlapped(a):
    n = 0
    for s, e in a:
        n += any(rs < e and re > s for rs, re in refill)
    return n
print(json.dumps(dict(launches=len(step), warmup_us=avg(warm), replay_us=avg(replay), timed_us=avg(timed),
                      probe_us=avg(probe), timed_beside_refill=overlapped(timed), timed_n=len(timed))))
