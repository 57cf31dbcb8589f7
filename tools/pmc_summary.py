"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc CSVs (FETCH_SIZE pass, WRITE_SIZE
pass), with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide
coalesced reads: doubled; WRITE_SIZE exact), the first quarter of launches dropped as warm-up.

The mean is what bench.py reports; the median and the per-launch lists are kept beside it because a
command that resets a second engine (the driver's command times both layouts) has a ring-filling
refill launch (~D episodes per env) among the kept launches, which moves the refill's mean but not
its median.

  python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR N_ENVS SIZE MISSION STEPS_PER_LAUNCH OUT.json
"""
import collections
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, kernel):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    fpath, wpath, kernel, n, size, mission, spl, out = sys.argv[1:9]
    f = [2.0 * 1024.0 * v for v in per_dispatch(fpath, "FETCH_SIZE", kernel)]
    w = [1024.0 * v for v in per_dispatch(wpath, "WRITE_SIZE", kernel)]
    f, w = f[len(f) // 4:], w[len(w) // 4:]
    fetch, write = sum(f) / len(f), sum(w) / len(w)
    d = {"kernel": kernel, "n_envs": int(n), "size": int(size), "mission": None if mission == "None" else int(mission),
         "steps_per_launch": int(spl), "launches": [len(f), len(w)], "fetch_bytes_per_launch": fetch,
         "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
         "fetch_bytes_median": statistics.median(f), "write_bytes_median": statistics.median(w),
         "fetch_bytes_by_launch": [round(v) for v in f], "write_bytes_by_launch": [round(v) for v in w],
         "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes); FETCH_SIZE x2 "
                   "(gfx950), KB units; first quarter of the launches dropped"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in d.items() if not k.endswith("_by_launch")}))


if __name__ == "__main__":
    main()
