"""Per-launch HBM bytes of one kernel from two rocprofv3 --pmc CSVs (FETCH_SIZE pass, WRITE_SIZE
pass), with the gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of wide
coalesced reads: doubled; WRITE_SIZE exact), the first quarter of launches dropped as warm-up.

  python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR N_ENVS SIZE MISSION STEPS_PER_LAUNCH OUT.json
"""
import collections
import csv
import json
import sys


def per_dispatch(path, counter, kernel):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    fpath, wpath, kernel, n, size, mission, spl, out = sys.argv[1:9]
    f = per_dispatch(fpath, "FETCH_SIZE", kernel)
    w = per_dispatch(wpath, "WRITE_SIZE", kernel)
    f, w = f[len(f) // 4:], w[len(w) // 4:]
    fetch = 2.0 * 1024.0 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    d = {"kernel": kernel, "n_envs": int(n), "size": int(size), "mission": None if mission == "None" else int(mission),
         "steps_per_launch": int(spl), "launches": [len(f), len(w)], "fetch_bytes_per_launch": fetch,
         "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
         "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes); FETCH_SIZE x2 "
                   "(gfx950), KB units; first quarter of the launches dropped"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
