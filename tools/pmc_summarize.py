"""Average per-launch HBM bytes of mgx_step_kernel from two rocprofv3 --pmc CSVs."""
import collections, csv, json, sys


def per_dispatch(path, counter):
    vals = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


KERNEL = sys.argv[3] if len(sys.argv) > 3 else "mgx_step_kernel"
f = per_dispatch(sys.argv[1], "FETCH_SIZE")     # KB
w = per_dispatch(sys.argv[2], "WRITE_SIZE")     # KB
f, w = f[len(f) // 4:], w[len(w) // 4:]          # drop warm-up launches
fetch = 2.0 * 1024.0 * sum(f) / len(f)           # gfx950: FETCH_SIZE counts half of wide reads
write = 1024.0 * sum(w) / len(w)
print(json.dumps({"kernel": KERNEL, "n_envs": 65536, "size": 8, "mission": 5,
                  "launches": [len(f), len(w)], "fetch_bytes_per_launch": fetch,
                  "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
                  "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE | WRITE_SIZE (separate passes); "
                            "FETCH_SIZE x2 (gfx950), KB units"}))
