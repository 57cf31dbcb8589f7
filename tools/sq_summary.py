"""SQ counters of one kernel from rocprofv3 --pmc passes (csv): per launch and per wave (SQ_WAVES), the
first quarter of the launches dropped as warm-up, plus fractions of SQ_WAVE_CYCLES for the WAIT / ACTIVE
buckets (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES, MI355X_MICROARCH.md).

  python tools/sq_summary.py KERNEL_SUBSTR OUT.json PASS1.csv [PASS2.csv ...]"""
import collections
import csv
import json
import sys


def main():
    kernel, out = sys.argv[1], sys.argv[2]
    acc = {}
    nl = {}
    for path in sys.argv[3:]:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(path)):
            if kernel in r["Kernel_Name"]:
                per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
        ids = sorted(per)[len(per) // 4:]
        for c in {c for i in ids for c in per[i]}:
            acc[c] = sum(per[i][c] for i in ids) / len(ids)
            nl[c] = len(ids)
    waves = acc.get("SQ_WAVES")
    d = {"kernel": kernel, "per_launch": acc, "launches": nl}
    if waves:
        d["per_wave"] = {k: v / waves for k, v in acc.items()}
    cyc = acc.get("SQ_WAVE_CYCLES")
    if cyc:
        d["fractions_of_wave_cycles"] = {k: v / cyc for k, v in acc.items() if k.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps({k: d[k] for k in ("fractions_of_wave_cycles",) if k in d}))


if __name__ == "__main__":
    main()
