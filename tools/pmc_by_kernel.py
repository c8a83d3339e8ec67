"""Per-kernel averages of rocprofv3 --pmc CSVs (one dir per pass: <dir>/p*/).
    python tools/pmc_by_kernel.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import re
import sys


def main(d, names):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
            short = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
            if names and not any(x in short for x in names):
                continue
            agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, cs in agg.items():
        print(f"== {k}  (avg dispatch {sum(dur[k]) / len(dur[k]):.3f} ms, profiled)")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.4g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
