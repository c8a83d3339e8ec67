"""Summarize rocprofv3 --pmc CSVs per kernel (average per dispatch)."""
import collections
import csv
import glob
import os
import sys


def main(d, pattern=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if pattern and pattern not in name:
                continue
            short = name.split("(")[0][-60:]
            agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[short].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for k, cs in agg.items():
        print(f"== {k}  (avg dispatch {sum(dur[k]) / len(dur[k]):.3f} ms, profiled)")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v) / len(v):16.4g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
