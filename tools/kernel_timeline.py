"""Per-kernel timeline from a rocprofv3 kernel-trace CSV.
    python tools/kernel_timeline.py <kernel_trace.csv>        the last call: the launches after the
                                                              last idle gap > 50 us, with each one's start
                                                              offset, duration and the gap before it
    python tools/kernel_timeline.py --all <kernel_trace.csv>  per-kernel totals over the whole trace,
                                                              then the last call's timeline"""
import collections
import csv
import sys


def main():
    args = sys.argv[1:]
    every = args[:1] == ["--all"]
    path = args[-1]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    if not rows:
        print("no kernels")
        return
    def name(r):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        return k.split("(")[0][-60:]
    if every:
        tot = collections.defaultdict(lambda: [0, 0])
        for r in rows:
            t = tot[name(r)]
            t[0] += 1
            t[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        busy = sum(t[1] for t in tot.values())
        span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
        print(f"{len(rows)} launches, kernels busy {busy / 1e6:.3f} ms of a {span / 1e6:.3f} ms span")
        for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
            print(f"{d / 1e6:9.3f} ms {c:6d} x {d / c / 1e3:8.1f} us  {k}")
        print()
    starts = [i for i in range(1, len(rows))
              if int(rows[i]["Start_Timestamp"]) - int(rows[i - 1]["End_Timestamp"]) > 50000]
    last = rows[starts[-1]:] if starts else rows
    t0 = pe = int(last[0]["Start_Timestamp"])
    for r in last:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} us dur {(e - s) / 1e3:7.1f} gap {(s - pe) / 1e3:6.1f}  {name(r)}")
        pe = e
    print(f"span {(pe - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
