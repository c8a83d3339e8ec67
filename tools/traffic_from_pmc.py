"""Turn a round profile (tools/profile_round.sh) into committed summaries:
profiles/<tag>/kernel_stats.csv (rocprofv3 --stats, trimmed) and
profiles/<tag>/traffic.json (HBM bytes per scan launch from PMC: FETCH_SIZE x 2
per the gfx950 correction + WRITE_SIZE, both in KiB units)."""
import csv
import json
import os
import sys


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r["Name"][:160], r["Calls"], r["TotalDurationNs"], r["AverageNs"],
                        r["Percentage"], r["MinNs"], r["MaxNs"]])

    def avg(path, counter, pattern):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
                if r["Counter_Name"] == counter and pattern in r["Kernel_Name"]]
        return sum(vals) / len(vals) if vals else None

    pat = "scan_kernel<0, 0, 1>"  # FracMinHash, flavour B, low-bits pre-filter
    fetch = avg(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE", pat)
    write = avg(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE", pat)
    scan = [r for r in rows if pat in r["Name"]]
    out = {
        "kernel": "scan_kernel<frac, boost-mix, pre-filter> (config 3 step)",
        "fetch_size_kib": fetch, "write_size_kib": write,
        "scan_hbm_bytes_per_launch": (2 * fetch + write) * 1024 if fetch and write else None,
        "correction": "FETCH_SIZE x 2 (gfx950 counts 128-B requests at 64 B, MI355X_MICROARCH.md HBM)",
        "trace_avg_ns": float(scan[0]["AverageNs"]) if scan else None,
    }
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
