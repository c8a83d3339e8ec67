"""Summaries of a round profile (tools/profile_round.sh) for profiles/<tag>/:
  kernel_stats.csv          rocprofv3 --stats of the default bench command (trimmed)
  scan_timed_launches.json  the config-3 scan dispatches bench.py times (its serial
                            pass: dispatches [warmup, warmup + steps) of the kernel)
                            from the kernel trace: durations, median, mean, and the
                            bench line's own hipEvent kernel time of the same run
  traffic.json              HBM bytes per timed launch from PMC: FETCH_SIZE x 2 (the
                            gfx950 correction, MI355X_MICROARCH.md HBM) + WRITE_SIZE,
                            KiB units, median over the same dispatch indices, and the
                            scan kernel's source hash (srchash.scan_hash) it was measured on
  scan_counters.txt / pair_counters.txt   SQ counter averages per kernel
    python tools/summarize_round.py <round_dir> <dst> <warmup> <steps>"""
import csv
import glob
import io
import json
import os
import statistics
import sys
from contextlib import redirect_stdout

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import pmc_by_kernel  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "spaced-kmer-sketching_amd"))
import srchash  # noqa: E402

SCAN = "scan_kernel<0, 0, 1>"  # FracMinHash, flavour B, low-bits pre-filter (config 3)


def _one(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return f[0] if f else None


def _scan_dispatches(rows, key="Dispatch_Id"):
    out = [r for r in rows if SCAN in r["Kernel_Name"]]
    out.sort(key=lambda r: int(r[key]))
    return out


def _pmc_per_dispatch(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and SCAN in r["Kernel_Name"]:
            vals[int(r["Dispatch_Id"])] = vals.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def _pmc_kernel(d, kernel, counter):
    """Per-dispatch values (summed over the counter's dimensions) of `counter`
    for dispatches of `kernel` in the PMC passes under d."""
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                k = (f, int(r["Dispatch_Id"]))
                vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def _pmc_kernel_ms(d, kernel):
    ms = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                ms[(f, int(r["Dispatch_Id"]))] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return statistics.median(ms.values()) if ms else None


def main(src, dst, warmup, steps):
    os.makedirs(dst, exist_ok=True)
    stats = _one(os.path.join(src, "trace"), "*kernel_stats.csv")
    rows = list(csv.DictReader(open(stats)))
    with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in rows:
            w.writerow([r["Name"][:160], r["Calls"], r["TotalDurationNs"], r["AverageNs"],
                        r["Percentage"], r["MinNs"], r["MaxNs"]])
    trace = list(csv.DictReader(open(_one(os.path.join(src, "trace"), "*kernel_trace.csv"))))
    scans = _scan_dispatches(trace)
    timed = scans[warmup:warmup + steps]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
    bench_ms = None
    try:
        line = [l for l in open(os.path.join(src, "bench_traced.json")) if l.startswith("{")][-1]
        bench_ms = json.loads(line)["roofline"]["kernel_ms"]
    except (OSError, IndexError, KeyError, ValueError):
        pass
    launches = {"kernel": SCAN, "dispatches_of_kernel": len(scans), "timed_indices": [warmup, warmup + steps],
                "timed_ms": dur, "median_ms": statistics.median(dur), "mean_ms": statistics.mean(dur),
                "bench_line_hipevent_kernel_ms": bench_ms,
                "note": "rocprofv3 --kernel-trace of the default bench command; the timed launches "
                        "are the serial pass (after --warmup), the ones bench.py's roofline uses"}
    with open(os.path.join(dst, "scan_timed_launches.json"), "w") as f:
        json.dump(launches, f, indent=1)
    fetch = _pmc_per_dispatch(_one(os.path.join(src, "fetch"), "*counter_collection.csv"), "FETCH_SIZE")
    write = _pmc_per_dispatch(_one(os.path.join(src, "write"), "*counter_collection.csv"), "WRITE_SIZE")
    fetch_t, write_t = fetch[warmup:warmup + steps], write[warmup:warmup + steps]
    fk, wk = statistics.median(fetch_t), statistics.median(write_t)
    traffic = {"kernel": SCAN + " (config 3 step)", "timed_indices": [warmup, warmup + steps],
               "fetch_size_kib_median": fk, "write_size_kib_median": wk,
               "scan_hbm_bytes_per_launch": (2 * fk + wk) * 1024,
               "correction": "FETCH_SIZE x 2 (gfx950 counts 128-B requests at 64 B, MI355X_MICROARCH.md HBM)",
               "dispatches_seen": [len(fetch), len(write)],
               # bench.py reports this traffic only while the scan's sources hash the same
               "scan_source_hash": srchash.scan_hash()}
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1)
    for sub, name, kernels in (("sq", "scan_counters.txt", ["scan_kernel"]),
                               ("pairs", "pair_counters.txt", ["k_join", "k_bottom_fused", "k_gl_"])):
        if os.path.isdir(os.path.join(src, sub)):
            buf = io.StringIO()
            with redirect_stdout(buf):
                pmc_by_kernel.main(os.path.join(src, sub), kernels)
            open(os.path.join(dst, name), "w").write(buf.getvalue())
    # scan VALU issue (roofline.valu): counted VALU per launch, the hot block's mix
    sq = os.path.join(src, "sq")
    if os.path.isdir(sq):
        insts = _pmc_kernel(sq, SCAN, "SQ_INSTS_VALU")
        import valu_mix
        buf = io.StringIO()
        with redirect_stdout(buf):
            valu_mix.main(None)
        mix = json.loads(buf.getvalue())
        windows = None
        try:
            line = [l for l in open(os.path.join(src, "bench_traced.json")) if l.startswith("{")][-1]
            windows = json.loads(line)["config"]["windows_per_genome"]
        except (OSError, IndexError, KeyError, ValueError):
            pass
        # the hardware's own view: VALU instructions issued per SIMD per cycle
        # (SQ_ACTIVE_INST_VALU summed over the SIMDs; cycles from GRBM_GUI_ACTIVE,
        # summed over the 8 XCDs) — beside the priced-mix peak above
        act = _pmc_kernel(sq, SCAN, "SQ_ACTIVE_INST_VALU")
        grbm = _pmc_kernel(sq, SCAN, "GRBM_GUI_ACTIVE")
        cyc = statistics.median(grbm) / 8 if grbm else None
        hw = {"sq_active_inst_valu_per_launch": statistics.median(act) if act else None,
              "kernel_cycles_per_launch": cyc,
              "valu_inst_per_simd_cycle": (statistics.median(act) / (1024 * cyc)) if act and cyc else None}
        valu = {"kernel": SCAN, "sq_insts_valu_per_launch": statistics.median(insts) if insts else None,
                **hw,
                "windows_per_launch": windows,
                "valu_per_window": (64 * statistics.median(insts) / windows) if insts and windows else None,
                "hot_block_valu": mix["hot_block_valu"], "hot_block_cycles": mix["hot_block_cycles"],
                "mean_cycles_per_valu": mix["mean_cycles_per_valu"],
                "mean_ns_per_valu_per_simd": mix["mean_cycles_per_valu"] / 2.4,
                "rates": mix["cycles_unit"], "scan_source_hash": srchash.scan_hash()}
        with open(os.path.join(dst, "scan_valu.json"), "w") as f:
            json.dump(valu, f, indent=1)
    # k_join LDS counters per all-pairs call (pairs.roofline / pairs_wide.roofline in bench.py)
    for sub, out, what in (("pairs", "pair_lds.json", "k_join<1, ...> (config 4, 1000 x bottom-s 10000, w = 31, "
                                                      "tools/bench_pairs.py family)"),
                           ("pairs_wide", "pair_lds_wide.json", "k_join<2, ...> (config 4, 1000 x bottom-s 10000, "
                                                                "w = 45 / k = 30, tools/bench_pairs.py family 45)")):
        pr = os.path.join(src, sub)
        if not os.path.isdir(pr):
            continue
        lds = {"kernel": what, "join_source_hash": srchash.join_hash()}
        for c in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_SALU",
                  "SQ_WAVE_CYCLES", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES",
                  "GRBM_GUI_ACTIVE"):
            v = _pmc_kernel(pr, "k_join", c)
            lds[c.lower() + "_per_call"] = statistics.median(v) if v else None
        lds["profiled_ms"] = _pmc_kernel_ms(pr, "k_join")
        pm = os.path.join(src, "pairs_mem")
        if sub == "pairs" and os.path.isdir(pm):  # the memory side of the same call
            for c in ("FETCH_SIZE", "TCC_HIT_sum", "TCC_MISS_sum"):
                v = _pmc_kernel(pm, "k_join", c)
                lds[c.lower() + "_per_call"] = statistics.median(v) if v else None
            lds["fetch_size_note"] = ("FETCH_SIZE in KiB per call: L2-to-fabric read requests x 64 B (Infinity-Cache "
                                      "hits included; x2 for wide streaming reads on gfx950, MI355X_MICROARCH.md)")
        with open(os.path.join(dst, out), "w") as f:
            json.dump(lds, f, indent=1)
    print(json.dumps({"launches": {k: launches[k] for k in ("median_ms", "mean_ms", "bench_line_hipevent_kernel_ms")},
                      "traffic": traffic["scan_hbm_bytes_per_launch"]}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
