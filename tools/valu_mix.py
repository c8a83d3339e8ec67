"""Cycle-weighted VALU mix of the config-3 scan kernel's hot block (for the
bench line's roofline.valu).

Compiles csrc/scan.hip for gfx950 with -save-temps (the Makefile's flags) in a
temp dir, takes the scan_kernel<0, 0, 1> function (FracMinHash, flavour B,
low-bits pre-filter: config 3), splits it into basic blocks and picks the block
with the most VALU instructions — the clean-wave window loop (one window per
lane per iteration).  Each VALU op is priced with the measured wave64 issue
cost per SIMD of profiles/r01/isa_rates_microbench.txt (cycles at 2.4 GHz):
ops measured there take their own figure; an unmeasured op takes the figure
of its encoding class (VOP3 / 64-bit / multiply ~4.2, VOP2 / VOP1 ~2.2).
Writes JSON: the hot block's VALU count, cycles, mean cycles per VALU, the
source hash of the scan files, and the per-op table.

    python tools/valu_mix.py [out.json]"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spaced-kmer-sketching_amd")
sys.path.insert(0, PKG)
import srchash  # noqa: E402

KERNEL = "_ZN3sks12_GLOBAL__N_111scan_kernelILi0ELi0ELi1EEEvNS_10ScanParamsE"
RATES = os.path.join(ROOT, "profiles", "r01", "isa_rates_microbench.txt")


def measured_rates():
    out = {}
    for line in open(RATES):
        m = re.match(r"(v_\w+)\s+[\d.]+ ms.*cycles@2\.4GHz=([\d.]+)\)", line)
        if m:
            out[m.group(1)] = float(m.group(2))
    return out


def price(op, enc64, rates):
    if op.startswith("v_cndmask_b32"):
        # the microbench's 22.9 cycles is a chain through VCC (each select waits
        # for the previous compare); a select fed by an independent compare issues
        # like any VOP2 / VOP3 op
        return (rates.get("v_and_b32", 2.25), "class (VOP2 cndmask)") if not enc64 else \
            (rates.get("v_mad_u64_u32", 4.27), "class (VOP3 cndmask)")
    if op in rates:
        return rates[op], "measured"
    base = re.sub(r"_e(32|64)$", "", op)
    if base in rates:
        return rates[base], "measured"
    cheap = rates.get("v_xor_b32", 2.35)
    dear = rates.get("v_mad_u64_u32", 4.27)
    if enc64 or any(t in base for t in ("_u64", "_b64", "_i64", "mul", "mad", "align", "perm", "bfe", "bfi",
                                        "lshl_add", "lshl_or", "add3", "or3", "xad", "cmp", "lshlrev", "lshrrev",
                                        "ashrrev", "readlane", "writelane", "mbcnt")):
        return dear, "class (VOP3 / 64-bit / multiply)"
    return cheap, "class (VOP1 / VOP2)"


def main(dst=None):
    rates = measured_rates()
    with tempfile.TemporaryDirectory() as td:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-I", os.path.join(ROOT, "include"), "-save-temps", "-c",
                        os.path.join(PKG, "csrc", "scan.hip"), "-o", os.path.join(td, "scan.o")],
                       cwd=td, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        s = [f for f in os.listdir(td) if f.endswith(".s") and "gfx950" in f][0]
        text = open(os.path.join(td, s)).read()
    a = text.index(KERNEL + ":")
    b = text.index(".Lfunc_end", a)
    blocks, cur, full, fcur = [], [], [], []
    for line in text[a:b].splitlines():
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", line):
            blocks.append(cur)
            full.append(fcur)
            cur, fcur = [], [line.strip()]
            continue
        t = line.strip()
        if t.startswith("v_"):
            cur.append(t)
        if t and not t.startswith((";", ".")):
            fcur.append(t)
    blocks.append(cur)
    full.append(fcur)
    hot_i = max(range(len(blocks)), key=lambda i: len(blocks[i]))
    hot = blocks[hot_i]
    if os.environ.get("SKS_VALU_LISTING"):  # the hot block's whole instruction text
        open(os.environ["SKS_VALU_LISTING"], "w").write("\n".join(full[hot_i]) + "\n")
    table, cycles = {}, 0.0
    for ins in hot:
        op = ins.split()[0]
        c, how = price(op, op.endswith("_e64") or "," in ins and ins.count("v[") > 1, rates)
        cycles += c
        e = table.setdefault(op, {"count": 0, "cycles_each": c, "priced_by": how})
        e["count"] += 1
    out = {"kernel": "scan_kernel<0, 0, 1>", "hot_block_valu": len(hot), "hot_block_cycles": cycles,
           "mean_cycles_per_valu": cycles / len(hot),
           "cycles_unit": "wave64 issue cycles per SIMD (profiles/r01/isa_rates_microbench.txt, 2.4 GHz)",
           "windows_per_hot_block_iteration_per_lane": 1,
           "scan_source_hash": srchash.scan_hash(), "ops": dict(sorted(table.items(), key=lambda x: -x[1]["count"]))}
    js = json.dumps(out, indent=1)
    if dst:
        open(dst, "w").write(js)
    print(js)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else None)
