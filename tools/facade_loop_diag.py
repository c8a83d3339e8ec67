import json, os, subprocess, sys, tempfile
sys.path[:0] = ["tests", "oracle"]
import synth
d = tempfile.mkdtemp()
files = []
for i in range(4):
    g = synth.bases(30000, seed=77, mut_seed=500 + i, mut_rate=0.01 * i)
    if i == 3:
        g[1000:1010] = ord("N")
    p = os.path.join(d, f"g{i}.fa")
    open(p, "wb").write(synth.fasta_text([(f"g{i}_a", g[:17000]), (f"g{i}_b", g[17000:])], width=70))
    files.append(p)
fails = 0
for it in range(40):
    r = subprocess.run(["tests/cpp/build/test_facade", "sketch", "31", "21", "0", "50", "frac"] + files,
                       capture_output=True, text=True, timeout=60)
    out = json.loads(r.stdout)
    if not out["serial_equal"]:
        fails += 1
        for i in range(4):
            a, b = out["sets"][i], out["serial_sets"][i]
            if a != b:
                sa, sb = set(a), set(b)
                print(it, "set", i, "sizes", len(a), len(b), "only_par", len(sa - sb), "only_ser", len(sb - sa),
                      "sample", sorted(sb - sa)[:3], flush=True)
print("fails", fails, "of 40")
