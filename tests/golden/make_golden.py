"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for oracle/_ref):
    python tests/golden/make_golden.py

Sources of truth, per fixture file:
  fasta_cases.json  records + ACGT runs of every file in tests/golden/fasta/,
                    produced by the REFERENCE's own fasta_processing.cpp
                    (compiled into oracle/_ref/, see oracle/Makefile).
  ani_cases.json    containment / binomial_estimator doubles from the
                    REFERENCE's own ani_estimation.cpp (oracle/_ref/).
  masks.json        generate_random_spaced_seed_mask(w, k, seed): the values
                    recorded in SURVEY.md Appendix A (libstdc++ std::shuffle +
                    std::mt19937, what kmer_bitset.cpp:132-152 calls) plus the
                    (w, k) sweep of kmer-sketching.cpp:219-239, from libstdc++.
  readme_kats.json  the two known-answer examples of the reference README.
  c1_sketch.json    config 1 (10 kb, w=k=21 contiguous) and a spaced variant:
                    canonical k-mer sets from the oracle's restatement of
                    kmer_sliding.cpp (RESTATEMENT-PINNED; the Boost hash is an
                    assumption, both flavours recorded), cross-checked against
                    the reference-faithful port oracle/ref_port.cpp.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
import synth  # noqa: E402

FASTA_DIR = os.path.join(HERE, "fasta")

# Edge-case corpus (fasta_processing.cpp:79-198 record rules).
CASES = {
    "probe.fa": b"junk\nACGT\n>r1 desc\nACGTn\nacgtNNgg\n\nTTTT\n>r2\nAC GT\nGGGG\n>r3\r\nACG\r\nTTA\r\n>r4\n>r5\nCC\n",
    "empty.fa": b"",
    "only_header.fa": b">only\n",
    "bare_gt.fa": b">\nACGTACGT\n>named\nGGGG\n",
    "no_trailing_newline.fa": b">a\nACGTACGTAC\nGTAC",
    "crlf.fa": b">a\r\nACGTACGTACGTACGTACGTACGTA\r\nCCGGTTAACCGGTTAACCGGTTAAC\r\n",
    "blank_lines.fa": b">a\nACGTACGTACGT\n\nGGGGCCCCAAAA\n\n\n>b\nTTTT\n",
    "space_mid.fa": b">a\nACGTACGT\nACG TACGT\nACGTACGT\n>b\nCCCCGGGG\n",
    "iupac.fa": b">a\nACGTRYKMSWBDHVNacgtrykmswbdhvn\nACGTU-.*ACGT\n",
    "lowercase.fa": b">a\nacgtacgtacgtacgtacgtacgtacgtacgtacgt\nACGTACGTACGTACGTACGTACGT\n",
    "comment.fa": b">a\n;comment line\nACGTACGTACGTACGTACGTACGTAAAA\n",
    "tabs.fa": b">a\tdesc\nACGT\tACGT\nACGTACGTACGTACGTACGTACGTACGT\n",
    "header_space_ok.fa": b">seq one two\nACGTACGTACGTACGTACGTACGTACGTACGTACGTACGT\n",
}


def hexs(bs):
    return [b.hex() for b in bs]


def make_c1():
    rng_seq = synth.bases(10000, seed=1)
    text = synth.fasta_text([("syn_c1_0", rng_seq)])
    path = os.path.join(FASTA_DIR, "c1_10kb.fa")
    with open(path, "wb") as f:
        f.write(text)
    runs = O.ref_fasta_runs(path)
    assert runs == O.fasta_runs(path)
    out = {"file": "c1_10kb.fa", "windows": None, "cases": []}
    for (w, k, seed) in [(21, 21, 0), (31, 21, 0), (10, 10, 0), (20, 10, 0)]:
        m = O.mask(w, k, seed)
        for flavour in (0, 1):
            for kind, param in (("frac", 200), ("frac", 1000), ("frac", 8), ("bottom", 100)):
                sk, nw = O.sketch(runs, w, m, kind, param, 1, flavour)
                if kind == "frac":
                    rp = O.refport_sketch_runs(runs, w, m, param, 1, flavour).elems()
                    assert np.array_equal(rp, sk), (w, k, flavour, param)
                out["cases"].append({
                    "w": w, "k": k, "mask_seed": seed, "mask": hex(m), "flavour": flavour,
                    "kind": kind, "param": param, "nonce": 1, "windows": nw,
                    "sketch": [hex(int(lo) | (int(hi) << 64)) for lo, hi in sk],
                })
        out["windows"] = nw
    # per-window dump of the first 40 windows, contiguous 21-mer, flavour 0 and 1
    m = O.mask(21, 21, 0)
    for flavour in (0, 1):
        rows = O.windows(runs, 21, m, 1, flavour)[:40]
        out.setdefault("window_dump", {})[str(flavour)] = [
            {"F": hex(int(r[0]) | int(r[1]) << 64), "R": hex(int(r[2]) | int(r[3]) << 64),
             "C": hex(int(r[4]) | int(r[5]) << 64), "H": hex(int(r[6])), "fmh": hex(int(r[7]))}
            for r in rows]
    return out


def main():
    if not O.ref_available():
        sys.exit("oracle/_ref/libref_fasta_ani.so missing: run `make -C oracle` with /root/reference present")
    os.makedirs(FASTA_DIR, exist_ok=True)
    fasta = {}
    for name, data in CASES.items():
        p = os.path.join(FASTA_DIR, name)
        with open(p, "wb") as f:
            f.write(data)
        recs = O.ref_fasta_records(p)
        runs = O.ref_fasta_runs(p)
        # the restatement must agree before anything is frozen
        assert recs == O.fasta_records(p), name
        assert runs == O.fasta_runs(p), name
        fasta[name] = {"records": hexs(recs), "runs": hexs(runs)}
    with open(os.path.join(HERE, "fasta_cases.json"), "w") as f:
        json.dump({"source": "reference src/fasta_processing.cpp via oracle/_ref", "cases": fasta},
                  f, indent=1, sort_keys=True)

    ani = []
    for k in (1, 10, 11, 21, 31, 40, 64):
        for size in (1, 7, 100, 10000, 2147483647):
            for inter in (0, 1, 3, 50, 99, 100, 9999, 10000):
                c = O.ref().refx_containment(inter, size)
                a = O.ref().refx_binomial_estimator(c, k)
                assert c == O.containment(inter, size) and a == O.binomial_estimator(c, k)
                ani.append({"inter": inter, "size": size, "k": k, "containment": c.hex(),
                            "ani": a.hex()})
    for c in (-1.0, 0.0, 1e-300, 0.5, 1.0, 1.5):
        for k in (1, 21):
            a = O.ref().refx_binomial_estimator(c, k)
            ani.append({"containment_in": c.hex(), "k": k, "ani": a.hex()})
    with open(os.path.join(HERE, "ani_cases.json"), "w") as f:
        json.dump({"source": "reference src/ani_estimation.cpp via oracle/_ref", "cases": ani}, f,
                  indent=1)

    appendix_a = [(31, 21, 0, 0x03ff3ccfff3c33f3), (31, 21, 1, 0x3c0fff03ffc3fff0),
                  (31, 21, 2, 0x3ffcfc3333c0fcff), (31, 21, 3, 0x33f3ffc3f3fc0f0f),
                  (31, 21, 4, 0x3ff3ffcc0cfff033), (31, 21, 5, 0x3ccf33cfff3fc33c),
                  (31, 21, 6, 0x3f3fc3c3ff03cfcf), (31, 21, 7, 0x3f3fff0ffff0003f),
                  (10, 10, 0, 0x00000000000fffff), (21, 21, 0, 0x000003ffffffffff),
                  (20, 10, 0, 0x0000000f0cfc330f)]
    masks = [{"w": w, "k": k, "seed": s, "mask": hex(v), "source": "SURVEY.md Appendix A"}
             for (w, k, s, v) in appendix_a]
    for (w, k, s, v) in appendix_a:
        assert O.mask(w, k, s) == v
    sweep = [(10, 10)] + [(k, k) for k in range(11, 41)] + [(k + 10, k) for k in range(10, 41)]
    for (w, k) in sweep + [(64, 64), (64, 40), (50, 40), (33, 21), (1, 1), (5, 0)]:
        masks.append({"w": w, "k": k, "seed": 0, "mask": hex(O.mask(w, k, 0)),
                      "source": "libstdc++ (GCC 11.4) shuffle, kmer-sketching.cpp:219-239 sweep"})
    with open(os.path.join(HERE, "masks.json"), "w") as f:
        json.dump(masks, f, indent=1)

    kats = {
        "source": "reference README.md:8-18 and :25-41",
        "kmers5": {"seq": "ACCGTAAATTCGA",
                   "expect": ["ACCGT", "CCGTA", "CGTAA", "GTAAA", "TAAAT", "AAATT", "AATTC",
                              "ATTCG", "TTCGA"]},
        "spaced": {"seq": "AAACGTACGTTT", "window_start": 2, "seed_oldest_to_newest": "11001011",
                   "expect": "ACAGT"},
    }
    with open(os.path.join(HERE, "readme_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    c1 = make_c1()
    with open(os.path.join(HERE, "c1_sketch.json"), "w") as f:
        json.dump(c1, f, indent=1)
    print("golden fixtures written:", len(fasta), "fasta cases,", len(ani), "ani cases,",
          len(masks), "masks,", len(c1["cases"]), "c1 sketch cases")


if __name__ == "__main__":
    main()
