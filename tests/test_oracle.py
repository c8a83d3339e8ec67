"""CPU: pin the oracle (oracle/sks_oracle.cpp) against the golden fixtures.

The fixtures come from the reference's own fasta_processing.cpp /
ani_estimation.cpp (compiled in oracle/_ref), SURVEY Appendix A masks, the
reference README's known answers, and (for k-mer sets) the restatement itself
cross-checked against the reference-faithful port oracle/ref_port.cpp.
"""
import os

import numpy as np
import pytest

import pyoracle as O
import synth

GOLDEN_FASTA = os.path.join(os.path.dirname(__file__), "golden", "fasta")


def test_fasta_records_and_runs_match_reference(golden):
    g = golden("fasta_cases.json")
    assert g["cases"], "empty fixture"
    for name, want in g["cases"].items():
        p = os.path.join(GOLDEN_FASTA, name)
        assert [r.hex() for r in O.fasta_records(p)] == want["records"], name
        assert [r.hex() for r in O.fasta_runs(p)] == want["runs"], name


def test_ani_matches_reference(golden):
    for case in golden("ani_cases.json")["cases"]:
        if "inter" in case:
            c = O.containment(case["inter"], case["size"])
            assert c.hex() == case["containment"]
            assert O.binomial_estimator(c, case["k"]).hex() == case["ani"]
        else:
            c = float.fromhex(case["containment_in"])
            assert O.binomial_estimator(c, case["k"]).hex() == case["ani"]


def test_masks(golden):
    for m in golden("masks.json"):
        assert O.mask(m["w"], m["k"], m["seed"]) == int(m["mask"], 16), m


def _decode_masked(value, w, mask):
    """Bases kept by `mask` in window order oldest -> newest (bit pair j = w-1-p)."""
    out = []
    for p in range(w):
        j = w - 1 - p
        if (mask >> (2 * j)) & 3:
            out.append("ACGT"[(value >> (2 * j)) & 3])
    return "".join(out)


def test_readme_kats(golden):
    kats = golden("readme_kats.json")
    seq = kats["kmers5"]["seq"].encode()
    runs = O.cut_runs(seq)
    rows = O.windows(runs, 5, O.mask(5, 5, 0))
    fwd = [_decode_masked(int(r[0]) | int(r[1]) << 64, 5, O.mask(5, 5, 0)) for r in rows]
    assert fwd == kats["kmers5"]["expect"]
    sp = kats["spaced"]
    seed = sp["seed_oldest_to_newest"]
    w = len(seed)
    mask = 0
    for p, ch in enumerate(seed):
        if ch == "1":
            mask |= 3 << (2 * (w - 1 - p))
    rows = O.windows(O.cut_runs(sp["seq"].encode()), w, mask)
    F = int(rows[sp["window_start"]][0]) | int(rows[sp["window_start"]][1]) << 64
    assert _decode_masked(F & mask, w, mask) == sp["expect"]


def test_c1_fixture_consistent(golden):
    g = golden("c1_sketch.json")
    runs = O.fasta_runs(os.path.join(GOLDEN_FASTA, g["file"]))
    for case in g["cases"][::3]:
        m = int(case["mask"], 16)
        sk, nw = O.sketch(runs, case["w"], m, case["kind"], case["param"], case["nonce"],
                          case["flavour"])
        assert nw == case["windows"]
        assert [hex(int(lo) | int(hi) << 64) for lo, hi in sk] == case["sketch"]


def test_refport_matches_oracle_spaced_and_wide():
    rng = np.random.default_rng(3)
    seq = synth.bases(60000, seed=11)
    seq[rng.integers(0, len(seq), 40)] = ord("N")
    runs = O.cut_runs(seq.tobytes())
    for (w, k) in [(31, 21), (40, 30), (64, 64), (1, 1), (17, 9)]:
        m = O.mask(w, k, 5)
        for flavour in (0, 1):
            want, _ = O.sketch(runs, w, m, "frac", 50, 1, flavour)
            got = O.refport_sketch_runs(runs, w, m, 50, 1, flavour).elems()
            assert np.array_equal(want, got), (w, k, flavour)


def test_refport_bottom_s_matches_oracle():
    """The reference-style bottom-s port (the CPU baseline of the bottom-s
    configs) keeps the same set as the oracle's bottom-s definition."""
    seq = synth.bases(40000, seed=13)
    seq[1000:1030] = ord("N")
    runs = O.cut_runs(seq.tobytes())
    codes = np.frombuffer(b"".join(runs), dtype=np.uint8)
    lens = np.array([len(r) for r in runs], dtype=np.uint64)
    assert O.refport_bottom_codes(codes, lens, 31, O.mask(31, 21, 2), 0).size() == 0
    for (w, k, s) in [(31, 21, 300), (21, 21, 1), (40, 30, 500), (31, 21, 100000)]:
        m = O.mask(w, k, 2)
        for flavour in (0, 1):
            want, _ = O.sketch(runs, w, m, "bottom", s, 1, flavour)
            got = O.refport_bottom_codes(codes, lens, w, m, s, 1, flavour).elems()
            assert np.array_equal(want, got), (w, k, s, flavour)


def test_refport_intersection_matches_merge():
    runs_a = O.cut_runs(synth.bases(30000, seed=21).tobytes())
    runs_b = O.cut_runs(synth.bases(30000, seed=21, mut_seed=5, mut_rate=0.01).tobytes())
    m = O.mask(21, 21, 0)
    sa, _ = O.sketch(runs_a, 21, m, "frac", 20)
    sb, _ = O.sketch(runs_b, 21, m, "frac", 20)
    pa = O.refport_sketch_runs(runs_a, 21, m, 20)
    pb = O.refport_sketch_runs(runs_b, 21, m, 20)
    mat = O.refport_all_pairs([pa, pb], threads=2)
    assert mat[0, 1] == mat[1, 0] == O.intersect(sa, sb) > 0
    assert mat[0, 0] == len(sa) and mat[1, 1] == len(sb)


M64 = (1 << 64) - 1


def _py_mix(x):  # boost hash_mix_impl<64> (Boost >= 1.81)
    x ^= x >> 32
    x = (x * 0x0E9846AF9B1A615D) & M64
    x ^= x >> 32
    x = (x * 0x0E9846AF9B1A615D) & M64
    return x ^ (x >> 28)


def _py_combine(s, v, flavour):
    if flavour == 0:
        return _py_mix((s + 0x9E3779B9 + v) & M64)
    m = 0xC6A4A7935BD1E995  # Boost 1.71-1.80 hash_combine_impl
    v = (v * m) & M64
    v ^= v >> 47
    v = (v * m) & M64
    s ^= v
    s = (s * m) & M64
    return (s + 0xE6546B64) & M64


def test_hash_matches_pure_python_restatement():
    rng = np.random.default_rng(9)
    for flavour in (0, 1):
        for _ in range(200):
            lo, hi = (int(x) for x in rng.integers(0, 2**63, 2, dtype=np.uint64))
            want = _py_combine(128, _py_combine(_py_combine(0, lo, flavour), hi, flavour), flavour)
            assert O.hash_bitset128(lo | hi << 64, flavour) == want
    m = O.mask(21, 21, 0)
    h0 = O.frac_min_hash(0x123456789, m, 21, 1, 0)
    assert h0 == (O.hash_bitset128(0x123456789, 0) ^ O.hash_bitset128(m, 0) ^ 21 ^ 1)
    assert h0 != O.frac_min_hash(0x123456789, m, 21, 1, 1)


@pytest.mark.parametrize("w", [1, 2, 7, 31, 32, 33, 64])
def test_window_counts(w):
    seq = synth.bases(5000, seed=2)
    seq[100:105] = ord("n")
    runs = O.cut_runs(seq.tobytes())
    _, nw = O.sketch(runs, w, O.mask(w, w, 0), "frac", 1)
    assert nw == sum(max(0, len(r) - w + 1) for r in runs)
