"""The reference-named C++ facade (spaced-kmer-sketching_amd/cpp/*.hpp) driven
like the reference's own driver (kmer-sketching.cpp:151-212) by
tests/cpp/test_facade.cpp, compared with the oracle."""
import json
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_facade")


def build_facade_test():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)


@pytest.fixture(scope="module")
def facade_bin():
    if not os.path.exists(BIN):
        build_facade_test()
    return BIN


def test_facade_host_semantics(facade_bin):
    r = subprocess.run([facade_bin, "errors"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout)["errors_ok"] == 6


def test_facade_missing_file_exits_like_reference(facade_bin, tmp_path):
    missing = str(tmp_path / "nope.fa")
    r = subprocess.run([facade_bin, "missing", missing], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert r.stderr.startswith(f"Unable to open {missing}. \n Exiting...")


# SKS_FACADE_DEVICES: the parallel_* entry points spread files and pairs over a
# device pool; "0,0,0" gives three contexts on the one GPU of the test box, so
# the split / per-device build / merge in file order runs (kmer_set.cpp:112-133,
# 167-184) and must equal the serial entry points and the oracle
POOLS = [None, "0,0,0"]


def _env(pool):
    env = dict(os.environ)
    env.pop("SKS_FACADE_DEVICES", None)
    if pool:
        env["SKS_FACADE_DEVICES"] = pool
    return env


@pytest.mark.gpu
@pytest.mark.parametrize("pool", POOLS)
@pytest.mark.parametrize("w,k,seed,param,kind", [(21, 21, 0, 200, "frac"), (31, 21, 0, 50, "frac"),
                                                 (31, 21, 3, 300, "bottom"), (40, 30, 0, 40, "frac")])
def test_facade_sketch_and_ani(facade_bin, tmp_path, w, k, seed, param, kind, pool):
    files = []
    for i in range(4):
        g = synth.bases(30000, seed=77, mut_seed=500 + i, mut_rate=0.01 * i)
        if i == 3:
            g[1000:1010] = ord("N")
        p = tmp_path / f"g{i}.fa"
        p.write_bytes(synth.fasta_text([(f"g{i}_a", g[:17000]), (f"g{i}_b", g[17000:])], width=70))
        files.append(str(p))
    r = subprocess.run([facade_bin, "sketch", str(w), str(k), str(seed), str(param), kind] + files,
                       capture_output=True, text=True, timeout=300, env=_env(pool))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    m = O.mask(w, k, seed)
    assert int(out["mask"], 16) == m
    sk = []
    for i, f in enumerate(files):
        want, _ = O.sketch(O.fasta_runs(f), w, m, kind, param)
        got = [int(h, 16) for h in out["sets"][i]]
        assert got == [int(lo) | int(hi) << 64 for lo, hi in want], (i, w, kind)
        sk.append(want)
    n = len(files)
    inter = [O.intersect(sk[i], sk[j]) for i in range(n) for j in range(n)]
    assert out["inter"] == inter
    for flag in ("serial_equal", "inter_serial_equal", "runs_equal", "cut_equal"):
        assert out[flag], flag
    if pool:
        assert out["devices"] == 3
    assert out["single01"] == inter[1]
    kk = bin(m).count("1") // 2
    assert out["k"] == kk
    for p, (i, j) in enumerate([(i, j) for i in range(n) for j in range(n)]):
        c = O.containment(inter[p], len(sk[i]))
        assert float.fromhex(out["ani"][p]) == O.binomial_estimator(c, kk)


@pytest.mark.gpu
@pytest.mark.parametrize("pool", POOLS)
@pytest.mark.parametrize("w,k,param", [(31, 21, 10), (40, 30, 5)])
def test_facade_all_pairs_matrix_path(facade_bin, tmp_path, w, k, param, pool):
    """70 sets: the all-pairs list of generate_all_pairs_from_vector covers the
    whole matrix, so the facade counts it with the join (one layout of the 70
    sketches, each pool entry's share of the upper-triangle tiles, packed) and
    gathers; counts and ANI equal the oracle's."""
    files = []
    for i in range(70):
        g = synth.bases(3000, seed=900 + i % 5, mut_seed=950 + i, mut_rate=0.02 * (i % 3))
        p = tmp_path / f"h{i}.fa"
        p.write_bytes(synth.fasta_text([(f"h{i}", g)], width=60))
        files.append(str(p))
    r = subprocess.run([facade_bin, "sketch", str(w), str(k), "0", str(param), "frac"] + files,
                       capture_output=True, text=True, timeout=300, env=_env(pool))
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    m = O.mask(w, k, 0)
    sk = [O.sketch(O.fasta_runs(f), w, m, "frac", param)[0] for f in files]
    n = len(files)
    inter = [O.intersect(sk[i], sk[j]) for i in range(n) for j in range(n)]
    assert out["inter"] == inter
    assert out["inter_serial_equal"]
    if pool:
        assert out["devices"] == 3
    # the sketches crossed PCIe once (not once per pool entry), every pool entry
    # of the one device shared that copy (no device-to-device bytes), and only
    # the 3 upper-triangle 64 x 64 tiles came back (16 KB each)
    ps = out["pair_stats"]
    ew = 2 if any(int(x) for s_ in sk for x in (s_[:, 1] if s_.ndim == 2 else [])) else 1
    want_h2d = sum(len(s_) for s_ in sk) * 8 * ew + n * 8 + n * 4
    assert ps["calls"] == 1 and ps["h2d"] == want_h2d and ps["d2d"] == 0, ps
    assert ps["d2h"] == 3 * 64 * 64 * 4 and ps["devices"] == (3 if pool else 1), ps


REF_CALLER = os.path.join(ROOT, "tests", "cpp", "build", "ref_caller")


def _odd_rule(lo):
    return bin(int(lo)).count("1") % 2 == 0 and (int(lo) & 0xffffffff) % 3 == 1


@pytest.mark.gpu
@pytest.mark.parametrize("w,k,c,piece", [(31, 21, 200, 0), (21, 21, 50, 0), (40, 30, 20, 0), (31, 21, 200, 997),
                                         (64, 40, 20, 1500)])
def test_reference_shaped_caller_std_function(tmp_path, w, k, c, piece):
    """tests/cpp/ref_caller.cpp uses only the reference's API names and passes
    std::function predicates (a free function like kmer-sketching.cpp:29-34 and
    lambdas) to the builders, as kmer-sketching.cpp:151-212 does.  Sets, pair
    counts and ANI equal the oracle's; the predicate runs once per window; a
    rule no sketch descriptor can express selects exactly the oracle's windows;
    kmer_hashes iterates the set; k-mers of two masks in one set count per mask.
    piece > 0 cuts every stream into pieces of that many window starts
    (SKS_FACADE_PIECE): windows whose F register carries run history from
    before a cut keep it (the 64 bytes handed over in front of each piece)."""
    build_facade_test()
    files = []
    for i in range(3):
        g = synth.bases(25000, seed=81, mut_seed=600 + i, mut_rate=0.02 * i)
        g[3000:3020] = ord("N")
        p = tmp_path / f"r{i}.fa"
        p.write_bytes(synth.fasta_text([(f"r{i}_a", g[:11000]), (f"r{i}_b", g[11000:])], width=61))
        files.append(str(p))
    env = dict(os.environ)
    if piece:
        env["SKS_FACADE_PIECE"] = str(piece)
    r = subprocess.run([REF_CALLER, str(w), str(k), str(c)] + files, capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    m = O.mask(w, k, 0)
    assert int(out["mask"], 16) == m
    kk = bin(m).count("1") // 2
    assert out["k"] == kk
    runs = [O.fasta_runs(f) for f in files]
    sk, nws = [], []
    for i in range(3):
        want, nw = O.sketch(runs[i], w, m, "frac", c)
        assert [int(h, 16) for h in out["sets"][i]] == [int(lo) | int(hi) << 64 for lo, hi in want]
        sk.append(want)
        nws.append(nw)
    n = 3
    order = [(i, j) for i in range(n) for j in range(n)]
    inter = [O.intersect(sk[i], sk[j]) for i, j in order]
    assert out["inter"] == inter
    assert out["pairs"] == [[files[i], files[j]] for i, j in order]
    for p, (i, j) in enumerate(order):
        assert float.fromhex(out["ani"][p]) == O.binomial_estimator(O.containment(inter[p], len(sk[i])), kk)
    assert out["lambda_equal"]
    assert out["calls0"] == nws[0] and out["one_size"] == len(sk[0])
    every = O.kmer_list(runs[0], w, m, c=1)  # every window in order: kmer_bits lo, hi, masked lo, hi
    keep = np.array([_odd_rule(lo) and True for lo in every[:, 2]], dtype=bool) if len(every) else \
        np.zeros(0, bool)
    sel = every[keep]
    assert [[int(a, 16) for a in row] for row in out["list"]] == \
        [[int(r_[0]) | int(r_[1]) << 64, int(r_[2]) | int(r_[3]) << 64] for r_ in sel]
    custom = sorted({int(r_[2]) | int(r_[3]) << 64 for r_ in sel})
    assert [int(h, 16) for h in out["custom"]] == custom and len(custom) > 0
    m2 = O.mask(w, k, 5)
    assert int(out["mask2"], 16) == m2
    # w = k: both masks are all ones, so the second insert adds nothing new
    s2 = [O.sketch(runs[i], w, m2, "frac", c)[0] for i in range(2)] if m2 != m else \
        [np.zeros((0, 2), np.uint64)] * 2
    assert out["mixed_sizes"] == [len(sk[0]) + len(s2[0]), len(sk[1]) + len(s2[1])]
    both = O.intersect(sk[0], sk[1]) + O.intersect(s2[0], s2[1])
    assert out["mixed_inter"] == both
    # (mixed0, mixed1), (mixed1, data[1]): only the mask-m part is shared, (mixed0, mixed0)
    assert out["mixed_pairs"] == [both, len(sk[1]), len(sk[0]) + len(s2[0])]
