"""CPU: the C-ABI library loads, exports every symbol include/sks.h declares,
and its host-side parts (ingress, masks, hash, ANI) match the golden fixtures.
No compute kernels run here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import pyoracle as O
import sksffi
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_FASTA = os.path.join(ROOT, "tests", "golden", "fasta")


def _declared_symbols():
    with open(os.path.join(ROOT, "include", "sks.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sks_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(sksffi.LIB_PATH)
    syms = _declared_symbols()
    assert len(syms) >= 35
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/sks.h but not exported"
    assert lib.sks_abi_version() == 3
    for s in sksffi.EXPORTED:
        assert s in syms


def test_masks_match_golden(golden):
    for m in golden("masks.json"):
        if m["k"] < 0:
            continue
        assert sksffi.mask_generate(m["w"], m["k"], m["seed"]) == int(m["mask"], 16), m


def test_mask_errors():
    for (w, k) in [(0, 0), (65, 10), (10, 11), (10, -1)]:
        with pytest.raises(sksffi.SksError) as e:
            sksffi.mask_generate(w, k, 0)
        assert e.value.code == 1
    assert sksffi.mask_contiguous(21) == 0x3FFFFFFFFFF
    assert sksffi.mask_contiguous(64) == (1 << 128) - 1
    with pytest.raises(sksffi.SksError, match="exceeds maximum k-mer length"):
        sksffi.mask_contiguous(65)


def test_frac_min_hash_matches_oracle():
    rng = np.random.default_rng(1)
    for w in (21, 31, 40, 64):
        m = O.mask(w, min(w, 21), 3)
        for flavour in (0, 1):
            for _ in range(50):
                v = int(rng.integers(0, 2**62)) | (int(rng.integers(0, 2**62)) << 64 if w > 32 else 0)
                v &= m
                assert sksffi.frac_min_hash(v, m, w, 1, flavour) == O.frac_min_hash(v, m, w, 1, flavour)
    # nonce is an int: negative values sign-extend (kmer.hpp:139-146)
    assert sksffi.frac_min_hash(5, 3, 1, -2, 0) == O.frac_min_hash(5, 3, 1, -2, 0)


def test_ani_matches_reference_doubles(golden):
    for case in golden("ani_cases.json")["cases"]:
        if "inter" in case:
            c = sksffi.containment(case["inter"], case["size"])
            assert c.hex() == case["containment"]
            assert sksffi.binomial_estimator(c, case["k"]).hex() == case["ani"]
        else:
            c = float.fromhex(case["containment_in"])
            assert sksffi.binomial_estimator(c, case["k"]).hex() == case["ani"]
    inter = np.array([0, 5, 10, 7], dtype=np.int32)
    size = np.array([10, 10, 10, 9], dtype=np.int32)
    cont, ani = sksffi.ani_from_counts(inter, size, 21)
    for i in range(4):
        assert cont[i] == O.containment(int(inter[i]), int(size[i]))
        assert ani[i] == O.binomial_estimator(cont[i], 21)


def test_fasta_ingress_matches_reference(golden):
    for name, want in golden("fasta_cases.json")["cases"].items():
        f = sksffi.Fasta(os.path.join(GOLDEN_FASTA, name))
        assert [r.hex() for r in f.records()] == want["records"], name
        assert [r.hex() for r in f.runs()] == want["runs"], name
        stream = f.stream().tobytes()
        assert stream == b"".join(bytes.fromhex(r) + b"\n" for r in want["records"])


def test_fasta_large_synthetic_matches_oracle(tmp_path):
    recs = [("syn_%d" % i, synth.bases(50000 + 37 * i, seed=100 + i)) for i in range(5)]
    text = synth.fasta_text(recs, width=61)
    p = tmp_path / "big.fa"
    p.write_bytes(text)
    f = sksffi.Fasta(str(p))
    assert f.records() == O.fasta_records(str(p))
    assert f.runs() == O.fasta_runs(str(p))


def test_fasta_missing_file():
    with pytest.raises(sksffi.SksError) as e:
        sksffi.Fasta("/nonexistent/dir/x.fa")
    assert e.value.code == 3
    assert "Unable to open /nonexistent/dir/x.fa" in str(e.value)


def test_context_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(sksffi.SksError) as e:
        sksffi.Context(0)
    assert e.value.code == 2 and "no HIP device" in str(e.value)


def test_ani_table_argument_errors():
    """sks_ctx_ani_table rejects a null context before touching a device (no GPU
    needed); the k check follows it (include/sks.h)."""
    lib = sksffi.lib()
    assert lib.sks_ctx_ani_table(None, C.c_uint32(100), 21) == 1
    assert b"null ctx" in lib.sks_last_error()


@pytest.mark.parametrize("w,k", [(31, 21), (21, 21), (32, 32), (45, 30), (64, 40), (12, 0)])
def test_join_layout_bounds_for_mask(w, k):
    """sks_join_layout_bounds_for_mask: (G + 1) non-decreasing bounds that hold
    only mask bits, bounds[0] = 0 and bounds[G] = all ones; on simulated
    canonical k-mers (min of two uniform masked values) the G value groups are
    balanced."""
    import sksffi
    m = sksffi.mask_generate(w, k, 3)
    ew = 1 if w <= 32 else 2
    log_b = 12
    G = sksffi.join_layout_groups(log_b)
    b = sksffi.join_layout_bounds_for_mask(m, log_b, ew)
    assert len(b) == (G + 1) * ew
    vals = [int(b[g * ew]) | (int(b[g * ew + 1]) << 64 if ew == 2 else 0) for g in range(G + 1)]
    assert vals[0] == 0 and vals[G] == (2 ** (64 * ew) - 1)
    assert all(x <= y for x, y in zip(vals, vals[1:]))
    assert all(v & ~m == 0 for v in vals[1:G])
    if k == 0:
        return
    P = 2 * k
    rng = np.random.default_rng(1)
    n = 200_000
    a = rng.integers(0, 2 ** min(P, 62), size=n, dtype=np.uint64).astype(object)
    c = rng.integers(0, 2 ** min(P, 62), size=n, dtype=np.uint64).astype(object)
    if P > 62:  # widen to P bits
        a = [int(x) << (P - 62) for x in a]
        c = [int(x) << (P - 62) for x in c]
    packed_bounds = []
    for v in vals[1:G]:  # pext of each bound
        x, j = 0, 0
        for bit in range(128):
            if (m >> bit) & 1:
                x |= ((v >> bit) & 1) << j
                j += 1
        packed_bounds.append(x)
    mins = np.sort(np.array([min(int(x), int(y)) for x, y in zip(a, c)], dtype=object))
    idx = np.searchsorted(mins, np.array(packed_bounds, dtype=object))
    counts = np.diff(np.concatenate([[0], idx, [n]]))
    assert counts.max() < 1.5 * n / G + 40
