"""The reference driver (src/kmer-sketching.cpp): the CSV writer's exact bytes
(:46-81) and the 62-configuration sweep of main (:214-239), run by
spaced-kmer-sketching_amd/bin/kmer-sketching, against a CSV assembled from the
oracle.  Doubles are written with C++'s default ostream formatting, which is
printf("%g") (precision 6); the mask is the 128-character bit string of
boost::dynamic_bitset's operator<< (most significant bit first)."""
import os
import subprocess

import numpy as np
import pytest

import pyoracle as O
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FACADE = os.path.join(ROOT, "tests", "cpp", "build", "test_facade")
DRIVER = os.path.join(ROOT, "spaced-kmer-sketching_amd", "bin", "kmer-sketching")
HEADER = "File 1,File 2,Estimated Value,Window Size,Mask\n"


def mask_text(m):
    return format(m >> 64, "064b") + format(m & ((1 << 64) - 1), "064b")


def csv_rows(names1, names2, values, w, m):
    return "".join(f"{a},{b},{'%g' % v},{w},{mask_text(m)}\n" for a, b, v in zip(names1, names2, values))


def reference_configs():
    return [(10, 10)] + [(k, k) for k in range(11, 41)] + [(k + 10, k) for k in range(10, 41)]


@pytest.fixture(scope="module")
def facade_bin():
    if not os.path.exists(FACADE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    return FACADE


def test_csv_writer_bytes(facade_bin, tmp_path):
    out = tmp_path / "o.csv"
    m = O.mask(31, 21, 0)
    vals = [1.0, 0.0, 0.953211458, 1e-05, 0.1234567, 123456789.0, 0.99999999]
    n1 = [f"dir/a{i}.fa" for i in range(len(vals))]
    n2 = [f"b{i}.fna" for i in range(len(vals))]
    args = [facade_bin, "csv", str(out), "0", "31", "%x" % (m & (2**64 - 1)), "%x" % (m >> 64),
            str(len(vals))] + n1 + n2 + [repr(v) for v in vals]
    subprocess.run(args, check=True, timeout=60)
    want = HEADER + csv_rows(n1, n2, vals, 31, m)
    assert out.read_text() == want
    # append mode: no header, rows added
    m2 = O.mask(50, 40, 0)
    args2 = [facade_bin, "csv", str(out), "1", "50", "%x" % (m2 & (2**64 - 1)), "%x" % (m2 >> 64),
             "1", "x", "y", "0.5"]
    subprocess.run(args2, check=True, timeout=60)
    assert out.read_text() == want + csv_rows(["x"], ["y"], [0.5], 50, m2)


def test_csv_writer_unopenable(facade_bin, tmp_path):
    bad = str(tmp_path / "no_dir" / "o.csv")
    r = subprocess.run([facade_bin, "csv", bad, "0", "21", "1", "0", "0"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0
    assert r.stderr == f"Error: Unable to open file {bad} for writing.\n"


def _genome_files(tmp_path, n=3, length=24000):
    files = []
    for i in range(n):
        g = synth.bases(length, seed=91, mut_seed=700 + i, mut_rate=0.004 * i)
        p = tmp_path / f"genome_{i}.fa"
        p.write_bytes(synth.fasta_text([(f"g{i}_a", g[: length // 2]), (f"g{i}_b", g[length // 2:])],
                                       width=60))
        files.append(str(p))
    return files


def oracle_sweep_csv(files, adjacent=False):
    runs = [O.fasta_runs(f) for f in files]
    n = len(files)
    pairs = [(i, (i + 1) % n) for i in range(n)] if adjacent else \
        [(i, j) for i in range(n) for j in range(n)]
    text = HEADER
    for w, k in reference_configs():
        m = O.mask(w, k, 0)
        sk = [O.sketch(r, w, m, "frac", 200, 1, 0)[0] for r in runs]
        vals = []
        for i, j in pairs:
            inter = O.intersect(sk[i], sk[j])
            vals.append(O.binomial_estimator(O.containment(inter, len(sk[i])), k))
        text += csv_rows([files[i] for i, _ in pairs], [files[j] for _, j in pairs], vals, w, m)
    return text


@pytest.mark.gpu
@pytest.mark.parametrize("adjacent", [False, True])
def test_driver_sweep_matches_oracle_csv(tmp_path, adjacent):
    files = _genome_files(tmp_path)
    out = tmp_path / "ani.csv"
    env = dict(os.environ)
    if adjacent:
        env["SKS_PAIRS"] = "adjacent"
    r = subprocess.run([DRIVER, str(out)] + files, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert len(lines) == 2 * 62
    assert all(l.startswith("Time taken for sketching = ") for l in lines[0::2])
    assert all(l.startswith("Time taken for comparison = ") for l in lines[1::2])
    assert out.read_text() == oracle_sweep_csv(files, adjacent)


def test_driver_missing_file_exits_like_reference(tmp_path):
    missing = str(tmp_path / "nope.fa")
    r = subprocess.run([DRIVER, str(tmp_path / "o.csv"), missing], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 1
    assert r.stderr.startswith(f"Unable to open {missing}. \n Exiting...")


@pytest.mark.gpu
def test_driver_sweep_many_files_matches_oracle_csv(tmp_path):
    """67 files (two 64-sketch blocks, the second ragged) through the drop-in
    driver's all-pairs step — one sks_all_pairs_ani call per configuration, the
    ANI written by the join into pinned host memory — including a file with no
    ACGT runs (header only), an all-N record and a record shorter than most
    windows (empty or tiny sketches: containment 0 -> ANI 0,
    ani_estimation.cpp:24-42).  The CSV equals the oracle's rendering of the
    reference writer byte for byte (kmer-sketching.cpp:46-81, 151-212)."""
    files = _genome_files(tmp_path, n=64, length=6000)
    extra = [("empty.fa", b">nothing here\n"), ("alln.fa", b">n\n" + b"N" * 500 + b"\n"),
             ("tiny.fa", b">t\nACGTACGTTGCAACGTTAGCCA\n")]
    for name, body in extra:
        p = tmp_path / name
        p.write_bytes(body)
        files.append(str(p))
    out = tmp_path / "ani.csv"
    r = subprocess.run([DRIVER, str(out)] + files, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr
    assert out.read_text() == oracle_sweep_csv(files)
