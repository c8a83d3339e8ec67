"""Ordered k-mer lists — nucleotide_string_list_to_kmers (kmer_sliding.cpp:112-238)
— on the device (sks_kmer_list_build: list-mode scan + position sort +
materialise) against the oracle's restatement (ora_kmer_list), which keeps the
reference's `kmer` fields exactly: kmer_bits is the chosen strand's raw window
register (F carries up to 64 bases of run history above bit 2w; R is 2w bits).

The oracle list is checked on CPU against the oracle's own window rows and
sketches; the GPU tests compare element by element (order, duplicates,
positions, both bit fields)."""
import os
import re
import subprocess

import numpy as np
import pytest

import pyoracle as O
import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FACADE = os.path.join(ROOT, "tests", "cpp", "build", "test_facade")


def _genome(n, seed, n_runs=3):
    g = synth.bases(n, seed=seed)
    rng = np.random.default_rng(seed)
    for _ in range(n_runs):
        a = int(rng.integers(0, max(1, n - 50)))
        g[a:a + int(rng.integers(1, 40))] = ord("N")
    return g


def expected(stream: bytes, seg_off, w, m, c, nonce=1, flavour=0):
    """Oracle rows for each segment, with stream positions."""
    pos, bits, counts = [], [], []
    for g in range(len(seg_off) - 1):
        seg = stream[seg_off[g]:seg_off[g + 1]]
        runs = O.cut_runs(seg)
        starts = [mm.start() for mm in re.finditer(rb"[ACGTacgt]+", seg)]
        assert len(starts) == len(runs)
        rows = O.kmer_list(runs, w, m, c, nonce, flavour)
        counts.append(len(rows))
        for r in rows:
            pos.append(seg_off[g] + starts[int(r[4])] + int(r[5]))
            bits.append([int(x) for x in r[:4]])
    return np.array(pos, np.uint64), np.array(bits, np.uint64).reshape(-1, 4), counts


def test_oracle_list_consistent_with_windows_and_sketch():
    seq = _genome(5000, 3).tobytes()
    runs = O.cut_runs(seq)
    for w, k, c in ((21, 21, 1), (31, 21, 7), (40, 30, 3), (64, 40, 2)):
        m = O.mask(w, k, 0)
        rows = O.kmer_list(runs, w, m, c)
        win = O.windows(runs, w, m)
        keep = win[win[:, 7] % np.uint64(c) == 0]
        assert len(rows) == len(keep)
        assert np.array_equal(rows[:, 2:4], keep[:, 4:6])      # masked = canonical C
        assert np.array_equal(rows[:, 4:6], keep[:, 8:10])     # (run, offset)
        sk, _ = O.sketch(runs, w, m, "frac", c)
        u = np.unique(rows[:, 2] + (rows[:, 3].astype(object) << 64)) if len(rows) else []
        assert len(u) == len(sk)
        # kmer_bits & mask == masked_bits; R-chosen rows have no bits at or above 2w
        mlo, mhi = np.uint64(m & (2**64 - 1)), np.uint64(m >> 64)
        assert np.array_equal(rows[:, 0] & mlo, rows[:, 2])
        assert np.array_equal(rows[:, 1] & mhi, rows[:, 3])


def test_oracle_f_history_above_window():
    # a run longer than w: when F is chosen its register keeps older bases
    seq = b"ACGTTGCAAC" * 8
    runs = O.cut_runs(seq)
    m = O.mask(10, 10, 0)
    rows = O.kmer_list(runs, 10, m, 1)
    hist = [r for r in rows if int(r[0]) >> 20 or int(r[1])]
    assert hist, "expected F registers carrying run history above bit 2w"


@pytest.fixture(scope="module")
def gpu():
    import torch
    import sksffi
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    c = sksffi.Context(0)
    yield torch, c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("w,k,c", [(5, 5, 1), (21, 21, 200), (31, 21, 1), (31, 21, 13), (32, 20, 5),
                                   (33, 25, 1), (40, 30, 11), (64, 40, 3), (64, 64, 1)])
def test_device_list_matches_oracle(gpu, w, k, c):
    torch, ctx = gpu
    genomes = [_genome(9000, 10 + i, n_runs=i) for i in range(3)] + [_genome(20, 99, 0)]
    stream = b"".join(g.tobytes() + b"\n" for g in genomes)
    offs = [0]
    for g in genomes:
        offs.append(offs[-1] + len(g) + 1)
    m = O.mask(w, k, 1)
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to("cuda:0")
    pos, bits, counts = ctx.kmer_list(d.data_ptr(), len(stream), offs, w, m, c)
    wpos, wbits, wcounts = expected(stream, offs, w, m, c)
    assert list(counts) == wcounts
    assert np.array_equal(pos, wpos)
    assert np.array_equal(bits, wbits)


@pytest.mark.gpu
def test_device_list_capacity_rerun(gpu):
    """c = 1 on low-complexity input: every window survives, far above the
    capacity estimate for c = 1 is exact; c = 2 on a constant run makes the
    estimate too small only if selection is skewed — force it with 'AAAA…'."""
    torch, ctx = gpu
    stream = b"A" * 200000 + b"\n"
    m = O.mask(21, 21, 0)
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to("cuda:0")
    for c in (1, 2, 3):
        pos, bits, counts = ctx.kmer_list(d.data_ptr(), len(stream), [0, len(stream)], 21, m, c)
        wpos, wbits, wcounts = expected(stream, [0, len(stream)], 21, m, c)
        assert list(counts) == wcounts
        assert np.array_equal(pos, wpos) and np.array_equal(bits, wbits)


@pytest.mark.gpu
def test_facade_nucleotide_string_list_to_kmers(tmp_path):
    if not os.path.exists(FACADE):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    g = _genome(30000, 5)
    path = tmp_path / "g.fa"
    path.write_bytes(synth.fasta_text([("a", g[:12000]), ("b", g[12000:])], width=61))
    for w, k, c in ((31, 21, 50), (45, 30, 7)):
        r = subprocess.run([FACADE, "list", str(w), str(k), "0", str(c), str(path)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        got = [tuple(int(x, 16) for x in line.split()) for line in r.stdout.split("\n") if line]
        rows = O.kmer_list(O.fasta_runs(str(path)), w, O.mask(w, k, 0), c)
        want = [(int(a) | int(b) << 64, int(cc) | int(d) << 64) for a, b, cc, d in rows[:, :4]]
        assert got == want


@pytest.mark.gpu
@pytest.mark.parametrize("w,k", [(5, 5), (21, 21), (31, 21), (32, 32), (33, 25), (45, 30), (64, 40)])
def test_windows_dense_matches_oracle(gpu, w, k):
    """sks_windows_dense (every window, dense by start, for a host predicate)
    against the oracle's every-window list (c = 1): the validity bits are set
    exactly at the oracle's window starts and each row holds that window's
    kmer_bits (with the 128-bit F history) and masked bits.  Done over the whole
    stream and again as pieces cut at odd offsets, each given
    min(start, 64 - w) bytes of history, as the facade's for_each_window does."""
    torch, ctx = gpu
    genomes = [_genome(7000, 20 + i, n_runs=i + 1) for i in range(3)] + [_genome(25, 98, 0)]
    stream = b"".join(g.tobytes() + b"\n" for g in genomes)
    n = len(stream)
    m = O.mask(w, k, 2)
    wpos, wbits, _ = expected(stream, [0, n], w, m, 1)
    words = 3 if w <= 32 else 4
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to("cuda:0")

    def dense(a, b):  # window starts [a, b)
        h = min(a, 64 - w)
        lo, hi = a - h, min(n, b + w - 1)
        nw = b - a
        rows = torch.zeros(max(nw, 1) * words, dtype=torch.int64, device="cuda:0")
        valid = torch.zeros(max((nw + 63) // 64, 1), dtype=torch.int64, device="cuda:0")
        ctx.windows_dense(d.data_ptr() + lo, hi - lo, h, nw, w, m, rows.data_ptr(), valid.data_ptr())
        torch.cuda.synchronize()
        v = valid.cpu().numpy().view(np.uint64)
        bits = np.unpackbits(v.view(np.uint8), bitorder="little")[:nw].astype(bool)
        return bits, rows.cpu().numpy().view(np.uint64).reshape(-1, words)[:nw]

    for cuts in ([0, n - w + 1], [0, 4099, 9000, 13333, n - w + 1]):
        got_pos, got_rows = [], []
        for a, b in zip(cuts[:-1], cuts[1:]):
            ok, rows = dense(a, b)
            idx = np.nonzero(ok)[0]
            got_pos.append(idx.astype(np.uint64) + np.uint64(a))
            got_rows.append(rows[idx])
        gp = np.concatenate(got_pos)
        gr = np.concatenate(got_rows)
        assert np.array_equal(gp, wpos)
        assert np.array_equal(gr[:, 0], wbits[:, 0]) and np.array_equal(gr[:, 1], wbits[:, 1])
        assert np.array_equal(gr[:, 2], wbits[:, 2])
        if words == 4:
            assert np.array_equal(gr[:, 3], wbits[:, 3])
        else:
            assert not wbits[:, 3].any()
