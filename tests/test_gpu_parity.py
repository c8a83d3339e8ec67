"""GPU parity: libsks.so (HIP, gfx950) against the oracle, through the C ABI.

Every comparison is bit-exact (sketch membership, sizes, windows hashed,
intersection counts); ANI is computed on the host from the exact counts.
"""
import os

import numpy as np
import pytest

import pyoracle as O
import sksffi
import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_FASTA = os.path.join(ROOT, "tests", "golden", "fasta")


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


@pytest.fixture(scope="module")
def ctx(torch_cuda):
    c = sksffi.Context(0)
    yield c
    c.close()


def upload(torch, data: bytes):
    t = torch.frombuffer(bytearray(data) if data else bytearray(b"\n"), dtype=torch.uint8)
    return t.to("cuda:0")


def build(torch, ctx, genomes, w, mask, kind="frac", param=200, flavour=0, nonce=1):
    """genomes: list of bytes; each segment is genome + '\\n'."""
    stream = b"".join(g + b"\n" for g in genomes)
    offs = [0]
    for g in genomes:
        offs.append(offs[-1] + len(g) + 1)
    dev = upload(torch, stream)
    k = sksffi.SKS_FRAC_MOD if kind == "frac" else sksffi.SKS_BOTTOM_S
    ss = ctx.sketch_build(dev.data_ptr(), len(stream), offs, w, mask, k, param, nonce, flavour)
    return ss, dev


def check_against_oracle(ss, genomes, w, mask, kind, param, flavour=0, nonce=1):
    sizes = ss.sizes()
    wins = ss.windows()
    for i, g in enumerate(genomes):
        want, nw = O.sketch(O.cut_runs(g), w, mask, kind, param, nonce, flavour)
        got = ss.sketch(i)
        assert int(wins[i]) == nw, (i, w, kind, param)
        assert int(sizes[i]) == len(want), (i, w, kind, param)
        assert np.array_equal(got, want), (i, w, kind, param, flavour)


def test_synth_device_matches_numpy(torch_cuda, ctx):
    torch = torch_cuda
    for (n, seed, ms, rate, off) in [(100003, 5, 0, 0.0, 0), (65536, 9, 77, 0.05, 12345)]:
        d = torch.empty(n, dtype=torch.uint8, device="cuda:0")
        ctx.synth_bases(d.data_ptr(), n, seed, ms, rate, off)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), synth.bases(n, seed, ms, rate, off))


def test_c1_golden(torch_cuda, ctx, golden):
    g = golden("c1_sketch.json")
    f = sksffi.Fasta(os.path.join(GOLDEN_FASTA, g["file"]))
    stream = f.stream().tobytes()
    dev = upload(torch_cuda, stream)
    for case in g["cases"]:
        k = sksffi.SKS_FRAC_MOD if case["kind"] == "frac" else sksffi.SKS_BOTTOM_S
        m = int(case["mask"], 16)
        ss = ctx.sketch_build(dev.data_ptr(), len(stream), [0, len(stream)], case["w"], m, k,
                              case["param"], case["nonce"], case["flavour"])
        got = [hex(int(lo) | int(hi) << 64) for lo, hi in ss.sketch(0)]
        assert int(ss.windows()[0]) == case["windows"]
        assert got == case["sketch"], case


def test_fasta_edge_corpus(torch_cuda, ctx, golden):
    for name in golden("fasta_cases.json")["cases"]:
        f = sksffi.Fasta(os.path.join(GOLDEN_FASTA, name))
        stream = f.stream().tobytes()
        dev = upload(torch_cuda, stream)
        for w in (1, 3, 4, 8):
            m = O.mask(w, w, 0)
            ss = ctx.sketch_build(dev.data_ptr(), len(stream), [0, len(stream)], w, m,
                                  sksffi.SKS_FRAC_MOD, 1)
            want, nw = O.sketch(f.runs(), w, m, "frac", 1)
            assert int(ss.windows()[0]) == nw, (name, w)
            assert np.array_equal(ss.sketch(0), want), (name, w)


def _genomes(seed, lens, n_frac=0.001, lower=False):
    rng = np.random.default_rng(seed)
    out = []
    for i, L in enumerate(lens):
        g = synth.bases(L, seed=seed * 1000 + i)
        if L:
            k = max(1, int(L * n_frac))
            g[rng.integers(0, L, k)] = ord("N")
            if lower:
                idx = rng.integers(0, L, L // 10)
                g[idx] = g[idx] | 0x20
        out.append(g.tobytes())
    return out


@pytest.mark.parametrize("w,k", [(1, 1), (2, 2), (5, 3), (16, 16), (17, 11), (21, 21), (31, 21),
                                 (32, 32), (32, 20)])
def test_frac_narrow_windows(torch_cuda, ctx, w, k):
    genomes = _genomes(w, [0, 3, w - 1 if w > 1 else 0, w, 4095, 4096, 4097, 20000, 131071],
                       lower=True)
    m = O.mask(w, k, 7)
    for flavour in (0, 1):
        for c in (1, 7, 200):
            ss, _ = build(torch_cuda, ctx, genomes, w, m, "frac", c, flavour)
            check_against_oracle(ss, genomes, w, m, "frac", c, flavour)


def test_frac_prefilter_even_c(torch_cuda, ctx):
    """The low-bits pre-filter kernel (scan_kernel<frac, 0, PRE>, even c) with
    c = 2^s * d for s below, at and above the 4 pre-filtered bits (the finished
    candidates test the remaining low bits only when s > 4), d = 1, and s >= 32
    (the high-word test): every sketch equals the oracle's (kmer.hpp:135-149,
    kmer-sketching.cpp:29-34 with c in place of 200)."""
    w, k = 31, 21
    genomes = _genomes(w, [0, 30, 4097, 90000, 400000], lower=True)
    m = O.mask(w, k, 0)
    for c in (2, 6, 16, 96, 1000, 1024, 3 << 20, 1 << 33):
        ss, _ = build(torch_cuda, ctx, genomes, w, m, "frac", c, 0)
        check_against_oracle(ss, genomes, w, m, "frac", c, 0)
        if c <= 1000:
            assert int(ss.sizes()[4]) > 0, c


@pytest.mark.parametrize("w,k", [(33, 33), (40, 21), (50, 40), (63, 30), (64, 64)])
def test_frac_wide_windows(torch_cuda, ctx, w, k):
    genomes = _genomes(w, [0, w, 4096 + w, 30000, 70001], lower=True)
    m = O.mask(w, k, 3)
    for flavour in (0, 1):
        for c in (1, 50):
            ss, _ = build(torch_cuda, ctx, genomes, w, m, "frac", c, flavour)
            check_against_oracle(ss, genomes, w, m, "frac", c, flavour)


@pytest.mark.parametrize("w,k", [(21, 21), (31, 21), (8, 8), (45, 21)])
def test_bottom_s(torch_cuda, ctx, w, k):
    genomes = _genomes(100 + w, [0, 10, 500, 9000, 60000, 250000])
    m = O.mask(w, k, 0)
    for flavour in (0, 1):
        for s in (1, 10, 1000, 20000):
            ss, _ = build(torch_cuda, ctx, genomes, w, m, "bottom", s, flavour)
            check_against_oracle(ss, genomes, w, m, "bottom", s, flavour)


def test_bottom_s_many_genomes(torch_cuda, ctx):
    """300 genomes in one build (one select workgroup each), related and
    unrelated, lengths around the candidate margin, both flavours."""
    genomes = []
    for i in range(300):
        L = 2000 + 517 * (i % 41)
        genomes.append(synth.bases(L, seed=800 + i % 7, mut_seed=1200 + i,
                                   mut_rate=0.01 * (i % 5)).tobytes())
    m = O.mask(31, 21, 2)
    for flavour in (0, 1):
        for s_ in (1, 200, 1500):
            ss, _ = build(torch_cuda, ctx, genomes, 31, m, "bottom", s_, flavour)
            check_against_oracle(ss, genomes, 31, m, "bottom", s_, flavour)


def test_bottom_s_fused_sort_paths(torch_cuda, ctx):
    """k_bottom_fused sorts each genome's candidates by a counting sort on the
    top 12 packed-key bits plus per-bucket insertion sorts, and falls back to
    rocPRIM's block radix sort when a bucket holds more than 64 keys. A genome
    of only A and C crowds its canonical k-mers into 2^6 of the 4096 buckets
    (fallback); the others are ordinary (bucket sort), one repeats a 5 kb
    stretch many times (equal keys in a bucket); all in one launch, both
    flavours, against the oracle."""
    rng = np.random.default_rng(77)
    ac = np.where(rng.random(200_000) < 0.5, ord("A"), ord("C")).astype(np.uint8).tobytes()
    rep = synth.bases(5000, seed=78).tobytes()
    genomes = [ac, synth.bases(150_000, seed=79).tobytes(), rep * 30 + synth.bases(80_000, seed=80).tobytes(),
               synth.bases(120_000, seed=81, mut_seed=82, mut_rate=0.02).tobytes()]
    m = O.mask(31, 21, 0)
    for flavour in (0, 1):
        for s_ in (2000, 10000):
            ss, _ = build(torch_cuda, ctx, genomes, 31, m, "bottom", s_, flavour)
            check_against_oracle(ss, genomes, 31, m, "bottom", s_, flavour)


@pytest.mark.parametrize("w,k", [(11, 8), (9, 5), (13, 12)])
def test_bottom_s_fused_small_k(torch_cuda, ctx, w, k):
    """k_bottom_fused with packed keys of 2k <= 24 bits: at 2k <= 12 the bucket
    is the whole key (shift 0), above it the top 12 bits; several genomes so the
    fused kernel (not the single-genome device-wide path) runs; against the
    oracle, both flavours."""
    genomes = [synth.bases(40_000 + 3001 * i, seed=900 + i, mut_seed=950 + i,
                           mut_rate=0.01 * i).tobytes() for i in range(6)]
    m = O.mask(w, k, 1)
    for flavour in (0, 1):
        for s_ in (50, 3000):
            ss, _ = build(torch_cuda, ctx, genomes, w, m, "bottom", s_, flavour)
            check_against_oracle(ss, genomes, w, m, "bottom", s_, flavour)


def test_bottom_s_unfused_paths(torch_cuda, ctx, monkeypatch):
    """The per-genome fused post kernel is the default for genomes of <= 16384
    candidates; SKS_NO_FUSED_BOTTOM routes a build of several genomes through
    compaction + segmented sort + unique
    + k_bottom_select instead. Both must give the oracle's sets; both selects
    stop their radix passes early once the chosen digit's bucket is kept whole."""
    genomes = [synth.bases(3000 + 997 * i, seed=1300 + i % 3, mut_seed=1400 + i,
                           mut_rate=0.02 * (i % 4)).tobytes() for i in range(40)]
    m = O.mask(31, 21, 5)
    monkeypatch.setenv("SKS_NO_FUSED_BOTTOM", "1")
    for flavour in (0, 1):
        for s_ in (1, 300):
            ss, _ = build(torch_cuda, ctx, genomes, 31, m, "bottom", s_, flavour)
            check_against_oracle(ss, genomes, 31, m, "bottom", s_, flavour)


def test_bottom_s_single_genome_paths(torch_cuda, ctx, monkeypatch):
    """One genome per build (kmer_set_from_fasta_file's shape): by default the
    single-round-trip path (scan + k_bottom_fused into the set's own arrays,
    one read-back); SKS_NO_FAST_BOTTOM takes the general build. Tiny, ordinary,
    A/C-only (the fused kernel's block-sort fallback), mutated and periodic
    genomes (too few distinct candidates: the fast path falls back and the
    threshold is raised), both flavours, each against the oracle."""
    rng = np.random.default_rng(91)
    ac = np.where(rng.random(150_000) < 0.5, ord("A"), ord("C")).astype(np.uint8).tobytes()
    unit = synth.bases(37, seed=92).tobytes()
    genomes = [synth.bases(10, seed=93).tobytes(), synth.bases(60_000, seed=94).tobytes(), ac,
               synth.bases(400_000, seed=95, mut_seed=96, mut_rate=0.03).tobytes(), unit * 4000]
    m = O.mask(31, 21, 0)
    for fast in (True, False):
        if fast:
            monkeypatch.delenv("SKS_NO_FAST_BOTTOM", raising=False)
        else:
            monkeypatch.setenv("SKS_NO_FAST_BOTTOM", "1")
        for flavour in (0, 1):
            for s_ in (1, 700, 10000):
                for g in genomes:
                    ss, _ = build(torch_cuda, ctx, [g], 31, m, "bottom", s_, flavour)
                    check_against_oracle(ss, [g], 31, m, "bottom", s_, flavour)


def test_bottom_s_low_complexity_forces_threshold_retry(torch_cuda, ctx):
    # periodic genome: few distinct k-mers, so the first threshold pass finds
    # fewer than s candidates and the build must raise the threshold
    unit = synth.bases(37, seed=4).tobytes()
    genomes = [unit * 5000, (unit * 300) + synth.bases(50000, seed=5).tobytes()]
    m = O.mask(21, 21, 0)
    for s in (30, 5000):
        ss, _ = build(torch_cuda, ctx, genomes, 21, m, "bottom", s)
        check_against_oracle(ss, genomes, 21, m, "bottom", s)


def test_frac_capacity_overflow_retry(torch_cuda, ctx):
    # c = 1 keeps every window; a homopolymer produces one k-mer many times
    genomes = [b"A" * 300000, synth.bases(100000, seed=8).tobytes()]
    m = O.mask(15, 15, 0)
    ss, _ = build(torch_cuda, ctx, genomes, 15, m, "frac", 1)
    check_against_oracle(ss, genomes, 15, m, "frac", 1)


def test_config2_5mb_bottom_s(torch_cuda, ctx):
    g = synth.bases(5_000_000, seed=2).tobytes()
    m = O.mask(31, 21, 0)
    assert m == 0x03FF3CCFFF3C33F3
    ss, _ = build(torch_cuda, ctx, [g], 31, m, "bottom", 10000)
    check_against_oracle(ss, [g], 31, m, "bottom", 10000)
    ss, _ = build(torch_cuda, ctx, [g], 31, m, "frac", 1000)
    check_against_oracle(ss, [g], 31, m, "frac", 1000)


def test_intersections_match_oracle(torch_cuda, ctx):
    torch = torch_cuda
    anc = synth.bases(40000, seed=50)
    genomes = [synth.bases(40000, seed=50, mut_seed=60 + i, mut_rate=0.004 * i).tobytes()
               for i in range(6)] + [b"", synth.bases(40000, seed=51).tobytes()]
    del anc
    for (w, k, kind, p) in [(21, 21, "frac", 20), (31, 21, "bottom", 500), (40, 30, "frac", 10)]:
        m = O.mask(w, k, 0)
        ss, _ = build(torch, ctx, genomes, w, m, kind, p)
        sk = [O.sketch(O.cut_runs(g), w, m, kind, p)[0] for g in genomes]
        data, starts, sizes = ss.device_ptrs()
        n = len(genomes)
        out = torch.zeros(n * n, dtype=torch.int32, device="cuda:0")
        ctx.intersect_all(data, starts, sizes, ss.elem_words, n, 0, n, out.data_ptr())
        torch.cuda.synchronize()
        got = out.cpu().numpy().reshape(n, n)
        want = np.array([[O.intersect(sk[i], sk[j]) for j in range(n)] for i in range(n)])
        assert np.array_equal(got, want), (w, kind)
        # row block form
        out2 = torch.zeros(3 * n, dtype=torch.int32, device="cuda:0")
        ctx.intersect_all(data, starts, sizes, ss.elem_words, n, 2, 5, out2.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(out2.cpu().numpy().reshape(3, n), want[2:5])
        # pair-list form (compute_pairwise_kmer_set_intersections)
        a = torch.tensor([0, 1, 7, 6, 3], dtype=torch.int32, device="cuda:0")
        b = torch.tensor([1, 0, 7, 2, 6], dtype=torch.int32, device="cuda:0")
        o3 = torch.zeros(5, dtype=torch.int32, device="cuda:0")
        ctx.intersect_pairs(data, starts, sizes, ss.elem_words, a.data_ptr(), b.data_ptr(), 5,
                            o3.data_ptr())
        torch.cuda.synchronize()
        assert o3.cpu().tolist() == [want[x][y] for x, y in zip(a.tolist(), b.tolist())]


def test_frac_chunk_union_property(torch_cuda, ctx):
    """Size-independent property at scale: the sketch of a genome equals the
    union of the sketches of overlapping chunks ((w-1)-base halos), and the
    c=1000 sketch is exactly the c=200 sketch filtered by fmh % 1000 == 0."""
    torch = torch_cuda
    L, w = 40_000_000, 31
    m = O.mask(31, 21, 0)
    dev = torch.empty(L + 1, dtype=torch.uint8, device="cuda:0")
    ctx.synth_bases(dev.data_ptr(), L, 33)
    dev[L] = ord("\n")
    dev[1000:1100] = ord("N")
    whole = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, sksffi.SKS_FRAC_MOD, 200)
    S200 = whole.sketch(0)
    cuts = [0, 7_000_003, 19_999_999, 31_000_000, L + 1]
    offs = []
    for i in range(len(cuts) - 1):
        offs.append((cuts[i], min(L + 1, cuts[i + 1] + w - 1)))
    # overlapping segments: build each separately
    parts = []
    for (a, b) in offs:
        ss = ctx.sketch_build(dev.data_ptr() + a, b - a, [0, b - a], w, m, sksffi.SKS_FRAC_MOD, 200)
        parts.append(ss.sketch(0))
    union = np.unique(np.concatenate([p[:, 0] for p in parts]))
    assert np.array_equal(union, S200[:, 0])
    # the same union on the device (sks_sketch_union, used by the sharded build)
    cat = torch.from_numpy(np.concatenate([p[:, 0] for p in parts]).view(np.int64)).to("cuda:0")
    uo = torch.empty_like(cat)
    k = ctx.sketch_union(cat.data_ptr(), cat.numel(), uo.data_ptr())
    torch.cuda.synchronize()
    assert k == len(S200) and np.array_equal(uo[:k].cpu().numpy().view(np.uint64), S200[:, 0])
    assert ctx.sketch_union(cat.data_ptr(), 0, uo.data_ptr()) == 0
    assert int(whole.windows()[0]) == (1000 - w + 1) + (L - 1100 - w + 1)
    s1000 = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, sksffi.SKS_FRAC_MOD, 1000)
    S1000 = s1000.sketch(0)
    keep = [x for x in S200[:, 0] if sksffi.frac_min_hash(int(x), m, w, 1, 0) % 1000 == 0]
    assert np.array_equal(np.array(keep, dtype=np.uint64), S1000[:, 0])
    for x in S1000[:50, 0]:
        assert sksffi.frac_min_hash(int(x), m, w, 1, 0) % 1000 == 0


def test_wide_chunk_union_w45(torch_cuda, ctx):
    """The sharded-genome union for 32 < w <= 64 (sks_sketch_union_wide): the
    union of w = 45 chunk sketches ((w-1)-base halos) equals the whole-genome
    sketch and the oracle's, ordered as 128-bit values (hi word first)."""
    torch = torch_cuda
    L, w, k, c = 3_000_000, 45, 30, 20
    m = O.mask(w, k, 1)
    assert m >> 64  # the mask reaches the high word
    dev = torch.empty(L + 1, dtype=torch.uint8, device="cuda:0")
    ctx.synth_bases(dev.data_ptr(), L, 57)
    dev[L] = ord("\n")
    dev[50_000:50_030] = ord("N")
    whole = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, sksffi.SKS_FRAC_MOD, c)
    S = whole.sketch(0)
    want, _ = O.sketch(O.cut_runs(dev.cpu().numpy().tobytes()), w, m, "frac", c)
    assert np.array_equal(S, want)
    cuts = [0, 1_000_001, 2_222_222, L + 1]
    parts = []
    for i in range(len(cuts) - 1):
        a, b = cuts[i], min(L + 1, cuts[i + 1] + w - 1)
        ss = ctx.sketch_build(dev.data_ptr() + a, b - a, [0, b - a], w, m, sksffi.SKS_FRAC_MOD, c)
        parts.append(ss.sketch(0))
    cat = np.concatenate(parts)
    rng = np.random.default_rng(4)
    cat = cat[rng.permutation(len(cat))]  # any order in
    d_in = torch.from_numpy(np.ascontiguousarray(cat).view(np.int64)).to("cuda:0")
    d_out = torch.empty_like(d_in)
    n = ctx.sketch_union(d_in.data_ptr(), len(cat), d_out.data_ptr(), elem_words=2)
    torch.cuda.synchronize()
    assert n == len(S)
    assert np.array_equal(d_out[:n].cpu().numpy().view(np.uint64), S)
    assert ctx.sketch_union(d_in.data_ptr(), 0, d_out.data_ptr(), elem_words=2) == 0
    with pytest.raises(sksffi.SksError):  # 16-byte alignment is required
        ctx.sketch_union(d_in.data_ptr() + 8, 4, d_out.data_ptr(), elem_words=2)


def test_genome_over_4gb_chunk_union(torch_cuda, ctx):
    """Maximum sizes: one 4.6 GB genome (byte offsets, tile and window counts past
    2^32) equals the union of the sketches of two halves with a (w-1)-base halo,
    and its window count is exact; FracMinHash 1/1000 and bottom-s both ways."""
    torch = torch_cuda
    L, w = 4_600_000_000, 31
    m = O.mask(31, 21, 0)
    dev = torch.empty(L + 1, dtype=torch.uint8, device="cuda:0")
    ctx.synth_bases(dev.data_ptr(), L, 4242)
    dev[L] = ord("\n")
    torch.cuda.synchronize()
    whole = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, sksffi.SKS_FRAC_MOD, 1000)
    assert int(whole.windows()[0]) == L - w + 1
    cut = 2_300_000_017
    a = ctx.sketch_build(dev.data_ptr(), cut + w - 1, [0, cut + w - 1], w, m, sksffi.SKS_FRAC_MOD,
                         1000)
    b = ctx.sketch_build(dev.data_ptr() + cut, L + 1 - cut, [0, L + 1 - cut], w, m,
                         sksffi.SKS_FRAC_MOD, 1000)
    union = np.union1d(a.sketch(0)[:, 0], b.sketch(0)[:, 0])
    S = whole.sketch(0)[:, 0]
    assert np.array_equal(union, S)
    assert int(a.windows()[0]) + int(b.windows()[0]) == L - w + 1
    for x in S[:: max(1, len(S) // 200)]:
        assert sksffi.frac_min_hash(int(x), m, w, 1, 0) % 1000 == 0
    # bottom-s over the whole genome: the s smallest fmh of the union of the halves' bottom-s
    s_ = 10000
    bw = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, sksffi.SKS_BOTTOM_S, s_).sketch(0)[:, 0]
    ba = ctx.sketch_build(dev.data_ptr(), cut + w - 1, [0, cut + w - 1], w, m, sksffi.SKS_BOTTOM_S,
                          s_).sketch(0)[:, 0]
    bb = ctx.sketch_build(dev.data_ptr() + cut, L + 1 - cut, [0, L + 1 - cut], w, m,
                          sksffi.SKS_BOTTOM_S, s_).sketch(0)[:, 0]
    cand = np.union1d(ba, bb)
    keyed = sorted((sksffi.frac_min_hash(int(x), m, w, 1, 0), int(x)) for x in cand)[:s_]
    assert np.array_equal(np.array(sorted(x for _, x in keyed), dtype=np.uint64), bw)
    del dev


def test_concurrent_contexts_on_streams(torch_cuda, ctx):
    """bench.py's headline mode: builds from several host threads, one context
    per HIP stream, in flight together (and sets freed, both ways, while another
    thread builds) give the serial build's sketches; small genomes also match
    the oracle."""
    import threading
    torch = torch_cuda
    L, w = 12_000_000, 31
    m = O.mask(31, 21, 0)
    dev = torch.empty(L + 1, dtype=torch.uint8, device="cuda:0")
    ctx.synth_bases(dev.data_ptr(), L, 91)
    dev[L] = ord("\n")
    dev[5000:5100] = ord("N")
    torch.cuda.synchronize()
    jobs = [(sksffi.SKS_FRAC_MOD, 1000), (sksffi.SKS_FRAC_MOD, 200), (sksffi.SKS_BOTTOM_S, 5000)]
    want = {j: ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, *j).sketch(0) for j in jobs}
    small = _genomes(5, [30_000, 20_011])
    streams = [torch.cuda.Stream() for _ in range(3)]
    ctxs = [sksffi.Context(0, st.cuda_stream) for st in streams]
    bad = []

    def worker(i):
        try:
            for r in range(4):
                kind, param = jobs[(i + r) % len(jobs)]
                ss = ctxs[i].sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, m, kind, param)
                if not np.array_equal(ss.sketch(0), want[(kind, param)]):
                    bad.append((i, r, kind, param))
                if r % 2:  # frees while the other threads build
                    ss.free(stream=streams[i].cuda_stream)  # stream-ordered
                else:
                    del ss  # device-wide wait, as hipFree
            stream = b"".join(g + b"\n" for g in small)
            d_small = upload(torch, stream)
            torch.cuda.synchronize()  # the upload ran on torch's stream, not ctxs[i]'s
            offs = np.cumsum([0] + [len(g) + 1 for g in small])
            sm = ctxs[i].sketch_build(d_small.data_ptr(), len(stream), offs, w, m,
                                      sksffi.SKS_FRAC_MOD, 200)
            check_against_oracle(sm, small, w, m, "frac", 200)
        except Exception as e:  # reported below
            bad.append(repr(e))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(3)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    assert not bad, bad


def test_block_cache_reuse_and_eviction(torch_cuda, ctx):
    """Sketch arrays freed (plainly or stream-ordered) return to the block cache
    and are handed to later builds; more than its 16 blocks evicts the oldest.
    Sets built from recycled arrays equal fresh ones and the oracle."""
    torch = torch_cuda
    m = O.mask(31, 21, 1)
    genomes = _genomes(77, [5000, 20000, 60000, 150000])
    want = []
    for i, g in enumerate(genomes):
        ss, _ = build(torch, ctx, [g], 31, m, "frac", 7 + i)
        want.append(ss.sketch(0))
        del ss
    st = torch.cuda.Stream()
    for rnd in range(3):
        held = []
        for i, g in enumerate(genomes * 6):  # 24 sets alive: more blocks than the cache keeps
            ss, _ = build(torch, ctx, [g], 31, m, "frac", 7 + i % 4)
            assert np.array_equal(ss.sketch(0), want[i % 4]), (rnd, i)
            held.append(ss)
        for j, ss in enumerate(held):
            if (j + rnd) % 2:
                ss.free(stream=st.cuda_stream)
            else:
                ss.free()
    torch.cuda.synchronize()
    ss, _ = build(torch, ctx, genomes, 31, m, "frac", 7)
    check_against_oracle(ss, genomes, 31, m, "frac", 7)


def test_argument_errors(torch_cuda, ctx):
    torch = torch_cuda
    d = upload(torch, b"ACGTACGT\n")
    m = O.mask(4, 4, 0)
    for (w, mask, param, code) in [(0, m, 5, 1), (65, m, 5, 1), (4, m, 0, 1),
                                   (2, m, 5, 5)]:  # mask bits >= 2w
        with pytest.raises(sksffi.SksError) as e:
            ctx.sketch_build(d.data_ptr(), 9, [0, 9], w, mask, sksffi.SKS_FRAC_MOD, param)
        assert e.value.code == code
    with pytest.raises(sksffi.SksError):
        ctx.sketch_build(d.data_ptr(), 9, [0, 10], 4, m, sksffi.SKS_FRAC_MOD, 5)


KERNELS = [sksffi.INTERSECT_AUTO, sksffi.INTERSECT_MERGE, sksffi.INTERSECT_JOIN,
           sksffi.INTERSECT_GLOBAL]


@pytest.fixture
def kernel_ctx(ctx, request):
    ctx.set_intersect_kernel(request.param)
    yield ctx
    ctx.set_intersect_kernel(sksffi.INTERSECT_AUTO)


@pytest.mark.parametrize("kernel_ctx", KERNELS, indirect=True)
def test_many_sketches_tiled_and_symmetric(torch_cuda, kernel_ctx):
    """130 sketches (3 tile blocks, ragged last block) of varied sizes: the
    tiled all-pairs kernel, its row-block form, and the symmetric tile form
    split across 3 'ranks' and summed, all equal the oracle's merge counts —
    for every intersection kernel (join, merge tiles, global)."""
    torch = torch_cuda
    ctx = kernel_ctx
    n = 130
    genomes = []
    for i in range(n):
        fam = i % 5
        L = 3000 + 97 * (i % 23)
        g = synth.bases(L, seed=700 + fam, mut_seed=900 + i, mut_rate=0.003 * (i % 7))
        genomes.append(g.tobytes() if i % 31 else b"")
    w = 21
    m = O.mask(w, w, 0)
    ss, _ = build(torch, ctx, genomes, w, m, "frac", 3)
    sk = [O.sketch(O.cut_runs(g), w, m, "frac", 3)[0] for g in genomes]
    want = np.array([[O.intersect(sk[i], sk[j]) for j in range(n)] for i in range(n)])
    data, starts, sizes = ss.device_ptrs()
    out = torch.full((n * n,), -7, dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(data, starts, sizes, 1, n, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(n, n), want)
    # block-aligned rows ending inside a block: the diagonal tile (rows 64..69
    # against columns 64..127) joins without probes and must skip rows >= 70
    rows = torch.zeros(((70 - 64) * n,), dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(data, starts, sizes, 1, n, 64, 70, rows.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(rows.cpu().numpy().reshape(6, n), want[64:70])
    rows = torch.zeros(((70 - 65) * n,), dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(data, starts, sizes, 1, n, 65, 70, rows.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(rows.cpu().numpy().reshape(5, n), want[65:70])
    T = sksffi.intersect_sym_tiles(n)
    assert T == 6
    acc = np.zeros((n, n), dtype=np.int64)
    ranges = [(0, T)] if ctx_kernel(ctx) == sksffi.INTERSECT_GLOBAL else [(0, 2), (2, 3), (3, T)]
    for (a, b) in ranges:
        part = torch.full((n * n,), 5, dtype=torch.int32, device="cuda:0")
        ctx.intersect_sym(data, starts, sizes, 1, n, a, b, part.data_ptr())
        torch.cuda.synchronize()
        acc += part.cpu().numpy().reshape(n, n)
    assert np.array_equal(acc, want)


def ctx_kernel(ctx):
    return getattr(ctx, "_intersect_kernel", sksffi.INTERSECT_AUTO)


def _device_sketch_arrays(torch, sketches):
    """Packs sorted unique u64 arrays as the CSR (data, starts, sizes) the
    sks_intersect_* entry points take (any caller-owned device arrays)."""
    sizes = np.array([len(x) for x in sketches], dtype=np.uint32)
    starts = np.zeros(len(sketches), dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    flat = np.concatenate([np.asarray(x, dtype=np.uint64) for x in sketches] + [np.zeros(1, np.uint64)])
    d = torch.from_numpy(flat.view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    return d, st, sz


@pytest.mark.parametrize("kernel_ctx", KERNELS, indirect=True)
@pytest.mark.parametrize("shape", ["families", "identical", "extremes"])
def test_intersect_kernels_adversarial_arrays(torch_cuda, kernel_ctx, shape):
    """Caller-provided sorted unique u64 arrays that stress the kernels:
    heavy sharing (every pair shares most values), all sketches identical
    (the join's worst case: every probe hits all 64 columns), and the extreme
    values 0 and 2^64-1 (the join table's empty key) plus runs of values that
    differ only in their high words.  Counts equal numpy's intersect1d."""
    torch = torch_cuda
    ctx = kernel_ctx
    rng = np.random.default_rng({"families": 1, "identical": 2, "extremes": 3}[shape])
    n = 150
    sk = []
    if shape == "families":
        base = [np.unique(rng.integers(0, 2**62, size=3000, dtype=np.uint64)) for _ in range(3)]
        for i in range(n):
            b = base[i % 3]
            keep = b[rng.random(b.size) < 0.3 + 0.6 * ((i * 7) % 10) / 10]
            extra = rng.integers(0, 2**62, size=int(rng.integers(0, 400)), dtype=np.uint64)
            sk.append(np.unique(np.concatenate([keep, extra])))
    elif shape == "identical":
        one = np.unique(rng.integers(0, 2**64 - 1, size=2500, dtype=np.uint64))
        sk = [one.copy() for _ in range(n)]
    else:
        hi = (np.arange(1, 40, dtype=np.uint64) << np.uint64(40))
        core = np.unique(np.concatenate([
            np.array([0, 1, 2**64 - 2, 2**64 - 1], dtype=np.uint64), hi,
            rng.integers(0, 2**64 - 1, size=1500, dtype=np.uint64)]))
        for i in range(n):
            sel = core[rng.random(core.size) < 0.5]
            if i % 4 == 0:
                sel = np.union1d(sel, np.array([0, 2**64 - 1], dtype=np.uint64))
            sk.append(sel if i % 37 else np.zeros(0, dtype=np.uint64))
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    out = torch.full((n * n,), -3, dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(n, n), want)
    for r0, r1 in ((64, 150), (3, 97)):  # row blocks aligned / not aligned with column blocks
        rows = torch.full(((r1 - r0) * n,), -5, dtype=torch.int32, device="cuda:0")
        ctx.intersect_all(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, r0, r1, rows.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(rows.cpu().numpy().reshape(r1 - r0, n), want[r0:r1])
    T = sksffi.intersect_sym_tiles(n)
    sym = torch.full((n * n,), 9, dtype=torch.int32, device="cuda:0")
    ctx.intersect_sym(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, 0, T, sym.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(sym.cpu().numpy().reshape(n, n), want)


def test_join_layout_build_and_concat(torch_cuda, ctx):
    """sks_join_layout_build + sks_intersect_sym_layout: one layout of all
    sketches, and two layouts of block-aligned halves concatenated the way the
    multi-GPU all-gather does (data/ids/boff appended, bstart shifted), both give
    the oracle matrix, for every tile range split."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n = 150
    base = [np.unique(rng.integers(0, 2**62, size=2500, dtype=np.uint64)) for _ in range(3)]
    sk = []
    for i in range(n):
        b = base[i % 3]
        keep = b[rng.random(b.size) < 0.2 + 0.7 * ((i * 5) % 9) / 9]
        extra = rng.integers(0, 2**64 - 1, size=int(rng.integers(0, 300)), dtype=np.uint64)
        sk.append(np.unique(np.concatenate([keep, extra, np.array([2**64 - 1], np.uint64)]))
                  if i % 7 == 0 else np.unique(np.concatenate([keep, extra])))
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    log_b = sksffi.join_layout_log_b(max(len(s) for s in sk))
    BW = sksffi.join_layout_boff_words(log_b)
    cap = sksffi.join_layout_capacity()

    # the halves share one set of value-group bounds, as a multi-GPU run's
    # layouts do (rank 0's, broadcast): here the last 86 sketches' own bounds
    gb = torch.empty(sksffi.join_layout_groups(log_b) + 1, dtype=torch.int64, device="cuda:0")
    ctx.join_layout_bounds(d.data_ptr(), st.data_ptr() + 8 * 64, sz.data_ptr() + 4 * 64, n - 64, log_b,
                           gb.data_ptr())

    def build(first, count):
        tot = int(sum(len(s) for s in sk[first:first + count]))
        nb = (count + 63) // 64
        out = (torch.empty(max(tot, 1), dtype=torch.int64, device="cuda:0"),
               torch.empty(max(tot, 1), dtype=torch.int64, device="cuda:0"),
               torch.empty(nb * BW, dtype=torch.int32, device="cuda:0"),
               torch.empty(nb + 1, dtype=torch.int64, device="cuda:0"))
        mx = ctx.join_layout_build(d.data_ptr(), st.data_ptr() + 8 * first, sz.data_ptr() + 4 * first,
                                   count, log_b, *(t.data_ptr() for t in out), bounds=gb.data_ptr())
        assert mx <= cap
        torch.cuda.synchronize()
        assert int(out[3][nb].item()) == tot
        return out, tot

    T = sksffi.intersect_sym_tiles(n)
    (a_d, a_i, a_b, a_s), _ = build(0, n)
    (p_d, p_i, p_b, p_s), tot0 = build(0, 64)
    (q_d, q_i, q_b, q_s), tot1 = build(64, n - 64)
    # regions sit at raw offsets: a layout of `tot` elements fills [0, tot) of
    # its buffers at most, so the raw-sized buffers concatenate as they are
    cat_d = torch.cat([p_d[:tot0], q_d[:tot1]])
    cat_i = torch.cat([p_i[:tot0], q_i[:tot1]])
    cat_b = torch.cat([p_b, q_b])
    cat_s = torch.cat([p_s[:1], q_s + tot0])
    for layout in ((a_d, a_i, a_b, a_s), (cat_d, cat_i, cat_b, cat_s)):
        acc = np.zeros((n, n), dtype=np.int64)
        for (t0, t1) in [(0, 1), (1, 4), (4, T)]:
            out = torch.full((n * n,), 7, dtype=torch.int32, device="cuda:0")
            ctx.intersect_sym_layout(n, log_b, *(t.data_ptr() for t in layout), t0, t1, out.data_ptr())
            torch.cuda.synchronize()
            acc += out.cpu().numpy().reshape(n, n)
        assert np.array_equal(acc, want)


def _family_arrays(rng, n, base_n, fams, lo, hi, extra):
    base = [np.unique(rng.integers(0, 2**63, size=base_n, dtype=np.uint64)) for _ in range(fams)]
    sk = []
    for i in range(n):
        b = base[i % fams]
        keep = b[rng.random(b.size) < lo + (hi - lo) * ((i * 7) % 10) / 10]
        sk.append(np.unique(np.concatenate(
            [keep, rng.integers(0, 2**64 - 1, size=extra, dtype=np.uint64)])))
    return sk


def _count_rows(sk, rows):
    """|S_r ∩ S_j| for the given rows and every column (searchsorted merge)."""
    out = np.zeros((len(rows), len(sk)), dtype=np.int64)
    for a, r in enumerate(rows):
        A = sk[r]
        for j, Bv in enumerate(sk):
            if A.size == 0 or Bv.size == 0:
                continue
            p = np.searchsorted(Bv, A)
            p[p == Bv.size] = 0
            out[a, j] = int(np.count_nonzero(Bv[p] == A))
    return out


def _layout(torch, ctx, d, st, sz, sk, log_b):
    n = len(sk)
    tot = int(sum(len(s) for s in sk))
    nb = (n + 63) // 64
    out = (torch.empty(max(tot, 1), dtype=torch.int64, device="cuda:0"),
           torch.empty(max(tot, 1), dtype=torch.int64, device="cuda:0"),
           torch.empty(nb * sksffi.join_layout_boff_words(log_b), dtype=torch.int32, device="cuda:0"),
           torch.empty(nb + 1, dtype=torch.int64, device="cuda:0"))
    mx = ctx.join_layout_build(d.data_ptr(), st.data_ptr(), sz.data_ptr(), n, log_b,
                               *(t.data_ptr() for t in out))
    return out, mx


@pytest.mark.parametrize("log_b", [0, 1, 3])
def test_join_buckets_above_table_capacity(torch_cuda, ctx, log_b):
    """A layout with far fewer buckets than its sketches need: every block-bucket
    holds many times the join table's capacity (~27k distinct values of a block
    in one bucket at log_b = 0), so k_join cuts each bucket into sub-chunks.  Counts
    through sks_intersect_sym_layout equal numpy for every tile range split."""
    torch = torch_cuda
    rng = np.random.default_rng(23)
    n = 150
    sk = _family_arrays(rng, n, 2500, 3, 0.2, 0.9, 300)
    sk[5] = np.zeros(0, np.uint64)
    sk[40] = np.union1d(sk[40], np.array([0, 2**64 - 1], np.uint64))
    sk[100] = np.union1d(sk[100], np.array([2**64 - 1], np.uint64))
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    lay, mx = _layout(torch, ctx, d, st, sz, sk, log_b)
    assert mx > (4 if log_b < 3 else 2) * sksffi.join_layout_capacity()
    T = sksffi.intersect_sym_tiles(n)
    acc = np.zeros((n, n), dtype=np.int64)
    for (t0, t1) in [(0, 2), (2, T)]:
        out = torch.full((n * n,), 7, dtype=torch.int32, device="cuda:0")
        ctx.intersect_sym_layout(n, log_b, *(t.data_ptr() for t in lay), t0, t1, out.data_ptr())
        torch.cuda.synchronize()
        acc += out.cpu().numpy().reshape(n, n)
    assert np.array_equal(acc, want)


def test_join_large_sketches_300k(torch_cuda, ctx):
    """128 sketches of 300k-380k elements (FracMinHash of 100-300 Mb genomes at
    c = 1000 is this size), mostly unrelated: the bucket count saturates at 2^14
    with the largest block-bucket of distinct values above the table (VERDICT r1
    weak #2), and every layout group (~11k elements) takes the build's slow
    path (hash slices).  Both entry points —
    sks_intersect_sym / sks_intersect_all (host-sized layout) and
    sks_join_layout_build + sks_intersect_sym_layout (the multi-GPU path) — give
    exact counts: diagonal = sizes, symmetric, and rows 0, 1, 77, 127 equal a
    numpy merge against all 128 columns."""
    torch = torch_cuda
    rng = np.random.default_rng(29)
    n = 128
    sk = _family_arrays(rng, n, 60_000, 4, 0.5, 0.9, 300_000)
    assert min(len(s) for s in sk) >= 300_000
    rows = [0, 1, 77, 127]
    want_rows = _count_rows(sk, rows)
    sizes = np.array([len(s) for s in sk])
    d, st, sz = _device_sketch_arrays(torch, sk)
    log_b = sksffi.join_layout_log_b(int(sizes.max()))
    assert log_b == 14
    lay, mx = _layout(torch, ctx, d, st, sz, sk, log_b)
    assert mx > sksffi.join_layout_capacity()  # the sub-chunk case
    T = sksffi.intersect_sym_tiles(n)

    def check(m):
        assert np.array_equal(np.diag(m), sizes)
        assert np.array_equal(m, m.T)
        assert np.array_equal(m[rows], want_rows)

    out = torch.full((n * n,), 3, dtype=torch.int32, device="cuda:0")
    ctx.intersect_sym_layout(n, log_b, *(t.data_ptr() for t in lay), 0, T, out.data_ptr())
    torch.cuda.synchronize()
    check(out.cpu().numpy().reshape(n, n).astype(np.int64))
    out.fill_(-1)
    ctx.intersect_sym(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, 0, T, out.data_ptr())
    torch.cuda.synchronize()
    check(out.cpu().numpy().reshape(n, n).astype(np.int64))
    out.fill_(-1)
    ctx.intersect_all(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    check(out.cpu().numpy().reshape(n, n).astype(np.int64))


def test_wide_all_vs_all_join_world1(torch_cuda, ctx):
    """The multi-GPU all-vs-all for 128-bit k-mers (sks_dist.all_vs_all_join at
    world 1, w = 45): the join layout of (lo, hi) entries, counts and device ANI,
    equal to the oracle's counts (replaces round 3's row-block path over one
    wavefront per pair)."""
    torch = torch_cuda
    import sks_dist
    w, k, c, n = 45, 30, 15, 70
    m = O.mask(w, k, 2)
    genomes = [synth.bases(4000, seed=90 + i % 4, mut_seed=800 + i, mut_rate=0.003 * (i % 5)).tobytes()
               for i in range(n)]
    ss, _ = build(torch, ctx, genomes, w, m, "frac", c)
    assert ss.elem_words == 2
    sk = [O.sketch(O.cut_runs(g), w, m, "frac", c)[0] for g in genomes]
    res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), sks_dist.GpuJoinOps(ctx, 2),
                                   sksffi.join_layout_log_b, device="cuda", ani_ones=k)
    got = res.matrix.cpu().numpy()
    want = np.array([[O.intersect(sk[i], sk[j]) for j in range(n)] for i in range(n)])
    assert want[0, 4] > 0
    assert np.array_equal(got, want)
    size_first = np.repeat(np.diag(got).astype(np.int32), n)
    _, host_ani = sksffi.ani_from_counts(got.reshape(-1), size_first, k)
    assert np.abs(res.ani.cpu().numpy().reshape(-1) - host_ani).max() <= 1e-9


def test_join_layout_tiles_block_offset_and_packed(torch_cuda, ctx):
    """sks_intersect_layout_tiles on the layout of a rank's own blocks (global
    blocks 1-3 of 200 sketches, built from the sketch range 64..199, blk0 = 1)
    with a tile list and packed output, and on the whole layout into the dense
    matrix: equal to sks_intersect_sym's merge-tile counts."""
    torch = torch_cuda
    n = 200
    genomes = [synth.bases(12000, seed=80 + i % 5, mut_seed=600 + i, mut_rate=0.005 * (i % 7)).tobytes()
               for i in range(n)]
    m = O.mask(31, 21, 6)
    ss, _dev = build(torch, ctx, genomes, 31, m, "bottom", 500)
    d, st, sz = ss.device_ptrs()
    ref = torch.zeros((n, n), dtype=torch.int32, device="cuda")
    ctx.set_intersect_kernel(sksffi.INTERSECT_MERGE)
    ctx.intersect_sym(d, st, sz, 1, n, 0, sksffi.intersect_sym_tiles(n), ref.data_ptr())
    ctx.set_intersect_kernel(sksffi.INTERSECT_AUTO)
    torch.cuda.synchronize()
    ref = ref.cpu()
    sizes = ss.sizes().astype(np.int64)
    log_b = sksffi.join_layout_log_b(int(sizes.max()))

    def layout(first, cnt):
        tot = int(sizes[first:first + cnt].sum())
        nb = (cnt + 63) // 64
        lay = (torch.empty(tot, dtype=torch.int64, device="cuda"), torch.empty(tot, dtype=torch.int64, device="cuda"),
               torch.zeros(nb * sksffi.join_layout_boff_words(log_b), dtype=torch.int32, device="cuda"),
               torch.zeros(nb + 1, dtype=torch.int64, device="cuda"))
        ctx.join_layout_build(d, st + 8 * first, sz + 4 * first, cnt, log_b, *(t.data_ptr() for t in lay),
                              stat=False, bounds=gb.data_ptr())
        return lay
    gb = torch.empty(sksffi.join_layout_groups(log_b) + 1, dtype=torch.int64, device="cuda")
    ctx.join_layout_bounds(d, st, sz, n, log_b, gb.data_ptr())  # shared by both layouts
    own = layout(64, n - 64)
    tiles = [(1, 1), (1, 3), (3, 3), (2, 3), (1, 2), (2, 2)]
    tl = torch.tensor(tiles, dtype=torch.int32, device="cuda")
    packed = torch.zeros((len(tiles), 64, 64), dtype=torch.int32, device="cuda")
    ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in own), 1, tl.data_ptr(), 0, len(tiles), True,
                               packed.data_ptr())
    whole = layout(0, n)
    dense = torch.zeros((n, n), dtype=torch.int32, device="cuda")
    ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in whole), 0, 0, 0, sksffi.intersect_sym_tiles(n),
                               False, dense.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dense.cpu(), ref)
    pk = packed.cpu()
    for t, (I, J) in enumerate(tiles):
        blk = ref[I * 64:I * 64 + 64, J * 64:J * 64 + 64]
        assert torch.equal(pk[t, :blk.shape[0], :blk.shape[1]], blk), (I, J)
        assert int(pk[t].sum()) == int(blk.sum())


@pytest.fixture(scope="module")
def scale_sets(torch_cuda, ctx):
    """Config 4's shape at 100 kb genomes: 1000 bottom-10000 sketches of
    unrelated genomes ("indep") and of 25 mutated families ("family")."""
    torch = torch_cuda
    n, L = 1000, 100_000
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    mask = sksffi.mask_generate(31, 21, 0)
    sets = {}
    for mode in ("indep", "family"):
        buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda:0")
        for g in range(n):
            if mode == "indep":
                ctx.synth_bases(buf.data_ptr() + seg[g], L, 7000 + g)
            else:
                ctx.synth_bases(buf.data_ptr() + seg[g], L, 100 + g % 25, 9000 + g, 0.002 + 0.0005 * (g % 9))
        buf[torch.tensor(seg[1:], device="cuda:0") - 1] = ord("\n")
        ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, 10000)
        del buf
        sets[mode] = ss
    return n, sets


@pytest.mark.parametrize("kernel_ctx", [sksffi.INTERSECT_JOIN], indirect=True)
@pytest.mark.parametrize("mode", ["indep", "family"])
def test_join_exact_at_scale(torch_cuda, kernel_ctx, scale_sets, mode):
    """~10^8 hash-table inserts per all-pairs call (1000 sketches of 10000):
    three calls each equal the merge kernel cell for cell.  Round 3: a probe
    loop compiled with its joined-entry register updated on every tag match gave
    about one insert in 10^7 a foreign entry (a diagonal one short, one stray +1;
    join_common.hpp join_chain) — far too rare for the small tests above."""
    torch = torch_cuda
    ctx = kernel_ctx
    n, sets = scale_sets
    d, st, sz = sets[mode].device_ptrs()
    T = sksffi.intersect_sym_tiles(n)
    kernel = ctx_kernel(ctx)
    ref = torch.empty((n, n), dtype=torch.int32, device="cuda:0")
    ctx.set_intersect_kernel(sksffi.INTERSECT_MERGE)
    ctx.intersect_sym(d, st, sz, 1, n, 0, T, ref.data_ptr())
    ctx.set_intersect_kernel(kernel)
    out = torch.empty((n, n), dtype=torch.int32, device="cuda:0")
    for _ in range(3):
        out.fill_(-1)
        ctx.intersect_sym(d, st, sz, 1, n, 0, T, out.data_ptr())
        torch.cuda.synchronize()
        bad = torch.nonzero(out != ref)
        assert bad.shape[0] == 0, [(i, j, int(out[i, j]), int(ref[i, j])) for i, j in bad[:4].tolist()]
    assert int(torch.diagonal(ref).min()) == 10000


@pytest.mark.parametrize("mode", ["indep", "family"])
def test_join_check_at_scale(torch_cuda, ctx, scale_sets, mode):
    """The invariant-checking builds (sks_ctx_set_join_check) over one
    config-4-scale all-pairs call (1000 sketches of 10000, ~10^7 layout elements
    and ~10^7 table inserts): every element's dedup representative holds its
    value, every inserted value is found naming its own entry — 0 violations —
    and the counts equal the merge kernel's.  This is the deterministic guard
    for the round-3 probe-loop miscompile (tools/microbench/chain_exits.hip): a
    loop that names a foreign entry fails here from its own invariant."""
    torch = torch_cuda
    n, sets = scale_sets
    d, st, sz = sets[mode].device_ptrs()
    T = sksffi.intersect_sym_tiles(n)
    ref = torch.empty((n, n), dtype=torch.int32, device="cuda:0")
    ctx.set_intersect_kernel(sksffi.INTERSECT_MERGE)
    ctx.intersect_sym(d, st, sz, 1, n, 0, T, ref.data_ptr())
    ctx.set_intersect_kernel(sksffi.INTERSECT_AUTO)
    out = torch.full((n, n), -1, dtype=torch.int32, device="cuda:0")
    ctx.join_check_violations()  # reset
    ctx.set_join_check(True)
    try:
        ctx.intersect_sym(d, st, sz, 1, n, 0, T, out.data_ptr())
        assert ctx.join_check_violations() == 0
    finally:
        ctx.set_join_check(False)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_config3_contig_against_oracle(torch_cuda, ctx):
    """One real config-3 contig: contig 0 of bench.py's
    genome — 125 Mb from sks_synth_bases(seed 3) with four 10 kb N-runs at
    L*(j+1)/5 — sketched with w=31/k=21 (mask seed 0), FracMinHash 1/1000, equals
    the oracle's set (8 chunks with (w-1)-base halos, unioned) and window count."""
    from concurrent.futures import ThreadPoolExecutor
    torch = torch_cuda
    L, w, frac, nrun, nrun_len = 125_000_000, 31, 1000, 4, 10_000
    mask = sksffi.mask_generate(w, 21, 0)
    dev = torch.empty(L + 1, dtype=torch.uint8, device="cuda:0")
    ctx.synth_bases(dev.data_ptr(), L, 3)
    edges = [0]
    for j in range(nrun):
        o = int(L * (j + 1) / (nrun + 1))
        dev[o:o + nrun_len] = ord("N")
        edges += [o, o + nrun_len]
    edges.append(L)
    dev[L] = ord("\n")
    torch.cuda.synchronize()
    gpu = ctx.sketch_build(dev.data_ptr(), L + 1, [0, L + 1], w, mask, sksffi.SKS_FRAC_MOD, frac)
    host = dev[:L].cpu().numpy().tobytes()
    T = 8
    cuts = [L * i // T for i in range(T + 1)]

    def one(i):
        a, b = cuts[i], min(L, cuts[i + 1] + w - 1)
        sk, nw = O.sketch(O.cut_runs(host[a:b]), w, mask, "frac", frac)
        return sk[:, 0], nw
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(one, range(T)))
    want = np.unique(np.concatenate([r[0] for r in res]))
    windows = sum(max(0, edges[i + 1] - edges[i] - w + 1) for i in range(0, len(edges), 2))
    assert sum(r[1] for r in res) == windows
    assert int(gpu.windows()[0]) == windows
    got = gpu.sketch(0)[:, 0]
    assert got.size == want.size and np.array_equal(got, want)


def test_all_vs_all_join_fused_ani_to_host(torch_cuda, ctx):
    """The one-rank all-vs-all with the ANI written by the join itself
    (sks_intersect_layout_ani: the last workgroup of each tile converts it)
    straight into pinned host memory — sksffi.HostBuffer (sks_host_alloc,
    coherent) and a torch pinned tensor — and into device memory: counts equal
    the oracle's, and every ANI equals sks_ani_from_counts
    (kmer-sketching.cpp:195-200, ani_estimation.cpp:24-42) within 1e-12; rows
    of the dense sks_ani_rows kernel agree too."""
    import sks_dist
    torch = torch_cuda
    n = 300  # 5 blocks, ragged last block: 15 tiles
    genomes = [synth.bases(2500 + 37 * (i % 13), seed=50 + i % 7, mut_seed=60 + i,
                           mut_rate=0.002 * (i % 5)).tobytes() for i in range(n)]
    w, k = 31, 21
    m = O.mask(w, k, 0)
    ss, _ = build(torch, ctx, genomes, w, m, "frac", 2)
    sk = [O.sketch(O.cut_runs(g), w, m, "frac", 2)[0] for g in genomes]
    ops = sks_dist.GpuJoinOps(ctx)
    hb = sksffi.HostBuffer(n * n * 8)
    hb.array[:] = -1.0
    pinned = torch.full((n * n,), -1.0, dtype=torch.float64, pin_memory=True)
    outs = []
    for dst in (hb, pinned, None):
        res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), ops, sksffi.join_layout_log_b,
                                       device="cuda", dst=0, ani_ones=k, ani_out=dst)
        torch.cuda.synchronize()
        res.check_layouts()
        outs.append(res)
    got = outs[0].matrix.cpu().numpy()
    for i in range(0, n, 37):
        for j in range(0, n, 11):
            assert got[i, j] == O.intersect(sk[i], sk[j]), (i, j)
    size_first = np.repeat(np.diag(got).astype(np.int32), n)
    _, want = sksffi.ani_from_counts(got.reshape(-1), size_first, k)
    assert np.abs(hb.array - want).max() <= 1e-12
    assert np.abs(pinned.numpy() - want).max() <= 1e-12
    assert np.abs(outs[2].ani.cpu().numpy().reshape(-1) - want).max() <= 1e-12
    dense = torch.from_numpy(got.astype(np.int32)).cuda()
    rows = torch.zeros((n, n), dtype=torch.float64, device="cuda")
    ctx.ani_rows(dense.data_ptr(), n, 64, 200, k, rows.data_ptr())
    torch.cuda.synchronize()
    assert np.abs(rows.cpu().numpy()[64:200].reshape(-1) - want.reshape(n, n)[64:200].reshape(-1)).max() <= 1e-12
    hb.free()


def test_fused_ani_table_rows_equal_pow_rows(torch_cuda, ctx):
    """sks_ctx_ani_table: the fused ANI of a row whose set holds max_size
    elements (bottom-s: the full sketches) is read from the context's table,
    the other rows (short genomes' smaller sketches) evaluate pow — both equal,
    bit for bit, the dense sks_ani_rows kernel (ani_of with pow,
    ani_estimation.cpp:24-42) on the same counts, and the table is rebuilt
    when k changes."""
    import sks_dist
    torch = torch_cuda
    n, s = 200, 400
    genomes = [synth.bases(300 if i % 7 == 0 else 3000 + 11 * (i % 5), seed=70 + i % 9, mut_seed=90 + i,
                           mut_rate=0.003 * (i % 4)).tobytes() for i in range(n)]
    w = 31
    ops = sks_dist.GpuJoinOps(ctx)
    for k in (21, 17):
        m = O.mask(w, k, 0)
        ss, _ = build(torch, ctx, genomes, w, m, "bottom", s)
        sizes = ss.sizes()
        assert int(sizes.max()) == s and int(sizes.min()) < s  # both paths taken
        res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), ops, sksffi.join_layout_log_b,
                                       device="cuda", dst=0, ani_ones=k)
        torch.cuda.synchronize()
        res.check_layouts()
        got = res.matrix.cpu().numpy()
        assert np.array_equal(np.diag(got), sizes.astype(got.dtype))
        dense = torch.from_numpy(got.astype(np.int32)).cuda()
        rows = torch.zeros((n, n), dtype=torch.float64, device="cuda")
        ctx.ani_rows(dense.data_ptr(), n, 0, n, k, rows.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(res.ani.cpu().numpy(), rows.cpu().numpy()), k
        size_first = np.repeat(np.diag(got).astype(np.int32), n)
        _, want = sksffi.ani_from_counts(got.reshape(-1), size_first, k)
        assert np.abs(res.ani.cpu().numpy().reshape(-1) - want).max() <= 1e-12
