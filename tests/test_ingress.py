"""Device FASTA ingress (ingress.hip, sks_fasta_parse_device) against the
oracle's strings_from_fasta (oracle/sks_oracle.cpp ora_fasta_records, which
restates fasta_processing.cpp:79-133 and is pinned against the reference's own
fasta_processing.cpp in test_oracle.py).

The CPU test checks the line-parallel formulation itself (the scans the
kernels run, restated in numpy) against the oracle, so the design is verified
without a GPU; the GPU tests run the kernels through the C ABI on the golden
edge-case corpus, fuzzed files, span-boundary cases and unaligned inputs.
"""
import os
import random

import numpy as np
import pytest

import pyoracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN_FASTA = os.path.join(ROOT, "tests", "golden", "fasta")


def oracle_stream(path):
    return b"".join(r + b"\n" for r in O.fasta_records(path))


def fuzz_fasta(rng, n_lines, long_every=0):
    """Random FASTA-ish bytes hitting every record rule."""
    parts = []
    for i in range(n_lines):
        r = rng.random()
        if r < 0.12:
            parts.append(b">" + bytes(rng.choice(b"abcXYZ_.|") for _ in range(rng.randrange(0, 12))))
        elif r < 0.15:
            parts.append(b">")
        elif r < 0.18:
            parts.append(b">name with space")
        elif r < 0.27:
            parts.append(b"")
        elif r < 0.31:
            parts.append(b"AC GT")
        elif r < 0.34:
            parts.append(b"ACGTN\r")
        elif r < 0.36:
            parts.append(b"AC\tGT")
        else:
            ln = rng.randrange(1, 90)
            if long_every and i % long_every == 0:
                ln = rng.randrange(5000, 20000)
            parts.append(bytes(rng.choice(b"ACGTacgtN") for _ in range(ln)))
    data = b"\n".join(parts)
    if rng.random() < 0.6:
        data += b"\n"
    return data


def line_parallel_model(data: bytes) -> bytes:
    """numpy restatement of ingress.hip's passes 1-8 (the design under test)."""
    raw = np.frombuffer(data, dtype=np.uint8)
    n = len(raw)
    if n == 0:
        return b""
    nl = np.flatnonzero(raw == 10)
    L = len(nl) + (raw[-1] != 10)
    starts = np.concatenate([[0], nl + 1])[:L]
    ends = np.concatenate([nl, [n]])[:L]
    lens = ends - starts
    has_space = np.zeros(L, bool)
    sp = np.flatnonzero(raw == 32)
    has_space[np.searchsorted(nl, sp, side="left")] = True
    first = np.where(lens > 0, raw[np.minimum(starts, n - 1)], 0)
    H = (lens > 0) & (first == ord(">"))
    E = lens == 0
    S = ~H & ~E
    Ssp = S & has_space
    setter = np.where(H, np.where(lens > 1, 2, 1), np.where(Ssp, 1, 0)).astype(np.uint8)
    event = np.where(H | E, 1, np.where(Ssp, 2, 0)).astype(np.uint8)

    def last_nonzero_scan(v):
        idx = np.where(v != 0, np.arange(len(v)), -1)
        idx = np.maximum.accumulate(idx)
        return np.where(idx >= 0, v[np.maximum(idx, 0)], 0)

    have_after = last_nonzero_scan(setter)
    nxt_rev = last_nonzero_scan(event[::-1])
    before = np.concatenate([[False], have_after[:-1] == 2])
    nxt = np.concatenate([nxt_rev[::-1][1:], [0]])  # first event strictly after l
    keep = S & ~Ssp & before & (nxt != 2)
    push = (H | E) & before
    out = bytearray()
    for l in range(L):
        if keep[l]:
            out += data[starts[l]:ends[l]]
        elif push[l]:
            out += b"\n"
    if have_after[-1] == 2:
        out += b"\n"
    return bytes(out)


def test_line_parallel_formulation_matches_oracle(tmp_path):
    files = sorted(os.listdir(GOLDEN_FASTA))
    rng = random.Random(7)
    cases = [(f, open(os.path.join(GOLDEN_FASTA, f), "rb").read()) for f in files]
    cases += [(f"fuzz{i}", fuzz_fasta(rng, rng.randrange(0, 60))) for i in range(300)]
    for name, data in cases:
        p = tmp_path / "x.fa"
        p.write_bytes(data)
        assert line_parallel_model(data) == oracle_stream(str(p)), name


# ---------------------------------------------------------------- GPU ------

@pytest.fixture(scope="module")
def gpu():
    import torch
    import sksffi
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    c = sksffi.Context(0)
    yield torch, c
    c.close()


def device_parse(torch, ctx, data: bytes, offset=0, with_rec=True):
    buf = torch.zeros(len(data) + offset + 16, dtype=torch.uint8)
    if data:
        buf[offset:offset + len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    d = buf.to("cuda:0")
    nb, nr = ctx.fasta_parse_device(d.data_ptr() + offset, len(data))
    out = torch.full((nb + 1,), 0xEE, dtype=torch.uint8, device="cuda:0")
    rec = torch.full((nr + 1,), -1, dtype=torch.int64, device="cuda:0")
    nb2, nr2 = ctx.fasta_parse_device(d.data_ptr() + offset, len(data), out.data_ptr(), nb,
                                      rec.data_ptr() if with_rec else None, nr)
    assert (nb2, nr2) == (nb, nr)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert o[nb] == 0xEE  # nothing written past the stream
    return o[:nb].tobytes(), rec.cpu().numpy()[:nr]


def check_case(torch, ctx, data, tmp_path, name, offset=0):
    p = tmp_path / "x.fa"
    p.write_bytes(data)
    want = oracle_stream(str(p))
    got, rec = device_parse(torch, ctx, data, offset)
    assert got == want, name
    ends = [i for i, b in enumerate(want) if b == 10]
    assert list(rec) == ends, name


@pytest.mark.gpu
def test_golden_corpus(gpu, tmp_path):
    torch, ctx = gpu
    for f in sorted(os.listdir(GOLDEN_FASTA)):
        data = open(os.path.join(GOLDEN_FASTA, f), "rb").read()
        for off in (0, 3):
            check_case(torch, ctx, data, tmp_path, f, off)


@pytest.mark.gpu
def test_fuzz(gpu, tmp_path):
    torch, ctx = gpu
    rng = random.Random(11)
    for i in range(150):
        data = fuzz_fasta(rng, rng.randrange(0, 400), long_every=rng.choice([0, 0, 37]))
        check_case(torch, ctx, data, tmp_path, f"fuzz{i}", offset=i % 16)


@pytest.mark.gpu
def test_span_boundaries(gpu, tmp_path):
    torch, ctx = gpu
    # 9000 newlines: spans holding 4097 lines
    check_case(torch, ctx, b">a\n" + b"\n" * 9000 + b"ACGT\n", tmp_path, "newlines")
    # one 3 MB line crossing hundreds of spans, headers on both sides
    rng = np.random.default_rng(5)
    seq = bytes(np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, 3_000_000)])
    for off in (0, 1, 15):
        check_case(torch, ctx, b">g1 x\n" + seq + b"\n>g2\nAC\n", tmp_path, "long", off)
    # lines of exactly span length, records ending at span edges
    for ln in (4095, 4096, 4097):
        body = b"\n".join(seq[i * ln:(i + 1) * ln] for i in range(6))
        check_case(torch, ctx, b">s\n" + body, tmp_path, f"ln{ln}")
    # a space line dropping a record that spans many spans
    check_case(torch, ctx, b">s\n" + seq[:50000] + b"\nA C\n" + seq[:100] + b"\n>t\nGG",
               tmp_path, "drop")


@pytest.mark.gpu
def test_empty_and_size_errors(gpu):
    torch, ctx = gpu
    import sksffi
    assert ctx.fasta_parse_device(0, 0) == (0, 0)
    d = torch.frombuffer(bytearray(b">a\nACGT\n>b\nGG\n"), dtype=torch.uint8).to("cuda:0")
    nb, nr = ctx.fasta_parse_device(d.data_ptr(), d.numel())
    assert (nb, nr) == (8, 2)
    out = torch.zeros(8, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(sksffi.SksError):
        ctx.fasta_parse_device(d.data_ptr(), d.numel(), out.data_ptr(), 7)
    rec = torch.zeros(2, dtype=torch.int64, device="cuda:0")
    with pytest.raises(sksffi.SksError):
        ctx.fasta_parse_device(d.data_ptr(), d.numel(), out.data_ptr(), 8, rec.data_ptr(), 1)
    ctx.fasta_parse_device(d.data_ptr(), d.numel(), out.data_ptr(), 8, rec.data_ptr(), 2)
    assert out.cpu().numpy().tobytes() == b"ACGT\nGG\n"
    assert list(rec.cpu().numpy()) == [4, 7]


@pytest.mark.gpu
def test_device_ingress_feeds_sketch_build(gpu, tmp_path):
    """raw FASTA bytes -> device stream -> sketch, equal to the oracle's sketch
    of the file (kmer_set_from_fasta_file, kmer_set.cpp:54-70)."""
    torch, ctx = gpu
    import sksffi
    path = os.path.join(GOLDEN_FASTA, "c1_10kb.fa")
    data = open(path, "rb").read()
    d = torch.frombuffer(bytearray(data), dtype=torch.uint8).to("cuda:0")
    nb, nr = ctx.fasta_parse_device(d.data_ptr(), len(data))
    out = torch.empty(nb, dtype=torch.uint8, device="cuda:0")
    ctx.fasta_parse_device(d.data_ptr(), len(data), out.data_ptr(), nb)
    m = O.mask(31, 21, 0)
    ss = ctx.sketch_build(out.data_ptr(), nb, [0, nb], 31, m, sksffi.SKS_FRAC_MOD, 20)
    want, nw = O.sketch(O.fasta_runs(path), 31, m, "frac", 20)
    assert np.array_equal(ss.sketch(0), want)
    assert int(ss.windows()[0]) == nw
