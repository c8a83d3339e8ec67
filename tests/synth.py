"""Synthetic genomes shared by the tests, the golden-fixture script and bench.py.

base(p) = splitmix64 output p of a stream seeded with `seed`, top two bits
(0..3 -> A C G T).  With a mutation rate r, position p mutates when
splitmix64_at(mut_seed, p) < r * 2^64, to (base + 1 + (u >> 32) % 3) & 3.
libsks.so's sks_synth_bases (post.hip k_synth) computes the same bytes on the
device; tests/test_gpu_parity.py checks the two agree.
"""
import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def splitmix64_at(seed, p):
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.asarray(p, dtype=np.uint64) + np.uint64(1)) * GOLD
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def mut_threshold(rate):
    if rate <= 0:
        return 0
    t = int(rate * 2.0**64)
    return min(t, 2**64 - 1)


def bases(n, seed, mut_seed=0, mut_rate=0.0, pos_offset=0, chunk=1 << 24):
    """n ASCII bytes (uint8 array)."""
    out = np.empty(n, dtype=np.uint8)
    thr = np.uint64(mut_threshold(mut_rate))
    for o in range(0, n, chunk):
        p = np.arange(pos_offset + o, pos_offset + min(n, o + chunk), dtype=np.uint64)
        b = splitmix64_at(seed, p) >> np.uint64(62)
        if mut_rate > 0:
            u = splitmix64_at(mut_seed, p)
            hit = u < thr
            b = np.where(hit, (b + np.uint64(1) + (u >> np.uint64(32)) % np.uint64(3)) & np.uint64(3), b)
        out[o:o + len(p)] = ACGT[b.astype(np.int64)]
    return out


def fasta_text(records, width=80):
    """records: list of (name, bytes) -> FASTA bytes with `width`-column lines."""
    parts = []
    for name, seq in records:
        parts.append(b">" + name.encode() + b"\n")
        for i in range(0, len(seq), width):
            parts.append(bytes(seq[i:i + width]) + b"\n")
    return b"".join(parts)
