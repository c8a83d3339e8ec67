"""GPU parity at the benchmark's own sizes (BASELINE.json configs 4 and 5).

Config 4: 1000 synthetic 5 Mb genomes (10 ancestors x 100 mutated
descendants, bench.c4_genome_seeds), spaced seed w=31/k=21, bottom-s
s=10000, counted all-vs-all through exactly the path bench.py times
(sks_dist.all_vs_all_join over sks_join_layout_build +
sks_intersect_sym_layout, world 1).  Checked: 8 genomes' sketches against the
oracle (oracle/sks_oracle.cpp) on the same 5 Mb bytes; the whole 1000 x 1000
count matrix against an independent host count of the exported sketches
(sparse 0/1 membership product); symmetry and diagonal = sizes; the ANI the
join writes into pinned host memory against the host's.  The same at w = 45 /
k = 30 (128-bit k-mers, the bench's pairs_wide leg).

Config 5: mask seeds 0..7 over the first 200 genomes, per seed all-vs-all and
ANI (kmer-sketching.cpp:185-200), consensus = mean over seeds through
sks_dist.seed_sweep like bench.py.  Checked: 2 genomes per seed against the
oracle, each seed's matrix against the host count, and the consensus against a
host recomputation of containment / ANI from the exported sketches (<= 1e-12).
"""
import os
import sys

import numpy as np
import pytest

import pyoracle as O
import sksffi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import bench
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    ctx = sksffi.Context(0)
    yield torch, bench, ctx
    ctx.close()


def _genomes(torch, bench, ctx, n):
    L = bench.C4_LEN
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, ms, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, ms, r)
        buf[seg[g] + L] = ord("\n")
    torch.cuda.synchronize()
    return buf, seg


def _host_counts(sketches):
    """|S_i ∩ S_j| for all pairs from sorted u64 arrays: 0/1 membership rows over
    the union of values, multiplied (independent of every GPU kernel)."""
    import scipy.sparse as sp
    n = len(sketches)
    allv = np.concatenate(sketches)
    rows = np.repeat(np.arange(n), [len(s) for s in sketches])
    _, inv = np.unique(allv, return_inverse=True)
    M = sp.csr_matrix((np.ones(len(allv), np.int32), (rows, inv)), shape=(n, int(inv.max()) + 1))
    return (M @ M.T).toarray().astype(np.int64)


def _exported(ss, n):
    return [ss.sketch(i)[:, 0].copy() for i in range(n)]


def test_config4_all_vs_all_1000x5mb(env):
    torch, bench, ctx = env
    import sks_dist
    n, s = bench.C4_GENOMES, bench.C4_S
    buf, seg = _genomes(torch, bench, ctx, n)
    mask = sksffi.mask_generate(bench.W, bench.K, bench.MASK_SEED)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, bench.W, mask, sksffi.SKS_BOTTOM_S, s)
    sizes = ss.sizes().copy()
    assert (sizes == s).all()  # every 5 Mb genome has > 10000 distinct k-mers
    # sketches against the oracle on the same bytes: both ends of the family
    # structure (rates 0 and 9.9 %) in several families
    for g in (0, 1, 99, 100, 457, 501, 998, 999):
        raw = buf[seg[g]:seg[g + 1]].cpu().numpy().tobytes()
        want, nw = O.sketch(O.cut_runs(raw), bench.W, mask, "bottom", s)
        assert np.array_equal(ss.sketch(g), want), g
        assert int(ss.windows()[g]) == nw
    # the bench's pair path, world 1: counts, and the ANI the join writes into
    # pinned host memory
    ones = bin(mask).count("1") // 2
    hb = sksffi.HostBuffer(n * n * 8)
    res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), sks_dist.GpuJoinOps(ctx),
                                   sksffi.join_layout_log_b, device="cuda", ani_ones=ones, ani_out=hb,
                                   size_bound=s, max_size=int(sizes.max()))
    mat = res.matrix
    torch.cuda.synchronize()
    res.check_layouts()
    got = mat.cpu().numpy().astype(np.int64)
    want = _host_counts(_exported(ss, n))
    assert np.array_equal(got, got.T)
    assert np.array_equal(np.diag(got), sizes.astype(np.int64))
    assert np.array_equal(got, want)
    # the family structure is real: related pairs share k-mers, unrelated ones do not
    assert got[0, 1] > 0 and got[0, 50] > 0 and got[0, 999] < 50
    # device ANI of all 10^6 ordered pairs against the host's sks_ani_from_counts
    # (kmer-sketching.cpp:195-200, ani_estimation.cpp:24-42): within 1e-9
    size_first = np.repeat(np.diag(got).astype(np.int32), n)
    _, host_ani = sksffi.ani_from_counts(got.reshape(-1), size_first, ones)
    dev_ani = hb.array.copy()
    hb.free()
    assert np.abs(dev_ani - host_ani).max() <= 1e-9
    assert (dev_ani == host_ani).mean() > 0.99  # the device pow is within 1 ulp; nearly all bit-equal


def _host_counts_wide(sketches):
    """_host_counts for (lo, hi) 128-bit k-mers: rows over the union of values."""
    import scipy.sparse as sp
    n = len(sketches)
    allv = np.ascontiguousarray(np.concatenate(sketches)).view(np.dtype((np.void, 16))).reshape(-1)
    rows = np.repeat(np.arange(n), [len(s) for s in sketches])
    _, inv = np.unique(allv, return_inverse=True)
    M = sp.csr_matrix((np.ones(len(allv), np.int32), (rows, inv)), shape=(n, int(inv.max()) + 1))
    return (M @ M.T).toarray().astype(np.int64)


def test_config4_wide_all_vs_all_1000x5mb(env):
    """Config 4 at w = 45 / k = 30 — a (k + 10, k) shape of the reference's sweep
    (kmer-sketching.cpp:228-239), 128-bit k-mers — through the bench's
    pairs_wide path (sks_dist.all_vs_all_join with GpuJoinOps(ew = 2): the
    (lo, hi) join layout, k_join<2> and the fused ANI into pinned host memory):
    4 genomes' sketches against the oracle, the whole 1000 x 1000 matrix
    against a host count of the exported (lo, hi) sketches, every ANI within
    1e-9 of the host's."""
    torch, bench, ctx = env
    import sks_dist
    n, s, w, k = bench.C4_GENOMES, bench.C4_S, bench.C4W_W, bench.C4W_K
    buf, seg = _genomes(torch, bench, ctx, n)
    mask = sksffi.mask_generate(w, k, bench.MASK_SEED)
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, s)
    assert ss.elem_words == 2
    sizes = ss.sizes().copy()
    assert (sizes == s).all()
    for g in (0, 377, 640, 999):
        raw = buf[seg[g]:seg[g + 1]].cpu().numpy().tobytes()
        want, _ = O.sketch(O.cut_runs(raw), w, mask, "bottom", s)
        assert np.array_equal(ss.sketch(g), want), g
    ones = bin(mask).count("1") // 2
    hb = sksffi.HostBuffer(n * n * 8)
    res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), sks_dist.GpuJoinOps(ctx, 2),
                                   sksffi.join_layout_log_b, device="cuda", ani_ones=ones, ani_out=hb,
                                   size_bound=s, max_size=int(sizes.max()))
    torch.cuda.synchronize()
    res.check_layouts()
    got = res.matrix.cpu().numpy().astype(np.int64)
    want = _host_counts_wide([ss.sketch(i) for i in range(n)])
    assert np.array_equal(np.diag(got), sizes.astype(np.int64))
    assert np.array_equal(got, want)
    assert got[0, 1] > 0 and got[0, 999] < 50
    size_first = np.repeat(np.diag(got).astype(np.int32), n)
    _, host_ani = sksffi.ani_from_counts(got.reshape(-1), size_first, ones)
    assert np.abs(hb.array - host_ani).max() <= 1e-9
    hb.free()


def test_config5_seed_sweep_8x200x5mb(env):
    torch, bench, ctx = env
    import sks_dist
    n, s, seeds = bench.C5_GENOMES, bench.C4_S, bench.C5_SEEDS
    buf, seg = _genomes(torch, bench, ctx, n)
    padded = torch.full((n, s), -1, dtype=torch.int64, device="cuda")
    psizes = torch.zeros(n, dtype=torch.int32, device="cuda")
    starts = torch.arange(n, dtype=torch.int64, device="cuda") * s
    T = sksffi.intersect_sym_tiles(n)
    host_ani = []
    checked = {0: (3, 150), 1: (0, 199), 2: (42, 77), 3: (100, 101), 4: (5, 6), 5: (120, 180),
               6: (7, 190), 7: (60, 61)}

    def ani_for_seed(k):
        m = sksffi.mask_generate(bench.W, bench.K, k)
        ones = bin(m).count("1") // 2
        ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, bench.W, m, sksffi.SKS_BOTTOM_S, s)
        for g in checked[k]:
            raw = buf[seg[g]:seg[g + 1]].cpu().numpy().tobytes()
            want, _ = O.sketch(O.cut_runs(raw), bench.W, m, "bottom", s)
            assert np.array_equal(ss.sketch(g), want), (k, g)
        ss.export(padded.data_ptr(), s, psizes.data_ptr())
        mat = torch.empty((n, n), dtype=torch.int32, device="cuda")
        ctx.intersect_sym(padded.data_ptr(), starts.data_ptr(), psizes.data_ptr(), 1, n, 0, T,
                          mat.data_ptr())
        torch.cuda.synchronize()
        counts = mat.cpu().numpy()
        sk = _exported(ss, n)
        hc = _host_counts(sk)
        assert np.array_equal(counts.astype(np.int64), hc), k
        size_first = np.repeat(np.diag(counts).astype(np.int32), n)
        _, ani = sksffi.ani_from_counts(counts.reshape(-1), size_first, ones)
        # host recomputation (kmer-sketching.cpp:195-200, ani_estimation.cpp:24-42)
        sz = np.array([len(x) for x in sk], dtype=np.float64)
        cont = hc / sz[:, None]
        host_ani.append(np.where(cont > 0, np.power(cont, 1.0 / ones), 0.0))
        return torch.from_numpy(ani.reshape(n, n))

    cons, mine = sks_dist.seed_sweep(seeds, 1, 0, ani_for_seed, n, device="cpu")
    assert mine == list(range(seeds))
    want = sum(host_ani) / seeds
    assert np.allclose(cons.numpy(), want, rtol=0, atol=1e-12)
    c = cons.numpy()
    assert np.allclose(np.diag(c), 1.0) and 0 < c[0, 1] < 1 and c[0, 150] < c[0, 1]
