"""GPU parity of the deduplicated join layout (layout.hip) and the join kernel
over it (join.hip): 128-bit k-mers (32 < w <= 64) through the tiled join, the
layout build's slow path and slice splits (forced with a small
SKS_LAYOUT_GROUP_CAP), and the instrumented check kernels at config-4 scale
(kmer_set.cpp:23-41, 143-184: every count equals the reference's)."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sksffi  # noqa: E402
import pyoracle as O  # noqa: E402
import synth  # noqa: E402
from test_gpu_parity import build, _device_sketch_arrays, torch_cuda, ctx  # noqa: E402,F401

pytestmark = pytest.mark.gpu


def _all_ways(torch, ctx, d, st, sz, ew, n, split=True):
    """all-pairs via sks_intersect_all (whole and two row blocks, one unaligned)
    and sks_intersect_sym split into two tile ranges (one range for the global
    kernel, which takes no partial tile ranges)"""
    out = torch.full((n * n,), -3, dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(d, st, sz, ew, n, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    res = [out.cpu().numpy().reshape(n, n)]
    rows = []
    for r0, r1 in ((0, 70), (70, n)):
        o = torch.full(((r1 - r0) * n,), -5, dtype=torch.int32, device="cuda:0")
        ctx.intersect_all(d, st, sz, ew, n, r0, r1, o.data_ptr())
        torch.cuda.synchronize()
        rows.append(o.cpu().numpy().reshape(r1 - r0, n))
    res.append(np.concatenate(rows))
    T = sksffi.intersect_sym_tiles(n)
    acc = np.zeros((n, n), dtype=np.int64)
    for a, b in (((0, 2), (2, T)) if split else ((0, T),)):
        o = torch.full((n * n,), 9, dtype=torch.int32, device="cuda:0")
        ctx.intersect_sym(d, st, sz, ew, n, a, b, o.data_ptr())
        torch.cuda.synchronize()
        acc += o.cpu().numpy().reshape(n, n)
    res.append(acc)
    return res


@pytest.mark.parametrize("w,k", [(45, 30), (33, 33), (64, 40)])
def test_wide_join_matches_oracle(torch_cuda, ctx, w, k):
    """130 genomes in 5 families at 32 < w <= 64: the 128-bit join (layout of
    (lo, hi) entries, sym tiles and row blocks) equals the oracle's counts, as
    does the one-wavefront-per-pair kernel."""
    torch = torch_cuda
    n = 130
    genomes = [synth.bases(3000 + 53 * (i % 11), seed=40 + i % 5, mut_seed=300 + i,
                           mut_rate=0.004 * (i % 6)).tobytes() if i % 29 else b"" for i in range(n)]
    m = O.mask(w, k, 1)
    ss, _ = build(torch, ctx, genomes, w, m, "frac", 4)
    assert ss.elem_words == 2
    sk = [O.sketch(O.cut_runs(g), w, m, "frac", 4)[0] for g in genomes]
    want = np.array([[O.intersect(sk[i], sk[j]) for j in range(n)] for i in range(n)])
    assert want[1, 6] > 0 and want[0].sum() == 0  # genome 0 is empty
    d, st, sz = ss.device_ptrs()
    for kind in (sksffi.INTERSECT_AUTO, sksffi.INTERSECT_GLOBAL):
        ctx.set_intersect_kernel(kind)
        try:
            for got in _all_ways(torch, ctx, d, st, sz, 2, n, split=kind != sksffi.INTERSECT_GLOBAL):
                assert np.array_equal(got, want), kind
        finally:
            ctx.set_intersect_kernel(sksffi.INTERSECT_AUTO)


def _wide_arrays(rng, n, base_n, fams, extra):
    """sorted unique (lo, hi) arrays [k, 2] (hi-major) of related families"""
    out = []
    base = []
    for _ in range(fams):
        v = rng.integers(0, 2**63, size=(base_n, 2), dtype=np.uint64)
        base.append(v)
    for i in range(n):
        b = base[i % fams]
        keep = b[rng.random(len(b)) < 0.3 + 0.6 * ((i * 7) % 10) / 10]
        ex = rng.integers(0, 2**63, size=(extra, 2), dtype=np.uint64)
        a = np.unique(np.concatenate([keep, ex]), axis=0)
        a = a[np.lexsort((a[:, 0], a[:, 1]))]
        out.append(a)
    return out


def _wide_count(a, b):
    va = a.view([("lo", np.uint64), ("hi", np.uint64)]).reshape(-1)
    vb = b.view([("lo", np.uint64), ("hi", np.uint64)]).reshape(-1)
    return np.intersect1d(va, vb, assume_unique=True).size


@pytest.mark.parametrize("gcap", [None, "64"])
def test_wide_join_caller_arrays_and_slow_path(torch_cuda, ctx, monkeypatch, gcap):
    """Caller-provided 128-bit arrays whose words differ in either half (so a
    hi- or lo-only comparison would miscount), 150 sketches in 3 families, with
    the layout's fast path and (group cap 64) its slow path for every group."""
    torch = torch_cuda
    if gcap:
        monkeypatch.setenv("SKS_LAYOUT_GROUP_CAP", gcap)
    rng = np.random.default_rng(5)
    n = 150
    sk = _wide_arrays(rng, n, 1500, 3, 200)
    sk[7] = np.zeros((0, 2), np.uint64)
    # values equal in lo but not hi (and the reverse) across sketches
    sk[10] = np.concatenate([sk[10], np.array([[5, 2**63 + 1]], np.uint64)])
    sk[11] = np.concatenate([sk[11], np.array([[5, 2**63 + 2]], np.uint64)])
    for i in (10, 11):
        sk[i] = sk[i][np.lexsort((sk[i][:, 0], sk[i][:, 1]))]
    want = np.array([[_wide_count(sk[i], sk[j]) for j in range(n)] for i in range(n)])
    sizes = np.array([len(x) for x in sk], dtype=np.uint32)
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    flat = np.concatenate([x.reshape(-1) for x in sk] + [np.zeros(2, np.uint64)])
    d = torch.from_numpy(flat.view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    for got in _all_ways(torch, ctx, d.data_ptr(), st.data_ptr(), sz.data_ptr(), 2, n):
        assert np.array_equal(got, want)


@pytest.mark.parametrize("shape", ["identical", "families", "extremes"])
def test_layout_slow_path_slice_splits(torch_cuda, ctx, monkeypatch, shape):
    """Group cap 64: every layout group takes the slow path; identical sketches
    put 64 copies of each value in a slice, so slices split down to single
    values.  With the check kernels on, no invariant is violated and the counts
    equal numpy's."""
    torch = torch_cuda
    monkeypatch.setenv("SKS_LAYOUT_GROUP_CAP", "64")
    rng = np.random.default_rng({"identical": 1, "families": 2, "extremes": 3}[shape])
    n = 140
    if shape == "identical":
        one = np.unique(rng.integers(0, 2**64 - 1, size=3000, dtype=np.uint64))
        sk = [one.copy() for _ in range(n)]
    elif shape == "families":
        base = [np.unique(rng.integers(0, 2**62, size=3000, dtype=np.uint64)) for _ in range(3)]
        sk = [np.unique(np.concatenate([base[i % 3][rng.random(base[i % 3].size) < 0.5],
                                        rng.integers(0, 2**62, size=100, dtype=np.uint64)])) for i in range(n)]
    else:
        core = np.unique(np.concatenate([np.array([0, 1, 2**64 - 2, 2**64 - 1], np.uint64),
                                         rng.integers(0, 2**64 - 1, size=2000, dtype=np.uint64)]))
        sk = [core[rng.random(core.size) < 0.5] if i % 13 else np.zeros(0, np.uint64) for i in range(n)]
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    ctx.set_join_check(True)
    try:
        for got in _all_ways(torch, ctx, d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n):
            assert np.array_equal(got, want)
        assert ctx.join_check_violations() == 0
    finally:
        ctx.set_join_check(False)


@pytest.mark.parametrize("shape", ["one_bucket", "gcap256"])
def test_layout_bucket_passes(torch_cuda, ctx, monkeypatch, shape):
    """Inputs that leave the layout build's normal path but not its register
    and bucket-pass paths.  one_bucket (default group cap): every value hashes
    into the same bucket of its value group (the top bits of
    v * 0x9E3779B97F4A7C15, layout.hip kv_mix), so that bucket's table region
    (512 of the 4096 slots) overflows and the group is redone in bucket passes.
    gcap256: group cap 256 with groups of ~750 elements in 3 families, so
    groups are placed in passes of consecutive buckets holding <= 256 elements,
    re-read from the sketches.  With the check kernels on, no invariant is
    violated and the counts equal numpy's."""
    torch = torch_cuda
    rng = np.random.default_rng({"one_bucket": 11, "gcap256": 12}[shape])
    n = 140
    if shape == "one_bucket":
        pool = rng.integers(0, 2**64 - 1, size=4_000_000, dtype=np.uint64)
        with np.errstate(over="ignore"):
            pool = pool[(pool * np.uint64(0x9E3779B97F4A7C15)) >> np.uint64(61) == 0]
        pool = np.unique(pool)[:200_000]
        sk = [np.unique(pool[rng.integers(0, pool.size, size=1500)]) for _ in range(n)]
    else:
        monkeypatch.setenv("SKS_LAYOUT_GROUP_CAP", "256")
        base = [np.unique(rng.integers(0, 2**62, size=3000, dtype=np.uint64)) for _ in range(3)]
        sk = [np.unique(np.concatenate([base[i % 3][rng.random(base[i % 3].size) < 0.9],
                                        rng.integers(0, 2**62, size=100, dtype=np.uint64)])) for i in range(n)]
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    ctx.set_join_check(True)
    try:
        for got in _all_ways(torch, ctx, d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n):
            assert np.array_equal(got, want)
        assert ctx.join_check_violations() == 0
    finally:
        ctx.set_join_check(False)


def test_layout_pass_splits_u64(torch_cuda, ctx):
    """u64 layout passes that overflow the 2048-slot value table and split
    (bucket halves, then hash slices): the group bounds come from the even
    sketches (the sampled ones, spread over the whole value range), while the
    odd sketches put 3000 values each into one narrow range, so one value group
    of each block holds ~96k distinct values.  Also the value 0 (the table's
    empty word) in some sketches.  With the check kernels on, no invariant is
    violated and the counts equal numpy's."""
    torch = torch_cuda
    rng = np.random.default_rng(21)
    n = 128
    sk = []
    for i in range(n):
        if i % 2 == 0:
            a = rng.integers(1, 2**62, size=3000, dtype=np.uint64)
        else:
            a = (np.uint64(2**40) + rng.integers(0, 2**20, size=3000, dtype=np.uint64))
        if i % 9 == 0:
            a = np.concatenate([a, np.zeros(1, np.uint64)])
        sk.append(np.unique(a))
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)]
                     for i in range(n)])
    d, st, sz = _device_sketch_arrays(torch, sk)
    ctx.set_join_check(True)
    try:
        for got in _all_ways(torch, ctx, d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n):
            assert np.array_equal(got, want)
        assert ctx.join_check_violations() == 0
    finally:
        ctx.set_join_check(False)


def test_layout_invalid_flag_reaches_all_vs_all(torch_cuda, ctx, monkeypatch):
    """128-bit values whose 64-bit layout mixes all collide (lo = C ^ (hi * K1 +
    K2), join_common.hpp kv_mix) fill a layout slice that no hash split can cut
    (group cap 64): the build sets status word 1 (layout invalid).
    sks_intersect_all retries and falls back to an exact kernel (counts equal
    numpy's); sks_dist.all_vs_all_join — the one-call native path and the
    layout-by-layout path — reports it through JoinResult.check_layouts
    (RuntimeError) instead of returning its counts silently."""
    import sks_dist
    torch = torch_cuda
    monkeypatch.setenv("SKS_LAYOUT_GROUP_CAP", "64")
    rng = np.random.default_rng(31)
    n = 70
    hi = np.arange(1000, 1300, dtype=np.uint64)
    with np.errstate(over="ignore"):
        lo = np.uint64(0x1234567) ^ (hi * np.uint64(0xC2B2AE3D27D4EB4F) + np.uint64(0x165667B19E3779F9))
    coll = np.stack([lo, hi], axis=1)
    sk = []
    for i in range(n):
        ex = rng.integers(2**40, 2**63, size=(300, 2), dtype=np.uint64)
        a = np.unique(np.concatenate([coll[rng.random(len(coll)) < 0.8], ex]), axis=0)
        sk.append(a[np.lexsort((a[:, 0], a[:, 1]))])
    want = np.array([[_wide_count(sk[i], sk[j]) for j in range(n)] for i in range(n)])
    sizes = np.array([len(x) for x in sk], dtype=np.uint32)
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    flat = np.concatenate([x.reshape(-1) for x in sk])
    d = torch.from_numpy(flat.view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    out = torch.full((n * n,), -3, dtype=torch.int32, device="cuda:0")
    ctx.intersect_all(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 2, n, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(n, n), want)
    src = sks_dist.Sketches(d, sz, 2, starts=st)
    ops = sks_dist.GpuJoinOps(ctx, ew=2)
    for native in (True, False):
        ops.no_native = not native
        res = sks_dist.all_vs_all_join(n, 1, 0, src, ops, sksffi.join_layout_log_b, device="cuda", dst=None,
                                       max_size=int(sizes.max()))
        with pytest.raises(RuntimeError, match="join layout"):
            res.check_layouts()
    ops.no_native = False


def test_layout_blocks_hint_sparse_rows(torch_cuda, ctx):
    """A layout over rows most of which are empty (a rank's exchange buffer: a
    slot per rank, only its own and its peers' rows filled) built with and
    without sks_ctx_set_layout_blocks_hint: the hint only sizes the build's
    regions, so the tiles among the filled blocks count the same — numpy's
    intersections — either way."""
    import sks_dist
    torch = torch_cuda
    rng = np.random.default_rng(41)
    n, filled = 640, (0, 3, 7)  # 10 blocks, three hold sketches
    base = [np.unique(rng.integers(0, 2**62, size=2500, dtype=np.uint64)) for _ in range(4)]
    sk = []
    for i in range(n):
        if i // 64 in filled:
            b = base[i % 4]
            sk.append(np.unique(np.concatenate([b[rng.random(b.size) < 0.6],
                                                rng.integers(0, 2**62, size=80, dtype=np.uint64)])))
        else:
            sk.append(np.zeros(0, np.uint64))
    d, st, sz = _device_sketch_arrays(torch, sk)
    src = sks_dist.Sketches(d, sz, 1, starts=st)
    ops = sks_dist.GpuJoinOps(ctx)
    log_b = sksffi.join_layout_log_b(max(len(x) for x in sk))
    tiles = np.array([[0, 0], [0, 3], [0, 7], [3, 3], [3, 7], [7, 7]], dtype=np.int64)
    got = []
    for hint in (0, len(filled)):
        lay = ops.build(src, log_b, None, ("hint", hint), blocks_hint=hint)
        out = ops.parts(len(tiles), "cuda")
        ops.count(n, log_b, lay, 0, lay, 0, tiles, out)
        torch.cuda.synchronize()
        got.append(out.cpu().numpy())
    assert np.array_equal(got[0], got[1])
    for t, (I, J) in enumerate(tiles):
        for r in range(0, 64, 7):
            for c in range(0, 64, 5):
                want = np.intersect1d(sk[I * 64 + r], sk[J * 64 + c], assume_unique=True).size
                assert got[1][t, r, c] == want, (I, J, r, c)


def test_join_plane_carry_out(torch_cuda, ctx):
    """Pairs sharing more values in one join workgroup's buckets than the
    bit-sliced counters hold (2^12 per workgroup: join.hip kPlanes) carry out
    of the top plane into the output: four sketches of up to 5 M values (two
    identical, a half, a partial overlap) counted by sks_all_pairs_ani (one
    k_join launch, ~4.9k shared values per workgroup on the identical pair)
    and sks_intersect_sym equal numpy's intersections (kmer_set.cpp:143-184)."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    a = np.unique(rng.integers(1, 2**63, size=5_100_000, dtype=np.uint64))[:5_000_000]
    other = np.unique(rng.integers(1, 2**63, size=2_000_000, dtype=np.uint64))
    d_part = np.unique(np.concatenate([a[1::3], other]))
    sk = [a, a.copy(), a[::2].copy(), d_part]
    n = len(sk)
    want = np.array([[np.intersect1d(sk[i], sk[j], assume_unique=True).size for j in range(n)] for i in range(n)])
    sizes = np.array([len(x) for x in sk], dtype=np.uint32)
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    flat = np.concatenate(sk + [np.zeros(1, np.uint64)])
    d = torch.from_numpy(flat.view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    cnt = torch.full((64 * 64,), -7, dtype=torch.int32, device="cuda:0")
    stat = torch.zeros(2, dtype=torch.int32, device="cuda:0")
    ctx.all_pairs_ani(d.data_ptr(), st.data_ptr(), sz.data_ptr(), n, int(sizes.max()), int(sizes.sum()), 21, 0,
                      cnt.data_ptr(), stat.data_ptr())
    torch.cuda.synchronize()
    assert int(stat.cpu()[1]) == 0
    got = cnt.cpu().numpy().reshape(64, 64)[:n, :n]
    assert want[0, 1] == 5_000_000 and np.array_equal(got, want)
    o = torch.full((n * n,), 9, dtype=torch.int32, device="cuda:0")
    ctx.intersect_sym(d.data_ptr(), st.data_ptr(), sz.data_ptr(), 1, n, 0, sksffi.intersect_sym_tiles(n), o.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(o.cpu().numpy().reshape(n, n), want)


def test_fused_ani_refuses_unmapped_host_memory(torch_cuda, ctx):
    """The fused ANI store runs inside k_join, so its destination must be device
    memory or pinned host memory mapped into the device.  An ordinary host
    buffer (numpy) is refused with SKS_E_ARG by both entry points that take it
    (sks_all_pairs_ani, sks_intersect_layout_ani) before any kernel runs, and the
    context still works afterwards."""
    import sks_dist
    torch = torch_cuda
    rng = np.random.default_rng(5)
    sk = [np.unique(rng.integers(1, 2**40, size=300, dtype=np.uint64)) for _ in range(3)]
    n = len(sk)
    sizes = np.array([len(x) for x in sk], dtype=np.uint32)
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    d = torch.from_numpy(np.concatenate(sk).view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    cnt = torch.zeros(64 * 64, dtype=torch.int32, device="cuda:0")
    host = np.zeros(n * n, dtype=np.float64)  # plain pageable memory
    with pytest.raises(sksffi.SksError) as e:
        ctx.all_pairs_ani(d.data_ptr(), st.data_ptr(), sz.data_ptr(), n, int(sizes.max()), int(sizes.sum()), 21,
                          host.ctypes.data, cnt.data_ptr(), 0)
    assert e.value.code == sksffi.SKS_E_ARG
    log_b = sksffi.join_layout_log_b(int(sizes.max()))
    ops = sks_dist.GpuJoinOps(ctx)
    lay = ops.build(sks_dist.Sketches(d, sz, 1, starts=st), log_b, None, "refuse")
    with pytest.raises(sksffi.SksError) as e:
        ctx.intersect_layout_ani(n, log_b, [t.data_ptr() for t in lay], 0, [t.data_ptr() for t in lay], 0, 0, 0,
                                 sksffi.intersect_sym_tiles(n), True, cnt.data_ptr(), sz.data_ptr(), 21,
                                 host.ctypes.data)
    assert e.value.code == sksffi.SKS_E_ARG
    # device memory is accepted and the counts are right
    ani = torch.zeros(n * n, dtype=torch.float64, device="cuda:0")
    ctx.all_pairs_ani(d.data_ptr(), st.data_ptr(), sz.data_ptr(), n, int(sizes.max()), int(sizes.sum()), 21,
                      ani.data_ptr(), cnt.data_ptr(), 0)
    torch.cuda.synchronize()
    got = cnt.cpu().numpy().reshape(64, 64)[:n, :n]
    want = np.array([[np.intersect1d(sk[i], sk[j]).size for j in range(n)] for i in range(n)])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("ew", [1, 2])
def test_layout_bounds_are_sample_medians(torch_cuda, ctx, ew):
    """k_gl_prep's group bounds: bounds[g] = the lower median over up to 64
    sample sketches (sketch lane * n / 64) of their element at g * size / G,
    bounds[0] = 0, bounds[G] = the largest value.  The values leave a gap
    (half of each sketch below 2^40, half above 2^62, as a spaced mask's
    masked-out positions do) and the sketch sizes differ, so a mean of the
    samples would land inside the gap; one sketch is empty (not sampled)."""
    torch = torch_cuda
    rng = np.random.default_rng(11)
    n, log_b = 100, 10
    G = sksffi.join_layout_groups(log_b)
    sk = []
    for i in range(n):
        m = 0 if i == 3 else 900 + 37 * (i % 13)
        lo = rng.integers(0, 2**40, size=m // 2, dtype=np.uint64)
        hi = rng.integers(2**62, 2**63, size=m - m // 2, dtype=np.uint64)
        v = np.concatenate([lo, hi])
        if ew == 1:
            a = np.unique(v).reshape(-1, 1)
        else:
            a = np.unique(np.stack([rng.integers(0, 2**64, size=m, dtype=np.uint64), v], 1), axis=0)
            a = a[np.lexsort((a[:, 0], a[:, 1]))]
        sk.append(a)
    sizes = np.array([len(x) for x in sk], dtype=np.uint32)
    starts = np.zeros(n, dtype=np.uint64)
    starts[1:] = np.cumsum(sizes[:-1], dtype=np.uint64)
    flat = np.concatenate([x.reshape(-1) for x in sk] + [np.zeros(2, np.uint64)])
    d = torch.from_numpy(flat.view(np.int64)).to("cuda:0")
    st = torch.from_numpy(starts.view(np.int64)).to("cuda:0")
    sz = torch.from_numpy(sizes.view(np.int32)).to("cuda:0")
    out = torch.zeros((G + 1) * ew, dtype=torch.int64, device="cuda:0")
    ctx.join_layout_bounds(d.data_ptr(), st.data_ptr(), sz.data_ptr(), n, log_b, out.data_ptr(), ew)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64).reshape(G + 1, ew)
    key = (lambda r: int(r[0])) if ew == 1 else (lambda r: (int(r[1]) << 64) | int(r[0]))
    lanes = [lane * n // 64 for lane in range(64)]
    assert [int(x) for x in got[0]] == [0] * ew and all(int(x) == 2**64 - 1 for x in got[G])
    for g in range(1, G):
        smp = sorted(key(sk[i][g * len(sk[i]) // G]) for i in lanes if len(sk[i]))
        assert key(got[g]) == smp[(len(smp) - 1) // 2], g
    # no group takes more than a few times its share of any sketch
    b = [key(got[g]) for g in range(G + 1)]
    worst = max(int(np.diff(np.searchsorted([key(r) for r in x], b)).max()) for x in sk if len(x))
    assert worst <= 4 * (sizes.max() // G + 1)
