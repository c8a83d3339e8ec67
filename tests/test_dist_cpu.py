"""CPU (gloo, world_size 2 to 8): the multi-GPU orchestration of
spaced-kmer-sketching_amd/sks_dist.py — genome / block sharding, the cyclic
tile plan of all_vs_all_join and its three sketch exchanges (p2p send/recv,
one all-gather, per-source broadcasts), the padded-sketch gather of
all_vs_all, the seed sweep and the sharded genome — assembles exactly the
single-process result.  The kernels are replaced by numpy restatements of the
same contracts (sks_join_layout_build / sks_intersect_layout_ani /
sks_sketches_export, sks_intersect_sym)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import pyoracle as O
import sks_dist
import synth

N_GENOMES = 70   # two tile blocks, ragged
STRIDE = 400


def _sketches():
    m = O.mask(21, 21, 0)
    out = []
    for g in range(N_GENOMES):
        seq = synth.bases(6000, seed=40 + g % 4, mut_seed=300 + g, mut_rate=0.002 * (g % 9))
        sk, _ = O.sketch(O.cut_runs(seq.tobytes()), 21, m, "bottom", 300 - (g % 5) * 40)
        out.append(sk[:, 0].astype(np.int64))
    return out


def _oracle_count_sym(src, src_sz, n, t0, t1, out):
    out.zero_()
    sk = [src[i, : int(src_sz[i])].numpy().astype(np.uint64) for i in range(n)]
    for t in range(t0, t1):
        I, J = sks_dist.sym_tile_coords(t, n)
        for i in range(I * 64, min(n, I * 64 + 64)):
            for j in range(J * 64, min(n, J * 64 + 64)):
                c = O.intersect(np.stack([sk[i], 0 * sk[i]], 1), np.stack([sk[j], 0 * sk[j]], 1))
                out[i, j] = c
                out[j, i] = c


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sk = _sketches()
    per, g0, g1 = sks_dist.genome_shard(N_GENOMES, world, rank)
    local = torch.full((per, STRIDE), -1, dtype=torch.int64)
    local_sz = torch.zeros(per, dtype=torch.int32)
    for i, g in enumerate(range(g0, g1)):
        local[i, : len(sk[g])] = torch.from_numpy(sk[g])
        local_sz[i] = len(sk[g])
    mat = sks_dist.all_vs_all(local, local_sz, N_GENOMES, world, rank, _oracle_count_sym)
    q.put((rank, mat.numpy()))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_all_vs_all_gloo_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sk = _sketches()
    want = np.array([[len(np.intersect1d(sk[i], sk[j])) for j in range(N_GENOMES)]
                     for i in range(N_GENOMES)])
    for r in range(world):
        assert np.array_equal(results[r], want)


def test_shard_arithmetic():
    for n in (1, 63, 64, 65, 1000):
        T = sks_dist.sym_tiles(n)
        seen = []
        for world in (1, 2, 3, 8):
            cov = []
            for r in range(world):
                a, b = sks_dist.tile_shard(T, world, r)
                cov += list(range(a, b))
            assert cov == list(range(T))
            covg = []
            for r in range(world):
                _, g0, g1 = sks_dist.genome_shard(n, world, r)
                covg += list(range(g0, g1))
            assert covg == list(range(n))
        nb = (n + 63) // 64
        for t in range(T):
            seen.append(sks_dist.sym_tile_coords(t, n))
        assert seen == [(i, j) for i in range(nb) for j in range(i, nb)]


# ---- config 5: seed sweep sharded by seed, consensus by all-reduce ------------------
SWEEP_GENOMES, SWEEP_SEEDS = 12, 5


def _sweep_ani(seed_index):
    """ANI matrix of one mask seed over the sweep collection, oracle-only."""
    m = O.mask(31, 21, seed_index)
    k = bin(m).count("1") // 2
    sk = []
    for g in range(SWEEP_GENOMES):
        seq = synth.bases(4000, seed=70 + g % 2, mut_seed=500 + g, mut_rate=0.004 * (g % 6))
        s, _ = O.sketch(O.cut_runs(seq.tobytes()), 31, m, "bottom", 150)
        sk.append(s)
    ani = np.zeros((SWEEP_GENOMES, SWEEP_GENOMES))
    for i in range(SWEEP_GENOMES):
        for j in range(SWEEP_GENOMES):
            ani[i, j] = O.binomial_estimator(O.containment(O.intersect(sk[i], sk[j]), len(sk[i])), k)
    return torch.from_numpy(ani)


def _sweep_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cons, mine = sks_dist.seed_sweep(SWEEP_SEEDS, world, rank, _sweep_ani, SWEEP_GENOMES)
    q.put((rank, cons.numpy(), mine))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_seed_sweep_gloo_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, cons, mine = q.get(timeout=240)
        results[r] = (cons, mine)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = sorted(s for r in results for s in results[r][1])
    assert covered == list(range(SWEEP_SEEDS))
    want = sum(_sweep_ani(s).numpy() for s in range(SWEEP_SEEDS)) / SWEEP_SEEDS
    for r in range(world):
        # summation order differs (all-reduce vs sequential): within 1e-12, the
        # north-star ANI tolerance is 1e-9
        assert np.allclose(results[r][0], want, rtol=0, atol=1e-12)
    assert want[0, 0] == 1.0 and 0 < want[0, 2] < 1


# ---- config 4 over per-source sketch broadcasts (sks_dist.all_vs_all_join) -----------------
M64 = (1 << 64) - 1


def _ival(data, ew, i):
    """element i of a flat int64 tensor of ew-word values, as a Python int (hi << 64 | lo)"""
    if ew == 1:
        return int(data[i]) & M64
    return ((int(data[2 * i + 1]) & M64) << 64) | (int(data[2 * i]) & M64)


class NpJoinOps:
    """numpy restatement of the join layout's contract: per 64-sketch block, each
    distinct value once with the mask of the block's sketches holding it, keyed
    by (value group from the GIVEN bounds, hash bucket in the group).  count()
    joins blocks bucket key by bucket key, so layouts built with different
    bounds miss shared values and show up as count errors."""

    def __init__(self, ew, rank):
        self.ew, self.rank = ew, rank
        self.built, self.calls = [], []

    def bounds_like(self, log_b):
        return torch.zeros((sks_dist_groups(log_b) + 1) * self.ew, dtype=torch.int64)

    def bounds(self, src, log_b):
        # rank 0's own quantile-ish bounds from its first sketch (rank-specific
        # values: every layout must end up with exactly these)
        assert self.rank == 0
        G = sks_dist_groups(log_b)
        vals = sorted(_ival(src.data, self.ew, i) for i in range(min(src.total, 500))) or [0]
        b = [0] + [vals[(g * len(vals)) // G] + g for g in range(1, G)] + [(1 << (64 * self.ew)) - 1]
        b = sorted(b)
        out = []
        for v in b:
            out += [v & M64] if self.ew == 1 else [v & M64, v >> 64]
        return torch.tensor(np.array(out, dtype=np.uint64).view(np.int64))

    def bounds_for_mask(self, mask, log_b):
        """sks_join_layout_bounds_for_mask (host; every rank computes the same)"""
        import sksffi
        return torch.from_numpy(sksffi.join_layout_bounds_for_mask(mask, log_b, self.ew).view(np.int64))

    def build(self, src, log_b, gb, key, blocks_hint=0):
        G = sks_dist_groups(log_b)
        bnd = [_ival(gb, self.ew, g) for g in range(G + 1)]
        self.built.append((key, log_b, tuple(bnd)))
        starts = src.starts.tolist()
        sizes = src.sizes.tolist()
        blocks = []
        for b0 in range(0, src.n, 64):
            ent = {}
            for slot in range(min(64, src.n - b0)):
                i = b0 + slot
                for e in range(sizes[i]):
                    v = _ival(src.data, self.ew, starts[i] + e)
                    g = int(np.searchsorted(bnd[1:G], v, side="right")) if G > 1 else 0
                    h = ((v & M64) * 0x9E3779B97F4A7C15 & M64) >> 61
                    ent.setdefault((g, h), {}).setdefault(v, 0)
                    ent[(g, h)][v] |= 1 << slot
            blocks.append(ent)
        return blocks

    def count(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, out):
        self.calls.append((r_blk0, c_blk0, len(tiles)))
        for t, (I, J) in enumerate(np.asarray(tiles).reshape(-1, 2)):
            R, C = rows[I - r_blk0], cols[J - c_blk0]
            rm, cm = [], []
            for key, rv in R.items():  # a value meets its partner only under the same bucket key
                cv = C.get(key, {})
                for v, m in rv.items():
                    if cv.get(v, 0):
                        rm.append(m)
                        cm.append(cv[v])
            if rm:  # every (row sketch, column sketch) pair of a shared value, as bit outer products
                out[t] += torch.from_numpy((_bits(rm).T @ _bits(cm)).astype(np.int32))

    def count_ani(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, out, sizes, k, ani):
        """count, then the ANI of both orientations of every counted pair into the
        dense n x n matrix (the contract of sks_intersect_layout_ani)."""
        self.count(n, log_b, rows, r_blk0, cols, c_blk0, tiles, out)
        for t, (I, J) in enumerate(np.asarray(tiles).reshape(-1, 2)):
            for r in range(64):
                for c in range(64):
                    i, j = I * 64 + r, J * 64 + c
                    if i < n and j < n:
                        x = int(out[t, r, c])
                        ani[i, j] = O.binomial_estimator(O.containment(x, int(sizes[i])), k)
                        ani[j, i] = O.binomial_estimator(O.containment(x, int(sizes[j])), k)

    def parts(self, T, device, zeroed=True):
        # (uncleared tiles for layout_tiles_ani, which clears them itself)
        f = torch.zeros if zeroed else (lambda *a, **k: torch.full(*a, -99, **k))
        return f((max(T, 1), 64, 64), dtype=torch.int32)

    def layout_tiles_ani(self, src, log_b, gb, blocks_hint, blk0, tiles, out, sizes_global, n_global, k, ani):
        """sks_layout_tiles_ani's contract: the layout of src (its block 0 is global
        block blk0), the global tiles joined into out (cleared first), and with k
        the ANI of both orientations (|S_g| by global g)."""
        lay = self.build(src, log_b, gb, "own" if not blocks_hint else "peers", blocks_hint)
        out.zero_()
        if k is None:
            self.count(n_global, log_b, lay, blk0, lay, blk0, tiles, out)
        else:
            self.count_ani(n_global, log_b, lay, blk0, lay, blk0, tiles, out, sizes_global, k, ani)

    def pad(self, src, stride, data, sizes):
        """the sketches at a fixed stride, padded with ~0 words (sks_sketches_export)"""
        st, sz = src.starts.tolist(), src.sizes.tolist()
        for i in range(src.n):
            a, m = st[i] * self.ew, sz[i] * self.ew
            data[i * stride * self.ew:i * stride * self.ew + m] = src.data[a:a + m]
        sizes[:src.n] = src.sizes


def _bits(masks):
    a = np.array(masks, dtype=np.uint64)
    return ((a[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.int64)


def sks_dist_groups(log_b):
    """value groups of a layout with 2^log_b buckets (sks_join_layout_groups: 8 buckets a group)"""
    return 1 << (log_b - 3) if log_b > 3 else 1


def _join_worker(rank, world, port, q, dst, n_genomes, ew, exchange, bound, mask_bounds=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sk = _join_sketches(n_genomes, ew)
    _, g0, g1 = sks_dist.block_shard(n_genomes, world, rank)
    mine = sk[g0:g1]
    flat = np.concatenate([x.reshape(-1) for x in mine] + [np.zeros(0, np.uint64)]).view(np.int64)
    src = sks_dist.Sketches(torch.from_numpy(flat.copy()), torch.tensor([len(x) for x in mine], dtype=torch.int32),
                            ew)
    ops = NpJoinOps(ew, rank)
    res = sks_dist.all_vs_all_join(n_genomes, world, rank, src, ops, lambda m: 5, dst=dst, ani_ones=21,
                                   exchange=exchange,
                                   size_bound=max(len(x) for x in sk) + 3 if bound else None,
                                   bounds_mask=(O.mask(21, 21, 0) if ew == 1 else O.mask(40, 30, 0))
                                   if mask_bounds else None)
    q.put((rank, None if res.matrix is None else res.matrix.numpy(), ops.built, ops.calls,
           res.tiles, res.counts.numpy(), res.ani.numpy()))
    dist.destroy_process_group()


def _sketches_n(n):
    """n small related sketches (six families, 50-90 elements) for the N = 8 plans"""
    m = O.mask(21, 21, 0)
    out = []
    for g in range(n):
        seq = synth.bases(1200, seed=80 + g % 6, mut_seed=2000 + g, mut_rate=0.004 * (g % 5))
        sk, _ = O.sketch(O.cut_runs(seq.tobytes()), 21, m, "bottom", 50 + (g % 5) * 10)
        out.append(np.sort(sk[:, 0].astype(np.int64)))
    return out


def _join_sketches(n_genomes, ew):
    if ew == 1:
        if n_genomes not in (N_GENOMES, N_200):
            return [s.astype(np.uint64) for s in _sketches_n(n_genomes)]
        return [s.astype(np.uint64) for s in (_sketches() if n_genomes == N_GENOMES else _sketches_200())]
    m = O.mask(40, 30, 0)
    out = []
    for g in range(n_genomes):
        seq = synth.bases(2500, seed=60 + g % 3, mut_seed=700 + g, mut_rate=0.004 * (g % 6))
        s, _ = O.sketch(O.cut_runs(seq.tobytes()), 40, m, "frac", 20)
        out.append(s)  # (k, 2) uint64 (lo, hi)
    return out


@pytest.mark.parametrize("world,dst,n_genomes,ew,exchange,bound,mask_bounds", [
    (2, 0, N_GENOMES, 1, "p2p", True, False), (3, "all", N_GENOMES, 1, "p2p", False, False),
    (2, 1, 200, 1, "allgather", True, True), (3, 0, 200, 1, "broadcast", True, False),
    (3, 0, 200, 1, "p2p", True, True), (3, 0, 130, 2, "allgather", False, True),
    (4, "all", 200, 1, "p2p", True, False), (8, 0, 600, 1, "p2p", True, True),
    (8, 3, 600, 1, "allgather", False, False)])
def test_all_vs_all_join_exchanges_gloo(world, dst, n_genomes, ew, exchange, bound, mask_bounds):
    """Ranks build the layout of their own block-aligned genomes with rank 0's
    bounds and count their own blocks' tiles first; once the peers' sketches
    have landed in the rank's exchange buffer (p2p send/recv, one all-gather, or
    per-source broadcasts; padded to the caller's size bound, or to the
    all-reduced largest sketch) they build ONE layout of their own and peer rows
    (global block numbers) and count every cross tile of the cyclic plan (rows
    from the lower rank's blocks) in one join; the packed tiles go to dst (every rank for
    "all"), whose matrix equals the single-process merge counts, and the ANI
    each rank wrote for its tiles (both orientations) equals the reference
    formula, every ordered pair written by exactly one rank.  mask_bounds:
    every rank takes the group bounds from the mask
    (sks_join_layout_bounds_for_mask) instead of rank 0's broadcast.  n = 200 at world
    3 and 4 leaves ranks without genomes; ew = 2 moves 128-bit (lo, hi) k-mers
    (w = 40); world 8 over 600 genomes (10 blocks) is the N = 8 plan with
    ragged block ranges."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_join_worker, args=(r, world, port, q, dst, n_genomes, ew, exchange, bound,
                                                    mask_bounds))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {r[0]: r[1:] for r in (q.get(timeout=600) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sk = _join_sketches(n_genomes, ew)
    want = _all_pairs(sk)
    sizes = [len(x) for x in sk]
    bnds = {b for r in range(world) for (_, _, b) in results[r][1]}
    assert len(bnds) == 1  # every layout on every rank used rank 0's bounds
    written = np.zeros((n_genomes, n_genomes), np.int32)
    for r in range(world):
        mat, built, calls, tiles, counts, ani = results[r]
        if dst == "all" or r == dst:
            assert np.array_equal(mat, want), r
        else:
            assert mat is None
        loc, rem = sks_dist.tile_plan_by_peer(n_genomes, world, r)
        _, g0, _ = sks_dist.block_shard(n_genomes, world, r)
        expect = [(g0 // 64, g0 // 64, len(loc))] if len(loc) else []
        hi, lo = sks_dist.peer_groups(n_genomes, world, r)
        n_remote = sum(len(rem[qq]) for qq in hi + lo)
        if n_remote:  # one layout of the own and peer rows (global blocks), one join of every cross tile
            expect.append((0, 0, n_remote))
        assert calls == expect, (r, calls, expect)
        # the cyclic plan: at most world // 2 peers, all in ONE peer layout per rank
        assert len(hi) + len(lo) <= world // 2
        assert len([k for (k, _, _) in built if k != "own"]) <= 1
        for t, (I, J) in enumerate(tiles):
            for a, b in ((0, 0), (3, 7), (63, 62)):
                i, j = I * 64 + a, J * 64 + b
                if i < n_genomes and j < n_genomes:
                    assert counts[t, a, b] == want[i, j]
            for a in range(64):
                for b in range(64):
                    i, j = I * 64 + a, J * 64 + b
                    if i < n_genomes and j < n_genomes:
                        written[i, j] += 1
                        if I != J:
                            written[j, i] += 1
    assert (written == 1).all()  # every ordered pair counted (and its ANI written) by exactly one rank
    # each rank's matrix holds the ANI of its own tiles' pairs (zero elsewhere)
    full = sum(np.asarray(results[r][5]) for r in range(world))
    want_ani = np.array([[O.binomial_estimator(O.containment(int(want[i, j]), sizes[i]), 21)
                          for j in range(n_genomes)] for i in range(n_genomes)])
    assert np.array_equal(full, want_ani)


def _w(x):
    x = np.asarray(x, dtype=np.uint64)
    return x if x.ndim == 2 else np.stack([x, 0 * x], 1)


def _all_pairs(sk):
    """|S_i ∩ S_j| for all pairs of distinct-valued sketches: the value incidence
    matrix times its transpose (checked against the oracle merge on a sample)."""
    rows = [_w(x) for x in sk]
    allv = np.concatenate(rows + [np.zeros((0, 2), np.uint64)])
    uniq, inv = np.unique(allv, axis=0, return_inverse=True)
    M = np.zeros((len(sk), len(uniq)), np.int64)
    o = 0
    for i, r in enumerate(rows):
        M[i, inv.reshape(-1)[o:o + len(r)]] = 1
        o += len(r)
    want = M @ M.T
    for i, j in ((0, 1), (len(sk) - 1, 0), (len(sk) // 2, len(sk) // 3)):
        assert want[i, j] == O.intersect(rows[i], rows[j])
    return want


def test_block_shard_covers_whole_blocks():
    for n in (1, 64, 65, 130, 1000):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                bpr, g0, g1 = sks_dist.block_shard(n, world, r)
                assert (g0 % 64 == 0 or g0 == n) and (g1 == n or (g1 - g0) == bpr * 64)
                seen += list(range(g0, g1))
            assert seen == list(range(n))


# ---- one genome chunk-sharded across ranks (sks_dist.sketch_genome_sharded) ----------
GENOME_LEN, GW = 250_000, 31


def _genome():
    g = synth.bases(GENOME_LEN, seed=91)
    g[100_000:100_040] = ord("N")
    return g.tobytes()


def _union128(t):
    """Sorted distinct (lo, hi) rows as 128-bit values (the contract of
    sks_sketch_union_wide), via numpy on the host."""
    a = t.numpy().view(np.uint64).reshape(-1, 2)
    a = np.unique(a, axis=0)
    order = np.lexsort((a[:, 0], a[:, 1]))  # hi major, lo minor
    return torch.from_numpy(a[order].view(np.int64).copy())


def _shard_worker(rank, world, port, q, w, k):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = _genome()
    m = O.mask(w, k, 0)

    def build_chunk(a, b):
        sk, nw = O.sketch(O.cut_runs(g[a:b]), w, m, "frac", 50)
        if w > 32:
            return torch.from_numpy(sk.view(np.int64).copy()), nw  # [k, 2] (lo, hi)
        return torch.from_numpy(sk[:, 0].view(np.int64).copy()), nw
    union = _union128 if w > 32 else (lambda t: torch.unique(t, sorted=True))
    sk, nw = sks_dist.sketch_genome_sharded(len(g), w, world, rank, build_chunk, union)
    q.put((rank, sk.numpy(), nw))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,w,k", [(2, GW, 21), (3, GW, 21), (3, 45, 30)])
def test_one_genome_sharded_gloo(world, w, k):
    """Every rank's union of the chunk sketches equals the whole genome's sketch,
    and the windows add up (no window counted twice across a halo); w = 45 moves
    (lo, hi) k-mer pairs through the same gather."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q, w, k)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want, nw = O.sketch(O.cut_runs(_genome()), w, O.mask(w, k, 0), "frac", 50)
    for _, sk, n in res:
        got = sk.view(np.uint64).reshape(-1, 2) if w > 32 else sk.view(np.uint64)
        assert np.array_equal(got, want if w > 32 else want[:, 0]) and n == nw


# ---- tile plan of all_vs_all_join ------------------------------------------------------------
N_200 = 200  # four tile blocks, ragged; at world 3 the last rank holds no genome


def _sketches_200():
    m = O.mask(21, 21, 0)
    out = []
    for g in range(N_200):
        seq = synth.bases(4000, seed=70 + g % 5, mut_seed=900 + g, mut_rate=0.003 * (g % 7))
        sk, _ = O.sketch(O.cut_runs(seq.tobytes()), 21, m, "bottom", 150 + (g % 3) * 40)
        out.append(np.sort(sk[:, 0].astype(np.int64)))
    if N_200 > 77:
        out[77] = out[77][:0]  # an empty sketch
    return out


@pytest.mark.parametrize("n,world", [(1000, 8), (1000, 4), (1000, 2), (1024, 8), (1000, 3), (200, 3), (64, 2),
                                     (1, 4), (5000, 7), (600, 8)])
def test_tile_plan_partitions_upper_triangle(n, world):
    for r in range(world):  # remote tiles by peer: rows in the lower rank's blocks
        _, rem = sks_dist.tile_plan_by_peer(n, world, r)
        for q, tq in enumerate(rem):
            lo, hi = sks_dist.block_shard(n, world, min(r, q)), sks_dist.block_shard(n, world, max(r, q))
            for I, J in tq:
                assert lo[1] // 64 <= I < (lo[2] + 63) // 64 and hi[1] // 64 <= J < (hi[2] + 63) // 64
    nb = (n + 63) // 64
    seen = {}
    sizes = []
    for r in range(world):
        loc, rem = sks_dist.tile_plan(n, world, r)
        sizes.append(len(loc) + len(rem))
        bpr, g0, g1 = sks_dist.block_shard(n, world, r)
        for I, J in loc:
            assert g0 // 64 <= I <= J < (g1 + 63) // 64
        for I, J in np.concatenate([loc, rem]):
            assert 0 <= I <= J < nb
            assert (I, J) not in seen
            seen[(I, J)] = r
    assert len(seen) == nb * (nb + 1) // 2
    # the cyclic plan: a rank joins with at most world // 2 peers' layouts
    for r in range(world):
        assert len(sks_dist.peer_needs(n, world, r)) <= world // 2
    full = all(sks_dist.block_shard(n, world, r)[2] - sks_dist.block_shard(n, world, r)[1] ==
               sks_dist.block_shard(n, world, r)[0] * 64 for r in range(world))
    if full:  # every rank holds a whole block range (config 4 at N = 1, 2, 4, 8): near-equal shares
        assert max(sizes) - min(sizes) <= 1, sizes


