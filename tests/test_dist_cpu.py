"""CPU (gloo, world_size 2 and 3): the multi-GPU all-vs-all orchestration of
spaced-kmer-sketching_amd/sks_dist.py — genome sharding, the all-gather of
padded sketches, the symmetric tile split and the all-reduce — assembles
exactly the single-process matrix.  The count kernel is replaced by the
oracle's merge count over the same tile contract (sks_intersect_sym)."""
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


# ---- all-vs-all in row blocks, (lo, hi) k-mers (w > 32): sks_dist.all_vs_all_rows ------
WIDE_N, WIDE_W, WIDE_K, WIDE_STRIDE = 45, 40, 30, 160


def _wide_sketches():
    m = O.mask(WIDE_W, WIDE_K, 0)
    out = []
    for g in range(WIDE_N):
        seq = synth.bases(2500, seed=60 + g % 3, mut_seed=700 + g, mut_rate=0.004 * (g % 6))
        sk, _ = O.sketch(O.cut_runs(seq.tobytes()), WIDE_W, m, "frac", 20)
        out.append(sk)  # (k, 2) uint64 (lo, hi)
    return out


def _oracle_count_rows(src, sizes, n, r0, r1, out):
    """count_rows contract (sks_intersect_all row blocks) on padded (lo, hi) rows."""
    a = src.numpy().view(np.uint64).reshape(src.shape[0], -1, 2)
    sz = sizes.numpy()
    for i in range(r0, r1):
        for j in range(n):
            out[i - r0, j] = O.intersect(a[i, : sz[i]], a[j, : sz[j]])


def _rows_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sk = _wide_sketches()
    per, g0, g1 = sks_dist.genome_shard(WIDE_N, world, rank)
    local = torch.full((per, 2 * WIDE_STRIDE), -1, dtype=torch.int64)
    local_sz = torch.zeros(per, dtype=torch.int32)
    for i, g in enumerate(range(g0, g1)):
        assert len(sk[g]) <= WIDE_STRIDE
        local[i, : 2 * len(sk[g])] = torch.from_numpy(sk[g].reshape(-1).view(np.int64))
        local_sz[i] = len(sk[g])
    mat = sks_dist.all_vs_all_rows(local, local_sz, WIDE_N, world, rank, _oracle_count_rows)
    q.put((rank, mat.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_all_vs_all_rows_wide_gloo(world):
    """w = 40 (128-bit k-mers): padded (lo, hi) sketches gathered, each rank counts its
    row block, row blocks gathered; every rank ends with the single-process matrix."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rows_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sk = _wide_sketches()
    want = np.array([[O.intersect(sk[i], sk[j]) for j in range(WIDE_N)] for i in range(WIDE_N)])
    assert want[0, 3] > 0  # related genomes share 128-bit k-mers
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


# ---- config 4 over gathered join layouts (sks_dist.all_vs_all_join) ------------------
PHI = np.uint64(0x9E3779B97F4A7C15)


def _np_layout(sketches, log_b):
    """numpy restatement of sks_join_layout_build: blocks of 64, hash buckets
    (v * phi) >> (64 - log_b), block-major; returns torch tensors like the ABI."""
    B = 1 << log_b
    data, ids, boff, bstart, mx = [], [], [], [0], 0
    for b0 in range(0, len(sketches), 64):
        blk = sketches[b0:b0 + 64]
        with np.errstate(over="ignore"):
            hb = [(s * PHI) >> np.uint64(64 - log_b) if log_b else np.zeros(len(s), np.uint64)
                  for s in blk]
        start = len(data)
        offs = []
        for b in range(B):
            offs.append(len(data) - start)
            here = 0
            for slot, (s, h) in enumerate(zip(blk, hb)):
                sel = s[h == b]
                data.extend(sel.tolist())
                ids.extend([slot] * len(sel))
                here += len(sel)
            mx = max(mx, here)
        offs.append(len(data) - start)
        boff.extend(offs)
        bstart.append(len(data))
    as_t = lambda x, dt: torch.tensor(np.array(x, dtype=np.uint64).view(np.int64) if dt == torch.int64
                                       else np.array(x), dtype=dt)
    return (as_t(data, torch.int64), torch.tensor(ids, dtype=torch.uint8),
            torch.tensor(boff, dtype=torch.int32), as_t(bstart, torch.int64), mx)


def _np_count_tiles_layout(n, log_b, lay, blk0, tiles, out):
    """The contract of sks_intersect_layout_tiles (packed, counts added), from a
    layout whose block 0 is global block blk0 (decodes block k's sketches by id)."""
    data, ids, boff, bstart = lay
    B1 = (1 << log_b) + 1
    d = data.numpy().view(np.uint64)

    def sketches_of(k):
        kk = k - blk0
        a = int(bstart[kk])
        e = a + int(boff[kk * B1 + B1 - 1])
        vals, sl = d[a:e], ids[a:e].numpy()
        return [np.sort(vals[sl == i]) for i in range(64)]
    for t, (I, J) in enumerate(np.asarray(tiles).reshape(-1, 2)):
        ri, cj = sketches_of(I), sketches_of(J)
        for a in range(64):
            for b in range(64):
                i, j = I * 64 + a, J * 64 + b
                if i < n and j < n:
                    out[t, a, b] += np.intersect1d(ri[a], cj[b], assume_unique=True).size


def _join_worker(rank, world, port, q, dst, n_genomes):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sk = [s.astype(np.uint64) for s in (_sketches() if n_genomes == N_GENOMES else _sketches_200())]
    _, g0, g1 = sks_dist.block_shard(n_genomes, world, rank)
    mine = sk[g0:g1]
    built, calls = [], []

    def bounds(lb):  # rank 0's bounds are broadcast: rank-specific values show it
        assert rank == 0
        return torch.arange(sks_dist.layout_groups(lb) + 1, dtype=torch.int64) * 1000 + 7

    def build(lb, pad, gb):
        built.append((lb, pad))
        assert torch.equal(gb, bounds.__wrapped__(lb)), gb  # every rank got rank 0's
        d, i, b, s, _ = _np_layout(mine, lb)
        if pad is None:
            return d, i, b, s
        cap_e, bpr = pad  # the padded send-buffer shape all_vs_all_join gathers
        assert d.numel() <= cap_e and b.numel() <= bpr * ((1 << lb) + 1)
        totals = [sum(len(x) for x in sk[sks_dist.block_shard(n_genomes, world, r)[1]:
                                         sks_dist.block_shard(n_genomes, world, r)[2]]) for r in range(world)]
        assert cap_e == max(max(totals), 1), (cap_e, totals)  # the largest rank's total, exactly
        pd = torch.full((cap_e,), -7, dtype=torch.int64)
        pi = torch.full((cap_e,), 99, dtype=torch.uint8)
        pb = torch.full((bpr * ((1 << lb) + 1),), -3, dtype=torch.int32)
        ps = torch.full((bpr + 1,), -5, dtype=torch.int64)  # junk past the own blocks
        pd[:d.numel()], pi[:i.numel()], pb[:b.numel()], ps[:s.numel()] = d, i, b, s
        return pd, pi, pb, ps

    def count(n, lb, lay, blk0, tiles, out):
        calls.append((blk0, len(tiles)))
        _np_count_tiles_layout(n, lb, lay, blk0, tiles, out)
    bounds.__wrapped__ = lambda lb: torch.arange(sks_dist.layout_groups(lb) + 1, dtype=torch.int64) * 1000 + 7
    mat = sks_dist.all_vs_all_join(
        n_genomes, world, rank, max((len(s) for s in mine), default=0), sum(len(s) for s in mine),
        lambda m: 3, build, count, dst=dst, bounds=bounds)
    q.put((rank, None if mat is None else mat.numpy(), built, calls))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,dst,n_genomes", [(2, 0, N_GENOMES), (3, None, N_GENOMES), (2, 1, 200),
                                                 (3, 0, 200)])
def test_all_vs_all_join_layout_gather_gloo(world, dst, n_genomes):
    """Ranks build layouts of their own block-aligned genomes into send buffers
    padded to the largest rank's element total, count their own blocks' tiles
    on their own layout (first call, blk0 = their first block) while the layouts
    are gathered, then their share of the cross-rank tiles on the gathered
    layout; the packed tiles go to dst (every rank for None), whose matrix equals
    the single-process merge counts; the others return None.  n = 200 at world 3
    leaves the last rank without genomes."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_join_worker, args=(r, world, port, q, dst, n_genomes))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {r: (m, b, c) for r, m, b, c in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sk = _sketches() if n_genomes == N_GENOMES else _sketches_200()
    want = np.array([[len(np.intersect1d(sk[i], sk[j])) for j in range(n_genomes)]
                     for i in range(n_genomes)])
    for r in range(world):
        mat, built, calls = results[r]
        if dst is None or r == dst:
            assert np.array_equal(mat, want), r
        else:
            assert mat is None
        assert [lb for lb, _ in built] == [3]
        loc, rem = sks_dist.tile_plan(n_genomes, world, r)
        _, g0, _ = sks_dist.block_shard(n_genomes, world, r)
        expect = ([(g0 // 64, len(loc))] if len(loc) else []) + ([(0, len(rem))] if len(rem) else [])
        assert calls == expect, (r, calls)


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


@pytest.mark.parametrize("n,world", [(1000, 8), (1000, 3), (200, 3), (64, 2), (1, 4), (5000, 7)])
def test_tile_plan_partitions_upper_triangle(n, world):
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
    full = [s for r, s in enumerate(sizes) if sks_dist.block_shard(n, world, r)[2] -
            sks_dist.block_shard(n, world, r)[1] == sks_dist.block_shard(n, world, r)[0] * 64]
    if full:  # ranks holding whole block ranges get near-equal shares
        assert max(full) - min(full) <= world
