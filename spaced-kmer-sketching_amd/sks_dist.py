"""Multi-GPU orchestration for all-vs-all ANI (one process per GPU).

The reference parallelises with cilk_for over files (kmer_set.cpp:124) and over
pairs (kmer_set.cpp:179) inside one process.  Here (all_vs_all_join):
  * genomes are sharded across ranks in whole 64-sketch blocks; each rank
    sketches its own and builds the join layout of its own blocks,
  * every rank's sketches are broadcast by their owner (RCCL over xGMI for
    "nccl"), and each receiver joins its blocks with the source's as they land
    (a fixed tile plan splits the upper-triangle 64x64 tiles between ranks),
  * containment / ANI are computed per tile on the rank that counted it, and
    the packed count tiles are assembled into the n x n matrix on one rank
    only when asked.
Config 5 shards seeds (seed_sweep: one all-reduce of ANI sums) and config 3
shards genomes or one genome's chunks (sketch_genome_sharded).  The functions
take the kernels as callables so the same orchestration is exercised on CPU
with gloo in tests/test_dist_cpu.py.
"""
import functools

import numpy as np
import torch
import torch.distributed as dist

TILE = 64


def _solo(world):
    """True when no exchange is needed: one rank and no process group.  A process
    group of size 1 (tests/test_rccl.py: RCCL on one GPU) takes the collective
    path, so every all-gather / all-reduce below runs on the backend."""
    return world == 1 and not (dist.is_available() and dist.is_initialized())


def genome_shard(n_genomes, world, rank):
    per = (n_genomes + world - 1) // world
    g0 = min(n_genomes, rank * per)
    return per, g0, min(n_genomes, g0 + per)


def sym_tiles(n):
    nb = (n + TILE - 1) // TILE
    return nb * (nb + 1) // 2


def tile_shard(n_tiles, world, rank):
    return rank * n_tiles // world, (rank + 1) * n_tiles // world


def sym_tile_coords(t, n):
    """(I, J) of upper-triangle tile t (row-major, I <= J) — intersect.hip sym_tile."""
    nb = (n + TILE - 1) // TILE
    i = 0
    while t >= nb - i:
        t -= nb - i
        i += 1
    return i, i + t


def gather_sketches(local, local_sizes, world):
    """local: [per, stride] int64 padded sketches; local_sizes: [per] int32."""
    if _solo(world):
        return local, local_sizes
    per, stride = local.shape
    if dist.get_backend() == "nccl":
        full = torch.empty((per * world, stride), dtype=local.dtype, device=local.device)
        full_sz = torch.empty(per * world, dtype=local_sizes.dtype, device=local.device)
        dist.all_gather_into_tensor(full, local)
        dist.all_gather_into_tensor(full_sz, local_sizes)
        return full, full_sz
    # gloo (CPU tests, single-GPU rehearsal): stage through host memory
    lc, lsc = local.cpu(), local_sizes.cpu()
    parts = [torch.empty_like(lc) for _ in range(world)]
    szs = [torch.empty_like(lsc) for _ in range(world)]
    dist.all_gather(parts, lc)
    dist.all_gather(szs, lsc)
    return torch.cat(parts).to(local.device), torch.cat(szs).to(local.device)


def sum_matrix(out):
    if dist.get_backend() == "nccl" or out.device.type == "cpu":
        dist.all_reduce(out)
        return out
    host = out.cpu()
    dist.all_reduce(host)
    out.copy_(host)
    return out


def all_vs_all(local, local_sizes, n_genomes, world, rank, count_sym, out=None):
    """Returns the full n x n int32 intersection matrix on every rank.

    count_sym(sketches, sizes, n, tile_begin, tile_end, out) must zero `out`
    and write the counts of upper-triangle tiles [tile_begin, tile_end) to
    both (i, j) and (j, i) — the contract of sks_intersect_sym.
    """
    src, src_sz = gather_sketches(local, local_sizes, world)
    t0, t1 = tile_shard(sym_tiles(n_genomes), world, rank)
    if out is None:
        out = torch.empty((n_genomes, n_genomes), dtype=torch.int32, device=local.device)
    count_sym(src, src_sz, n_genomes, t0, t1, out)
    if not _solo(world):
        sum_matrix(out)
    return out


# ---- seed sweep (BASELINE config 5) ----------------------------------------------------
# The reference sweeps (w, k) configurations serially, re-sketching every file
# per configuration (kmer-sketching.cpp:214-239 around :151-212).  Config 5 runs
# several spaced seeds over one genome collection; seeds are independent, so
# ranks shard by seed (rank r takes seeds r, r + world, ...), each rank keeps
# the whole collection resident, sketches it and computes its own all-vs-all
# matrix per seed.  The only exchange is the consensus: one all-reduce (sum)
# of the per-seed ANI matrices, divided by the number of seeds.

def seed_shard(n_seeds, world, rank):
    return list(range(rank, n_seeds, world))


def seed_sweep(n_seeds, world, rank, ani_for_seed, n_genomes, device="cpu"):
    """ani_for_seed(seed_index) -> [n_genomes, n_genomes] float64 tensor (row i =
    first set of the pair, as kmer-sketching.cpp:195-200).  Returns (consensus,
    local_seeds): the mean over all seeds of the ANI matrices, on every rank."""
    acc = torch.zeros((n_genomes, n_genomes), dtype=torch.float64, device=device)
    mine = seed_shard(n_seeds, world, rank)
    # ani_for_seed may return a future (host ANI of seed s overlapping the GPU
    # work of seed s + 1); resolve all of them, then sum in seed order
    parts = [ani_for_seed(s) for s in mine]
    for r in parts:
        acc += (r.result() if hasattr(r, "result") else r).to(device)
    if not _solo(world):
        sum_matrix(acc)
    acc /= n_seeds
    return acc, mine


# ---- stream ordering, packed tiles, one receiving rank ---------------------------------------
# Each rank counts a fixed plan of upper-triangle 64x64 tiles (tile_plan): the
# tiles of its own blocks first — from its own data, while the exchange is in
# flight — then the tiles pairing its blocks with those of the peers the cyclic
# plan gives it.  Counts stay packed ([tile][64][64] int32, 16 KB per tile);
# when asked they go to ONE rank (dst), where the n x n matrix is assembled: no
# collective carries n^2 words.  Containment and ANI are written by the join
# itself (sks_intersect_layout_ani), straight into the caller's n x n matrix.

def _ctx_waits_for_torch(ctx):
    """Order the context's HIP stream after work queued so far on torch's current
    stream (no-op when they are the same stream)."""
    s = _ctx_torch_stream(ctx)
    if s is not None:
        s.wait_stream(torch.cuda.current_stream())


def _torch_waits_for_ctx(ctx):
    s = _ctx_torch_stream(ctx)
    if s is not None:
        torch.cuda.current_stream().wait_stream(s)


_EXT_STREAMS = {}


def _ctx_torch_stream(ctx):
    h = getattr(ctx, "stream", 0) or 0
    cur = torch.cuda.current_stream()
    if h == cur.cuda_stream:
        return None
    if h == 0:
        return torch.cuda.default_stream()
    if h not in _EXT_STREAMS:  # one wrapper per HIP stream (building one per call costs host time)
        _EXT_STREAMS[h] = torch.cuda.ExternalStream(h)
    return _EXT_STREAMS[h]


def _gather_tiles(parts, world, dst):
    """parts: [Tmax, 64, 64] (padded) of this rank -> [world, Tmax, 64, 64] on dst
    (None elsewhere), or on every rank when dst is None."""
    if dst is None:
        return _gather_flat(parts.reshape(-1), world).view((world,) + tuple(parts.shape))
    nccl = dist.get_backend() == "nccl"
    src = parts if nccl else parts.cpu()
    lst = [torch.empty_like(src) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(src, gather_list=lst, dst=dst)
    if lst is None:
        return None
    return torch.stack(lst).to(parts.device)


_PLACE_CACHE = {}


def place_tiles(mat, tiles, parts, n):
    """Writes packed tile counts into the n x n matrix: tile (I, J) at rows
    64 I.., columns 64 J.., and mirrored when I != J (a diagonal tile holds both
    triangles).  The index maps depend only on (tiles, n): built once per
    process and device, then every step is two gathers and two scatters."""
    dev = mat.device
    tiles = np.asarray(tiles, dtype=np.int64).reshape(-1, 2)
    key = (tiles.tobytes(), n, str(dev))
    if key not in _PLACE_CACHE:
        if len(_PLACE_CACHE) > 4:
            _PLACE_CACHE.clear()
        t = torch.as_tensor(tiles.copy(), device=dev)  # (a cached tile list is read-only)
        ar = torch.arange(TILE, device=dev, dtype=torch.int64)
        gr = (t[:, 0:1] * TILE + ar.view(1, -1)).view(-1, TILE, 1).expand(-1, TILE, TILE)
        gc = (t[:, 1:2] * TILE + ar.view(1, -1)).view(-1, 1, TILE).expand(-1, TILE, TILE)
        ok = ((gr < n) & (gc < n)).reshape(-1)
        off = ((t[:, 0] != t[:, 1]).view(-1, 1, 1).expand(-1, TILE, TILE).reshape(-1)) & ok
        src_up = torch.nonzero(ok).view(-1)
        src_lo = torch.nonzero(off).view(-1)
        flat_up = (gr * n + gc).reshape(-1)[src_up]
        flat_lo = (gc * n + gr).reshape(-1)[src_lo]
        _PLACE_CACHE[key] = (src_up, flat_up, src_lo, flat_lo)
    src_up, flat_up, src_lo, flat_lo = _PLACE_CACHE[key]
    vals = parts.reshape(-1).to(dev)
    flat = mat.view(-1)
    flat[flat_up] = vals[src_up]
    flat[flat_lo] = vals[src_lo]
    return mat


# ---- all-vs-all over join layouts -------------------------------------------------------------
# The join kernel's input (sks_join_layout_build) is built per 64-sketch block.
# Each rank owns whole blocks (block_shard), sketches them and builds the layout
# of its own blocks; it counts its own blocks' tiles on that layout at once.
# The cross-rank tiles follow a cyclic plan (tile_plan_by_peer): rank r counts
# every tile pairing its blocks with those of rank r + d (mod N) for
# d = 1 .. N/2, the d = N/2 pairs (even N) split in halves between the two, so
# a rank needs the sketches of N/2 peers, not N - 1.  They land in one buffer
# holding a slot per rank (row g = genome g): ONE layout of the own and peer
# rows (global block numbers, the other rows empty) and ONE join launch count
# every cross tile.  Sketches travel padded to a common stride
# (the caller's size bound, e.g. bottom-s s: no size exchange and no host
# round trip), by one of three exchanges:
#   "p2p"        batched send/recv, step d: send to r - d, receive from r + d
#                (each rank receives only what its plan needs; the joins of
#                step d start as soon as step d has landed),
#   "allgather"  one all_gather_into_tensor of the per-rank padded blocks (the
#                collective north_star names; every peer lands at once),
#   "broadcast"  one broadcast per source rank, queued in rank order.
# Raw sketches travel rather than layouts: a deduplicated layout keeps its
# regions at raw offsets with 16 B per slot, so it is larger than the sketch,
# and rebuilding a peer's layout costs less than moving twice the bytes.  All
# layouts share rank 0's value-group bounds (broadcast first), so every pair of
# blocks is bucketed alike.  Containment / ANI are written by the join into the
# caller's n x n matrix as each tile completes (the rank's own tiles only).

def block_shard(n_genomes, world, rank):
    """(blocks per rank, g0, g1): genome range of `rank`, whole 64-sketch blocks."""
    n_blk = (n_genomes + TILE - 1) // TILE
    bpr = max(1, (n_blk + world - 1) // world)
    g0 = min(n_genomes, rank * bpr * TILE)
    return bpr, g0, min(n_genomes, g0 + bpr * TILE)


@functools.lru_cache(maxsize=64)
def tile_plan_by_peer(n_genomes, world, rank):
    """(local, remote): local int64 [T, 2] — the upper-triangle tiles (I, J)
    with both blocks in the rank's own block range; remote — a list over ranks
    q of the tiles pairing the two ranks' blocks that `rank` counts (I in the
    lower rank's blocks, J in the higher's).  Cyclic: rank r counts the pairs
    with q = r + d (mod world) for d = 1 .. world // 2; at d = world / 2 (even
    world) the two ranks reach each other, and the lower rank takes the first
    half of the pair's tiles (row-major), the higher the rest."""
    nb = (n_genomes + TILE - 1) // TILE
    bpr = block_shard(n_genomes, world, rank)[0]

    def blocks(q):
        return np.arange(min(nb, q * bpr), min(nb, (q + 1) * bpr), dtype=np.int64)

    mine = blocks(rank)
    I, J = np.meshgrid(mine, mine, indexing="ij")
    keep = I <= J
    local = np.stack([I[keep], J[keep]], axis=1).reshape(-1, 2) if mine.size else np.zeros((0, 2), np.int64)
    remote = [np.zeros((0, 2), np.int64) for _ in range(world)]
    for d in range(1, world // 2 + 1):
        q = (rank + d) % world
        a, b = min(rank, q), max(rank, q)
        ba, bb = blocks(a), blocks(b)
        if not ba.size or not bb.size:
            continue
        I, J = np.meshgrid(ba, bb, indexing="ij")
        pairs = np.stack([I.reshape(-1), J.reshape(-1)], axis=1)
        if 2 * d == world:
            h = (len(pairs) + 1) // 2
            pairs = pairs[:h] if rank == a else pairs[h:]
        remote[q] = pairs
    local.flags.writeable = False  # cached: shared by every caller
    for r in remote:
        r.flags.writeable = False
    return local, tuple(remote)


def tile_plan(n_genomes, world, rank):
    """(local, remote) int64 arrays [T, 2] of the upper-triangle tiles (I, J) that
    `rank` counts: its own blocks' tiles, then its share of the cross-rank
    block pairs (tile_plan_by_peer, concatenated in rank order).  Every tile of
    the n x n upper triangle is in exactly one rank's plan."""
    local, remote = tile_plan_by_peer(n_genomes, world, rank)
    return local, np.concatenate(remote).reshape(-1, 2)


def peer_needs(n_genomes, world, rank):
    """Ranks whose sketches `rank` needs (its plan pairs its blocks with theirs):
    the higher ranks ascending, then the lower ranks ascending (each run covers
    consecutive global blocks, so it is one layout: peer_groups)."""
    _, remote = tile_plan_by_peer(n_genomes, world, rank)
    need = [q for q in range(world) if q != rank and len(remote[q])]
    return [q for q in need if q > rank] + [q for q in need if q < rank]


def peer_groups(n_genomes, world, rank):
    """(hi, lo): the peers above and below `rank` that its plan joins with,
    ascending (the cyclic plan's peers r + 1 .. r + N/2 (mod N) are at most two
    runs of consecutive ranks)."""
    need = peer_needs(n_genomes, world, rank)
    return [q for q in need if q > rank], [q for q in need if q < rank]


class Sketches:
    """A rank's sketch set as tensors: data int64 [total * ew] (sketches back to
    back, or at a fixed stride), sizes int32 [n], starts int64 [n] (element
    index of each sketch); total = elements the data holds (an upper bound of
    the sizes' sum)."""

    def __init__(self, data, sizes, ew=1, starts=None):
        self.data, self.sizes, self.ew = data, sizes, ew
        self.n = int(sizes.numel())
        if starts is None:
            starts = torch.zeros(self.n, dtype=torch.int64, device=sizes.device)
            if self.n > 1:
                starts[1:] = torch.cumsum(sizes[:-1].to(torch.int64), 0)
        self.starts = starts
        self.total = int(data.numel()) // ew


_STRIDE_STARTS = {}


def _strided(data, sizes, ew, stride):
    n = int(sizes.numel())
    key = (n, stride, str(sizes.device))
    st = _STRIDE_STARTS.get(key)
    if st is None:  # the starts of a strided set depend on its shape only: built once
        if len(_STRIDE_STARTS) > 16:
            _STRIDE_STARTS.clear()
        st = _STRIDE_STARTS[key] = torch.arange(n, dtype=torch.int64, device=sizes.device) * stride
    return Sketches(data[:n * stride * ew], sizes, ew, starts=st)


def _exchange_start(own, n_genomes, world, rank, stride, ops, mode):
    """Starts moving the sketches the cyclic plan needs into ONE buffer of every
    rank's slot — `per` rows (a whole rank's block range) of `stride` elements per
    rank, so row g is genome g — and returns wait() -> those rows as Sketches
    (this rank's own rows and its peers'; the rows of ranks it does not need,
    and padding rows, hold size 0): one layout of all the rank's peers, with the
    global block numbering.  This rank's slot is written by the export itself.
    With RCCL everything runs on the collective stream and wait() only orders
    torch's current stream after it (the host does not block); with gloo the
    data goes through host memory."""
    ew, dev = own.ew, own.data.device
    nccl = dist.get_backend() == "nccl"
    bdev = dev if nccl else "cpu"
    per = block_shard(n_genomes, world, rank)[0] * TILE  # sketches of a full rank
    counts = [block_shard(n_genomes, world, q)[2] - block_shard(n_genomes, world, q)[1] for q in range(world)]
    row = per * stride * ew
    full = torch.empty((world * row,), dtype=torch.int64, device=bdev)  # rows past a size are never read
    full_sz = torch.zeros((world * per,), dtype=torch.int32, device=bdev)
    slot = (slice(rank * row, (rank + 1) * row), slice(rank * per, (rank + 1) * per))
    if nccl:
        send, send_sz = full[slot[0]], full_sz[slot[1]]
    else:  # the export runs where the sketches are; gloo sends from host memory
        send = torch.full((row,), -1, dtype=torch.int64, device=dev)
        send_sz = torch.zeros(per, dtype=torch.int32, device=dev)
    if own.n:
        ops.pad(own, stride, send, send_sz)
    if not nccl:
        full[slot[0]] = send.cpu()
        full_sz[slot[1]] = send_sz.cpu()
        send, send_sz = full[slot[0]], full_sz[slot[1]]
    need = peer_needs(n_genomes, world, rank)
    works = []
    if mode == "allgather":
        if nccl:  # in place: this rank's input is its own slot of the output
            works = [dist.all_gather_into_tensor(full, send, async_op=True),
                     dist.all_gather_into_tensor(full_sz, send_sz, async_op=True)]
        else:
            dist.all_gather(list(full.view(world, row).unbind(0)), send.clone())
            dist.all_gather(list(full_sz.view(world, per).unbind(0)), send_sz.clone())
    elif mode == "broadcast":
        for q in range(world):
            if counts[q]:
                works += [dist.broadcast(full[q * row:(q + 1) * row], src=q, async_op=nccl),
                          dist.broadcast(full_sz[q * per:(q + 1) * per], src=q, async_op=nccl)]
    elif mode == "p2p":
        # every send and receive in one batch: all xGMI links at once (batches
        # issued one after another serialise on the communicator's stream)
        ops_ = []
        for d_ in range(1, world):
            to, frm = (rank - d_) % world, (rank + d_) % world
            if counts[rank] and rank in peer_needs(n_genomes, world, to):
                ops_ += [(dist.isend, send, to), (dist.isend, send_sz, to)]
            if frm in need:
                ops_ += [(dist.irecv, full[frm * row:(frm + 1) * row], frm),
                         (dist.irecv, full_sz[frm * per:(frm + 1) * per], frm)]
        if ops_:
            if nccl:
                works = dist.batch_isend_irecv([dist.P2POp(f, t, p) for f, t, p in ops_])
            else:
                works = [f(t, p) for f, t, p in ops_]
    else:
        raise ValueError(f"unknown exchange {mode!r}")
    if not nccl:  # gloo: the host copies complete here
        for w in works:
            if w is not None:
                w.wait()
        works = []

    def wait():
        for w in works:
            if w is not None:
                w.wait()
        works.clear()
        d, sz = (full, full_sz) if nccl else (full.to(dev), full_sz.to(dev))
        return _strided(d, sz, ew, stride)
    return wait


class JoinResult:
    """What all_vs_all_join leaves on a rank.  tiles: int64 [T, 2] of the tiles
    this rank counted (None for one rank without a process group counting into
    the dense matrix); counts: packed int32 [T, 64, 64] (or the dense n x n
    matrix); ani: the n x n float64 matrix the join wrote the ANI of this rank's
    tiles into (both orientations), when asked; matrix: the n x n int32 counts
    on the assembling rank(s), else None.  check_layouts() (after the stream
    has passed the call) raises if a join layout could not be built."""

    def __init__(self):
        self.tiles = self.counts = self.ani = self.matrix = None
        self._stats = None

    def check_layouts(self):
        if self._stats is None:
            return
        torch.cuda.current_stream().synchronize()
        bad = int(self._stats[:, 1].max()) if self._stats.numel() else 0
        if bad:
            raise RuntimeError("sks_dist: a join layout could not place a value group (adversarial 128-bit "
                               "values); its counts are invalid — use sks_intersect_all")


@functools.lru_cache(maxsize=16)
def _all_tiles(nb):
    I, J = np.triu_indices(nb)
    t = np.stack([I, J], axis=1).astype(np.int64)
    t.flags.writeable = False  # cached: shared by every caller
    return t


def all_vs_all_join(n_genomes, world, rank, mine, ops, log_b_for, device="cpu", dst=0, ani_ones=None,
                    ani_out=None, max_size=None, size_bound=None, exchange="p2p", world1_exchange=False,
                    bounds_mask=None):
    """All-vs-all intersection counts (kmer_set.cpp:143-184 over the
    generate_all_pairs_from_vector list, generators.hpp:44-58), and ANI when
    ani_ones (the k of binomial_estimator) is given (kmer-sketching.cpp:195-200).

    mine: Sketches of this rank's block-aligned genomes (block_shard).
    ops: the kernels (GpuJoinOps on the GPU; a numpy restatement in the CPU
    tests): ew; bounds(src, log_b) -> group bounds tensor; build(src, log_b,
    bounds, key) -> layout (cached by key); count(n, log_b, rows, r_blk0, cols,
    c_blk0, tiles, out) — the contract of sks_intersect_layout_pair_tiles
    (tiles None: every upper-triangle tile of one layout into the dense matrix
    out); count_ani(..., out, sizes, k, ani) — the same with the ANI of every
    counted pair written into the n x n matrix ani (sks_intersect_layout_ani);
    pad(src, stride, data, sizes) — the sketches at a fixed stride.
    dst: the rank that assembles the n x n count matrix (None: none, "all":
    every rank).  ani_out: where the ANI goes (n * n float64: a device tensor
    or pinned host memory, e.g. sksffi.HostBuffer — the join writes it; each
    rank fills the cells of its own tiles); None with ani_ones: a new device
    tensor.  max_size: the largest local sketch, known to the caller's host
    (else one device reduction and a read-back).  size_bound: an upper bound of
    every rank's sketch sizes that all ranks pass alike (bottom-s: s) — the
    exchange then needs no size all-gather and no host round trip.  exchange:
    "p2p", "allgather" or "broadcast" (see above).  bounds_mask: the k-mer
    mask the sketches were built with; every rank then takes the value-group
    bounds from the mask alone (ops.bounds_for_mask, sks_join_layout_bounds_for_mask)
    instead of rank 0 sampling its sketches and broadcasting them.  One rank — with or without
    a process group — counts every tile of one layout in one native call
    (sks_all_pairs_ani); world1_exchange keeps a world-1 process group on the
    exchange path instead (the RCCL rehearsal tests).  Returns a JoinResult."""
    res = JoinResult()
    bpr, g0, g1 = block_shard(n_genomes, world, rank)
    solo = _solo(world)
    mx = (int(max_size) if max_size is not None else int(mine.sizes.max().item())) if mine.n else 0
    if size_bound is not None:
        if mx > size_bound:
            raise ValueError(f"all_vs_all_join: a local sketch holds {mx} > size_bound {size_bound} elements")
        gmax = int(size_bound)
    elif solo or world == 1:
        gmax = mx
    else:
        gmax = _max_over(mx, world, device)  # one all-reduce and a read-back
    log_b = log_b_for(max(gmax, 1))
    fused = ani_ones is not None
    if fused and ani_out is None:
        ani_out = torch.zeros((n_genomes, n_genomes), dtype=torch.float64, device=device)
    res.ani = ani_out if fused else None
    if fused and gmax and hasattr(ops, "ani_table"):
        ops.ani_table(gmax, ani_ones)  # rows of gmax elements (bottom-s: all) read their ANI from a table
    stats_mark = ops.stats_mark() if hasattr(ops, "stats_mark") else None
    native = hasattr(ops, "all_pairs") and not getattr(ops, "no_native", False)
    if (solo or (world == 1 and not world1_exchange)) and native and (fused or dst is None):
        # one call: layout + every tile (+ the fused ANI) natively (sks_all_pairs_ani)
        nb = (n_genomes + TILE - 1) // TILE
        res.tiles = _all_tiles(nb)
        res.counts = ops.parts(len(res.tiles), device, zeroed=False)  # the call clears them
        if n_genomes:
            ops.all_pairs(mine, mx, res.counts, ani_ones if fused else None, ani_out if fused else None)
        if dst is not None:
            out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
            res.matrix = place_tiles(out, res.tiles, res.counts, n_genomes)
        if stats_mark is not None:
            res._stats = ops.stats_since(stats_mark)
        return res
    if solo:
        lay = ops.build(mine, log_b, None, "own")
        if not fused:  # counts only: the dense matrix, both halves by the join
            out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
            if n_genomes:
                ops.count(n_genomes, log_b, lay, 0, lay, 0, None, out)
            res.counts = res.matrix = out
        else:
            nb = (n_genomes + TILE - 1) // TILE
            res.tiles = _all_tiles(nb)
            res.counts = ops.parts(len(res.tiles), device)
            if n_genomes:
                ops.count_ani(n_genomes, log_b, lay, 0, lay, 0, None, res.counts, mine.sizes, ani_ones, ani_out)
            if dst is not None:
                out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
                res.matrix = place_tiles(out, res.tiles, res.counts, n_genomes)
        if stats_mark is not None:
            res._stats = ops.stats_since(stats_mark)
        return res
    # one set of group bounds shared by every layout (blocks of different ranks
    # are joined bucket by bucket): fixed by the mask on every rank alike, or
    # rank 0's sampled bounds broadcast
    if bounds_mask is not None and hasattr(ops, "bounds_for_mask"):
        gb = ops.bounds_for_mask(bounds_mask, log_b)
    else:
        gb = ops.bounds(mine, log_b) if rank == 0 else ops.bounds_like(log_b)
        if world > 1:
            gb = _broadcast(gb, 0, world)
    local, remote = tile_plan_by_peer(n_genomes, world, rank)
    tq, held = _cross_plan(n_genomes, world, rank)
    T = len(local) + len(tq)
    native = hasattr(ops, "layout_tiles_ani")  # layout + join (+ ANI) in one call, clearing its own outputs
    parts = ops.parts(T, device, zeroed=not native)
    wait = _exchange_start(mine, n_genomes, world, rank, max(gmax, 1), ops, exchange) if world > 1 else None
    if native:
        # the rank's own tiles while the peers' sketches travel; the ANI finisher
        # reads |S_g| by global genome g, so the own set's sizes are offset by g0
        if len(local):
            ops.layout_tiles_ani(mine, log_b, gb, 0, g0 // TILE, local, parts[:len(local)], _OffsetSizes(mine.sizes, g0),
                                 n_genomes, ani_ones if fused else None, ani_out if fused else None)
        if len(tq):
            union = wait()
            ops.layout_tiles_ani(union, log_b, gb, held, 0, tq, parts[len(local):T], union.sizes, n_genomes,
                                 ani_ones if fused else None, ani_out if fused else None)
    else:
        sizes_all = torch.zeros(max(n_genomes, 1), dtype=torch.int32, device=device) if fused else None
        if fused and mine.n:
            sizes_all[g0:g1] = mine.sizes
        own = ops.build(mine, log_b, gb, "own") if mine.n else None

        def count(rows, rb, cols, cb, tiles, out):
            if fused:
                ops.count_ani(n_genomes, log_b, rows, rb, cols, cb, tiles, out, sizes_all, ani_ones, ani_out)
            else:
                ops.count(n_genomes, log_b, rows, rb, cols, cb, tiles, out)
        if len(local):  # the rank's own tiles while the peers' sketches travel
            count(own, g0 // TILE, own, g0 // TILE, local, parts[:len(local)])
        off = len(local)
        # every cross-rank tile of the plan in one join over one layout of the rank's
        # own and peer rows (the exchange buffer: row g = genome g, so block numbers
        # are global and blk0 = 0); rows the plan does not need are empty.  (One
        # layout of the peer rows alone and two joins, own x peers and peers x own,
        # measured 0.585 against 0.524 ms per rank at N = 8: tools/rank_sim.py)
        if len(tq):
            union = wait()
            lu = ops.build(union, log_b, gb, "peers", blocks_hint=held)
            if fused:
                sizes_all[:n_genomes] = union.sizes[:n_genomes]
            count(lu, 0, lu, 0, tq, parts[off:off + len(tq)])
    res.tiles = np.concatenate([local, tq]).reshape(-1, 2)
    res.counts = parts[:T]
    if stats_mark is not None:
        res._stats = ops.stats_since(stats_mark)
    if dst is None:
        return res
    plans = [_plan_in_count_order(n_genomes, world, q) for q in range(world)]
    counts = [len(pl) for pl in plans]
    pad = torch.zeros((max(max(counts), 1), TILE, TILE), dtype=torch.int32, device=device)
    pad[:T] = res.counts
    gathered = _gather_tiles(pad, world, None if dst == "all" else dst)
    if gathered is None:
        return res
    tiles = np.concatenate(plans).reshape(-1, 2)
    got = torch.cat([gathered[q, :counts[q]] for q in range(world)])
    out = torch.zeros((n_genomes, n_genomes), dtype=torch.int32, device=device)
    res.matrix = place_tiles(out, tiles, got, n_genomes)
    return res


class _OffsetSizes:
    """The sizes of genomes [g0, g0 + n) addressed by GLOBAL genome index: the
    device pointer moved back by g0 words (only indices in range are read)."""

    def __init__(self, t, g0):
        self.t, self.g0 = t, g0

    def data_ptr(self):
        return self.t.data_ptr() - 4 * self.g0

    def __getitem__(self, g):
        return self.t[g - self.g0]


@functools.lru_cache(maxsize=64)
def _cross_plan(n_genomes, world, rank):
    """(tiles, held): the rank's cross-rank tiles in count order (its peers in
    peer_needs order) and the 64-sketch blocks its exchange buffer holds (its own
    and its peers'), computed once per shape."""
    _, remote = tile_plan_by_peer(n_genomes, world, rank)
    need = peer_needs(n_genomes, world, rank)
    tq = np.concatenate([remote[q] for q in need] + [np.zeros((0, 2), np.int64)]).reshape(-1, 2)
    tq.flags.writeable = False
    held = sum((block_shard(n_genomes, world, q)[2] - block_shard(n_genomes, world, q)[1] + TILE - 1) // TILE
               for q in [rank] + need)
    return tq, held


def _plan_in_count_order(n_genomes, world, rank):
    """The tiles of `rank` in the order all_vs_all_join counts them: its own,
    then per peer in peer_needs order (the higher run, then the lower)."""
    local, remote = tile_plan_by_peer(n_genomes, world, rank)
    return np.concatenate([local] + [remote[q] for q in peer_needs(n_genomes, world, rank)]).reshape(-1, 2)


def _max_over(x, world, device):
    if _solo(world):
        return int(x)
    t = torch.tensor([int(x)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def _gather_flat(t, world):
    return _gather_many([t], world)[0]


def _gather_many(ts, world):
    """All-gather of flat tensors, rank-major; with RCCL the gathers are queued
    together (async) and waited on once, so their latencies overlap."""
    if _solo(world):
        return list(ts)
    if dist.get_backend() == "nccl":
        outs, works = [], []
        for t in ts:
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=t.device)
            works.append(dist.all_gather_into_tensor(out, t.contiguous(), async_op=True))
            outs.append(out)
        for w in works:
            w.wait()
        return outs
    res = []
    for t in ts:
        host = t.cpu()
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host)
        res.append(torch.cat(parts).to(t.device))
    return res


def _broadcast(t, src, world):
    if _solo(world):
        return t
    if dist.get_backend() == "nccl" or t.device.type == "cpu":
        dist.broadcast(t, src=src)
        return t
    host = t.cpu()
    dist.broadcast(host, src=src)
    t.copy_(host)
    return t


class GpuJoinOps:
    """The kernels of all_vs_all_join on the GPU through libsks: a context `ctx`
    and the k-mer width (ew = 1: u64, 2: 128-bit).  Layout buffers persist per
    build key across calls of the same shape; the context's HIP stream is
    ordered after torch's current stream before its kernels and torch's after
    them, so a context on any stream works with the collectives on torch's.
    Every layout build's status words are copied to a device log (no read-back;
    JoinResult.check_layouts reads them after the join)."""

    def __init__(self, ctx, ew=1):
        import sksffi
        self.sksffi, self.ctx, self.ew = sksffi, ctx, ew
        self.bufs, self.tile_cache, self.keep = {}, {}, {}
        self.stats = torch.zeros((16, 2), dtype=torch.int32, device="cuda")
        self.n_stats = 0

    def stats_mark(self):
        """Starts a call's log of layout status words (the previous call's view
        is overwritten from here on)."""
        self.n_stats = 0
        return 0

    def stats_since(self, mark):
        """The call's status rows as a copy (queued on torch's stream), so a later
        call reusing the log's rows cannot change an earlier JoinResult's view."""
        return self.stats[mark:self.n_stats].clone()

    def parts(self, T, device, zeroed=True):
        """Packed count tiles [T, 64, 64], zeroed unless the kernels clear them."""
        f = torch.zeros if zeroed else torch.empty
        return f((max(T, 1), TILE, TILE), dtype=torch.int32, device="cuda")

    def bounds_like(self, log_b):
        return torch.empty((self.sksffi.join_layout_groups(log_b) + 1) * self.ew, dtype=torch.int64, device="cuda")

    def bounds_for_mask(self, mask, log_b):
        """The mask-derived group bounds on the device (uploaded once per (mask, log_b))."""
        key = ("mask_bounds", int(mask), log_b, self.ew)
        if key not in self.keep:
            h = self.sksffi.join_layout_bounds_for_mask(int(mask), log_b, self.ew)
            self.keep[key] = torch.from_numpy(h.view(np.int64)).to("cuda")
        return self.keep[key]

    def bounds(self, src, log_b):
        b = self.bounds_like(log_b)
        _ctx_waits_for_torch(self.ctx)
        self.ctx.join_layout_bounds(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n, log_b,
                                    b.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)
        self.keep["bounds"] = src
        return b

    def build(self, src, log_b, gb, key, blocks_hint=0):
        """The join layout of src (cached buffers per key).  blocks_hint: how many
        of src's 64-sketch blocks hold sketches when most rows are empty (the
        exchange buffer), so the build sizes its regions for the real work."""
        nb = (src.n + TILE - 1) // TILE
        shape = (max(src.total, 1), log_b, max(nb, 1))
        if self.bufs.get(key, (None,))[0] != shape:
            BW = self.sksffi.join_layout_boff_words(log_b)
            self.bufs[key] = (shape, (torch.empty(shape[0] * self.ew, dtype=torch.int64, device="cuda"),
                                      torch.empty(shape[0], dtype=torch.int64, device="cuda"),
                                      torch.zeros(shape[2] * BW, dtype=torch.int32, device="cuda"),
                                      torch.zeros(shape[2] + 1, dtype=torch.int64, device="cuda")))
        lay = self.bufs[key][1]
        if src.n:
            _ctx_waits_for_torch(self.ctx)  # the buffers' previous readers, the source's writers
            if blocks_hint:
                self.ctx.set_layout_blocks_hint(blocks_hint)
            try:
                self.ctx.join_layout_build(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n,
                                           log_b, *(t.data_ptr() for t in lay), stat=False, total=src.total,
                                           bounds=gb.data_ptr() if gb is not None else None, elem_words=self.ew)
            finally:
                if blocks_hint:
                    self.ctx.set_layout_blocks_hint(0)
            self.ctx.join_layout_stat_copy(self._stat_slot())
            _torch_waits_for_ctx(self.ctx)
        self.keep[key] = (src, gb)  # alive until torch's stream is past the build
        return lay

    def _stat_slot(self):
        if self.n_stats == self.stats.shape[0]:
            self.stats = torch.cat([self.stats, torch.zeros_like(self.stats)])
        self.n_stats += 1
        return self.stats.data_ptr() + 8 * (self.n_stats - 1)  # row n_stats - 1: two int32

    def all_pairs(self, src, max_size, out, k, ani):
        """sks_all_pairs_ani: one layout of src, every upper-triangle tile into the
        packed out [T, 64, 64], and the ANI into ani when k is given."""
        ani_ptr = (ani.data_ptr() if hasattr(ani, "data_ptr") else ani.ptr) if k is not None else 0
        d, st, sz = src.ptrs if getattr(src, "ptrs", None) else \
            (src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr())
        _ctx_waits_for_torch(self.ctx)
        self.ctx.all_pairs_ani(d, st, sz, src.n, max(int(max_size), 1), max(src.total, 1), k or 0, ani_ptr,
                               out.data_ptr(), self._stat_slot(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)
        self.keep["all_pairs"] = src

    def pad(self, src, stride, data, sizes):
        _ctx_waits_for_torch(self.ctx)
        self.ctx.sketches_export(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n,
                                 data.data_ptr(), stride, sizes.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)

    def _tiles(self, tiles):
        key = tiles.tobytes()  # the plan repeats every step: upload it once
        if key not in self.tile_cache:
            if len(self.tile_cache) > 64:
                self.tile_cache.clear()
            self.tile_cache[key] = torch.from_numpy(np.array(tiles, dtype=np.int32)).reshape(-1, 2).to("cuda")
        return self.tile_cache[key]

    def layout_tiles_ani(self, src, log_b, gb, blocks_hint, blk0, tiles, out, sizes_global, n_global, k, ani):
        """sks_layout_tiles_ani: the layout of src (block 0 = global block blk0) and
        the join of the global tile list into the packed out (cleared by the call),
        with the ANI into ani when k is given; the build's status words go to the
        call's log."""
        ani_ptr = (ani.data_ptr() if hasattr(ani, "data_ptr") else ani.ptr) if k is not None else 0
        tl = self._tiles(tiles)
        _ctx_waits_for_torch(self.ctx)
        self.ctx.layout_tiles_ani(src.data.data_ptr(), src.starts.data_ptr(), src.sizes.data_ptr(), src.n,
                                  max(src.total, 1), log_b, gb.data_ptr() if gb is not None else 0, blocks_hint, blk0,
                                  tl.data_ptr(), tl.shape[0], n_global, sizes_global.data_ptr() if k is not None else 0,
                                  k or 0, ani_ptr, out.data_ptr(), self._stat_slot(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)
        self.keep[("lt", blk0)] = (src, gb, sizes_global)

    def count(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, out):
        _ctx_waits_for_torch(self.ctx)
        if tiles is None:
            self.ctx.intersect_layout_tiles(n, log_b, *(t.data_ptr() for t in rows), 0, 0, 0,
                                            self.sksffi.intersect_sym_tiles(n), False, out.data_ptr(),
                                            elem_words=self.ew)
        else:
            tl = self._tiles(tiles)
            self.ctx.intersect_layout_pair_tiles(n, log_b, [t.data_ptr() for t in rows], r_blk0,
                                                 [t.data_ptr() for t in cols], c_blk0, tl.data_ptr(), 0,
                                                 tl.shape[0], out.dim() == 3, out.data_ptr(), elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)

    def ani_table(self, size, k):
        """sks_ctx_ani_table: the fused ANI of rows of `size` elements from a table (queued, cached)."""
        self.ctx.ani_table(size, k)

    def count_ani(self, n, log_b, rows, r_blk0, cols, c_blk0, tiles, out, sizes, k, ani):
        """count + the ANI of every counted pair into ani (n * n float64: a device
        tensor, or an object with .ptr — pinned host memory, sksffi.HostBuffer)."""
        ani_ptr = ani.data_ptr() if hasattr(ani, "data_ptr") else ani.ptr
        if tiles is None:
            tl, t_end = None, self.sksffi.intersect_sym_tiles(n)
        else:
            tl = self._tiles(tiles)
            t_end = tl.shape[0]
        _ctx_waits_for_torch(self.ctx)
        self.ctx.intersect_layout_ani(n, log_b, [t.data_ptr() for t in rows], r_blk0, [t.data_ptr() for t in cols],
                                      c_blk0, tl.data_ptr() if tl is not None else 0, 0, t_end, out.dim() == 3,
                                      out.data_ptr(), sizes.data_ptr(), k, ani_ptr, elem_words=self.ew)
        _torch_waits_for_ctx(self.ctx)
        self.keep["ani_sizes"] = sizes


class _SetSketches(Sketches):
    """Sketches of a SketchSet: the device pointers at once (`ptrs`, all the
    one-call native path needs), the zero-copy torch views built on first use."""

    def __init__(self, ss):
        self._ss, self.ew, self.n = ss, ss.elem_words, ss.n
        self.total = int(ss.sizes().astype(np.int64).sum())
        self.ptrs = tuple(int(p or 0) for p in ss.device_ptrs())
        self._t = None

    def _views(self):
        if self._t is None:
            self._t = self._ss.device_tensors(torch.cuda.current_device())
        return self._t

    data = property(lambda self: self._views()[0])
    starts = property(lambda self: self._views()[1])
    sizes = property(lambda self: self._views()[2])


def sketches_of(ss, ew=None):
    """Sketches (zero-copy device views) of a SketchSet, or an empty set for None."""
    if ss is None:
        e = ew or 1
        return Sketches(torch.zeros(0, dtype=torch.int64, device="cuda"),
                        torch.zeros(0, dtype=torch.int32, device="cuda"), e)
    return _SetSketches(ss)


# ---- one genome across ranks (SURVEY §8e, config 3 strong scaling) -----------------------
# FracMinHash keeps a k-mer on its own hash, so the sketch of a genome is the
# union of the sketches of chunks cut with (w-1)-base halos: rank r scans the
# windows that start in [r*n/world, (r+1)*n/world), the chunk sets are
# all-gathered (padded to the largest) and every rank forms the sorted union.

def genome_chunk(n_bytes, w, world, rank):
    a = n_bytes * rank // world
    b = n_bytes * (rank + 1) // world
    return a, min(n_bytes, b + w - 1) if b > a else b


def sketch_genome_sharded(n_bytes, w, world, rank, build_chunk, union, device="cpu"):
    """build_chunk(a, b) -> (int64 tensor of the chunk's sorted k-mers, windows):
    shape [k] for w <= 32, [k, 2] (lo, hi) for w > 32; union(t) -> sorted distinct
    k-mers of t (same shape convention).  Returns (sketch, total windows) on
    every rank."""
    a, b = genome_chunk(n_bytes, w, world, rank)
    vals, nw = build_chunk(a, b)
    if _solo(world):
        return vals, nw
    k = vals.shape[0]
    rest = tuple(vals.shape[1:])
    kmax = max(1, _max_over(k, world, device))
    pad = torch.zeros((kmax,) + rest, dtype=torch.int64, device=device)
    pad[:k] = vals
    g = _gather_flat(pad.reshape(-1), world).view((world, kmax) + rest)
    sizes = _gather_flat(torch.tensor([k], dtype=torch.int64, device=device), world)
    keep = torch.arange(kmax, device=device).view(1, kmax) < sizes.view(world, 1)
    t = torch.tensor([nw], dtype=torch.int64, device=device)
    dist.all_reduce(t)
    return union(g[keep]), int(t.item())
