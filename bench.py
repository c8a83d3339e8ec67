"""bench.py — spaced-k-mer sketch + ANI engine on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Headline (`value`): k-mers hashed/s, whole job, on config 3 of BASELINE.json
(one 3 Gb human-scale synthetic genome per GPU: 24 contigs x 125 Mb, four 10 kb
N-runs per contig, spaced seed w=31/k=21 mask seed 0, FracMinHash 1/1000).
A step = one complete sketch build of that genome (fused scan kernel + sort +
unique, host syncs included) with the bytes already resident in HBM. The timed
steps run with --inflight (default 3) builds in flight, one context and HIP
stream each, so one build's post-processing overlaps the next build's scan; a
serial pass (`ms_per_step_serial`) and the scan kernel's own time are reported
beside it.
Genomes are independent, so ranks shard them with no collective: weak scaling.

Secondary (`pairs`): genome-pairs ANI/s on config 4 (1000 x 5 Mb genomes =
10 ancestors x 100 mutated descendants, w=31/k=21, bottom-s s=10000), strong
scaling.  A pair step is what the reference's "Time taken for comparison"
covers (kmer-sketching.cpp:185-203): every ordered pair's intersection count,
containment and ANI, with the ANI delivered to host memory.  Rank r owns whole
64-genome blocks, sketches them and builds their join layout; every rank's
sketches are broadcast by their owner over RCCL (torch.distributed "nccl") and
each rank joins its blocks with a source's as they land (a fixed plan splits
the upper-triangle 64x64 tiles); containment and ANI are computed on the
device per tile and copied to the rank's host memory.  At N = 1 the counts go
straight into the n x n matrix and the ANI matrix (8 MB) is copied to host
memory.  `pairs_wide`:
the same leg at w = 45 / k = 30 (128-bit k-mers).

`cpu_baseline`: the reference-faithful CPU port (oracle/ref_port.cpp, see
BASELINE.md) timed on this box's host cores on a bounded sample of the same
workload (rank 0, N=1 only).
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "spaced-kmer-sketching_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import sksffi  # noqa: E402
import synth  # noqa: E402

METRIC = "k-mers hashed/s + genome-pairs ANI/s at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

W, K, MASK_SEED = 31, 21, 0
C3_CONTIGS, C3_CONTIG_LEN, C3_NRUN, C3_NRUN_LEN, C3_FRAC = 24, 125_000_000, 4, 10_000, 1000
C4_GENOMES, C4_LEN, C4_ANCESTORS, C4_S = 1000, 5_000_000, 10, 10000
C4W_W, C4W_K = 45, 30  # config 4 at a 128-bit (k+10, k) shape of the reference sweep
C5_GENOMES, C5_SEEDS = 200, 8  # first 200 genomes of config 4, mask seeds 0..7


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus, backend, rehearsal=False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob: SKS_BENCH_DEVICE=0 puts every rank on GPU 0 (use with gloo)
    if os.environ.get("SKS_BENCH_DEVICE") is not None:
        local = int(os.environ["SKS_BENCH_DEVICE"])
    # --dist-rehearsal: a process group even at world 1 (torchrun --nproc-per-node 1),
    # so every all-gather / all-reduce of the N > 1 paths runs on RCCL on one GPU
    if world > 1 or rehearsal:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    return world, rank, local


def collective():
    """A process group is up (world > 1, or the world-1 RCCL rehearsal)."""
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized()


def backend_label():
    """What the collectives run on, from the process group itself."""
    import torch.distributed as dist
    b = dist.get_backend()
    return {"nccl": "RCCL over xGMI", "gloo": "gloo, via host memory"}.get(b, b)


def barrier(world):
    if collective():
        import torch.distributed as dist
        dist.barrier()


def _reduce_scalar(x, op):
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def max_over_ranks(x, world):
    if not collective():
        return x
    import torch.distributed as dist
    return _reduce_scalar(x, dist.ReduceOp.MAX)


def sum_over_ranks(x, world):
    if not collective():
        return x
    import torch.distributed as dist
    return _reduce_scalar(x, dist.ReduceOp.SUM)


def sum_vector_over_ranks(v, world):
    if not collective():
        return v
    import torch.distributed as dist
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.int64)).to(dev)
    dist.all_reduce(t)
    return t.cpu().numpy()


# all-vs-all sketch exchange between ranks (sks_dist.all_vs_all_join): p2p | allgather | broadcast
EXCHANGE = "p2p"
WORLD1_EXCHANGE = False  # --world1-exchange: a world-1 process group keeps the exchange path


# ---- config 3 ---------------------------------------------------------------------
def c3_layout():
    """Byte layout of one genome: contigs separated by '\\n'; N-run offsets."""
    contig_starts = [i * (C3_CONTIG_LEN + 1) for i in range(C3_CONTIGS)]
    n_bytes = C3_CONTIGS * (C3_CONTIG_LEN + 1)
    nrun_off = [int(C3_CONTIG_LEN * (j + 1) / (C3_NRUN + 1)) for j in range(C3_NRUN)]
    return contig_starts, n_bytes, nrun_off


def c3_windows():
    # per contig: runs cut by the N-runs; windows = sum(max(0, L - w + 1))
    _, _, nrun_off = c3_layout()
    edges = [0]
    for o in nrun_off:
        edges += [o, o + C3_NRUN_LEN]
    edges.append(C3_CONTIG_LEN)
    per = sum(max(0, edges[i + 1] - edges[i] - W + 1) for i in range(0, len(edges), 2))
    return per * C3_CONTIGS


def make_c3(ctx, seed_base):
    contig_starts, n_bytes, nrun_off = c3_layout()
    buf = torch.empty(n_bytes, dtype=torch.uint8, device="cuda")
    for i, s in enumerate(contig_starts):
        ctx.synth_bases(buf.data_ptr() + s, C3_CONTIG_LEN, seed_base + i)
        for o in nrun_off:
            buf[s + o:s + o + C3_NRUN_LEN] = ord("N")
        buf[s + C3_CONTIG_LEN] = ord("\n")
    torch.cuda.synchronize()
    return buf, n_bytes


def run_c3_inflight(device, buf, n_bytes, mask, steps, inflight, world):
    """K config-3 builds with `inflight` of them in flight; returns (whole-job
    k-mers/s, max-over-ranks seconds, set of sketch sizes)."""
    import threading
    inflight = max(1, inflight)
    streams = [torch.cuda.Stream() for _ in range(inflight)]
    ctxs = [sksffi.Context(device, st.cuda_stream) for st in streams]

    def build(c):
        return c.sketch_build(buf.data_ptr(), n_bytes, [0, n_bytes], W, mask,
                              sksffi.SKS_FRAC_MOD, C3_FRAC)

    for c in ctxs:  # warm each context's scratch
        del_ = build(c)
        del del_
    kept = [[] for _ in ctxs]
    errors = []

    def worker(i):
        try:
            for _ in range(i, steps, inflight):
                ss = build(ctxs[i])
                kept[i].append((int(ss.windows()[0]), int(ss.sizes()[0])))
                # stream-ordered free: the arrays return to the block cache
                # without waiting for the other build in flight
                ss.free(stream=streams[i].cuda_stream)
        except Exception as e:  # surfaced after the join
            errors.append(e)

    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    threads = [threading.Thread(target=worker, args=(i,)) for i in range(inflight)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    if errors:
        raise errors[0]
    windows = sum(w for k in kept for w, _ in k)
    sizes = {z for k in kept for _, z in k}
    assert windows == steps * c3_windows(), (windows, steps * c3_windows())
    del kept
    total = sum_over_ranks(windows, world)
    return total / elapsed, elapsed, sizes


def run_end_to_end(ctx, mask, buf, steps):
    """Config 3 from FASTA bytes in host memory (SURVEY §8d "end-to-end"): the
    genome as a FASTA file image (80-column lines, one '>' header per contig) in
    pinned host memory; a step = H2D copy + device strings_from_fasta
    (sks_fasta_parse_device) + sketch build + D2H of the sketch.  The sketch
    must equal the HBM-resident run's."""
    contig_starts, n_bytes, _ = c3_layout()
    parts = []
    nl = torch.full((C3_CONTIG_LEN // 80, 1), ord("\n"), dtype=torch.uint8, device="cuda")
    for i, s0 in enumerate(contig_starts):
        hdr = torch.tensor(list(f">syn_3_{i}\n".encode()), dtype=torch.uint8, device="cuda")
        body = buf[s0:s0 + C3_CONTIG_LEN].view(-1, 80)
        parts += [hdr, torch.cat([body, nl], dim=1).reshape(-1)]
    dev_fa = torch.cat(parts)
    total = dev_fa.numel()
    host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev_fa)
    del dev_fa, parts
    raw = torch.empty(total, dtype=torch.uint8, device="cuda")
    stream = torch.empty(total + 1, dtype=torch.uint8, device="cuda")
    ref = ctx.sketch_build(buf.data_ptr(), n_bytes, [0, n_bytes], W, mask, sksffi.SKS_FRAC_MOD,
                           C3_FRAC).sketch(0)
    out = torch.empty(len(ref) + 1, dtype=torch.int64, pin_memory=True)
    ph = {"h2d": 0.0, "parse": 0.0, "sketch": 0.0, "d2h": 0.0}
    tot = 0.0
    for it in range(steps + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        raw.copy_(host, non_blocking=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        nb, nrec = ctx.fasta_parse_device(raw.data_ptr(), total, stream.data_ptr(), total + 1)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ss = ctx.sketch_build(stream.data_ptr(), nb, [0, nb], W, mask, sksffi.SKS_FRAC_MOD, C3_FRAC)
        t3 = time.perf_counter()
        size = ss.copy_into(0, out.data_ptr())
        t4 = time.perf_counter()
        del ss
        if it == 0:
            got = out[:size].numpy().view(np.uint64)
            assert nb == n_bytes and nrec == C3_CONTIGS and np.array_equal(got, ref[:, 0])
            continue
        for k, d in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
            ph[k] += d / steps
        tot += (t4 - t0) / steps
    ov = run_end_to_end_overlapped(ctx, mask, host, ref[:, 0], steps)
    return {"ms": tot * 1e3, "kmers_per_s": c3_windows() / tot, "fasta_bytes": total,
            "ms_phases": {k: v * 1e3 for k, v in ph.items()},
            "pcie_h2d_GBps": total / ph["h2d"] / 1e9,
            "note": "pinned host FASTA -> H2D -> sks_fasta_parse_device -> sks_sketch_build "
                    "-> D2H sketch; sketch equals the HBM-resident run's",
            "overlapped": ov}


def run_end_to_end_overlapped(ctx, mask, host, ref, steps, pieces=8):
    """The same FASTA image cut at record starts into `pieces`: piece p + 1 is
    copied to the device (pinned, its own stream, two slots) while piece p is
    parsed and sketched; FracMinHash keeps a k-mer on its own hash and no
    window crosses a record, so the genome's sketch is the union of the pieces'
    (sks_sketch_union), read back at the end."""
    arr = host.numpy()
    heads = np.flatnonzero(arr == ord(">"))
    heads = heads[(heads == 0) | (arr[np.maximum(heads - 1, 0)] == ord("\n"))]
    total = arr.size
    cuts = [0]
    for p in range(1, pieces):
        j = np.searchsorted(heads, total * p // pieces)
        if j < len(heads) and heads[j] > cuts[-1]:
            cuts.append(int(heads[j]))
    cuts.append(total)
    lens = [cuts[i + 1] - cuts[i] for i in range(len(cuts) - 1)]
    big = max(lens)
    slots = [torch.empty(big, dtype=torch.uint8, device="cuda") for _ in range(2)]
    rec = torch.empty(big + 1, dtype=torch.uint8, device="cuda")
    # HIP maps streams round-robin onto GPU_MAX_HW_QUEUES (4) hardware queues, so
    # a copy stream of normal priority can share the compute stream's queue (it
    # did after the config-3 and config-2 legs had taken six pool streams: every
    # copy then waited behind a piece's kernels, 78 instead of 57 ms); a
    # high-priority stream comes from a queue pool of its own
    copy_stream = torch.cuda.Stream(priority=-1)
    ev = [torch.cuda.Event() for _ in range(2)]
    cat = torch.empty(2 * len(ref) + 4096, dtype=torch.int64, device="cuda")
    uni = torch.empty_like(cat)
    sz_tmp = torch.empty(1, dtype=torch.int32, device="cuda")
    out = torch.empty(len(ref) + 1, dtype=torch.int64, pin_memory=True)

    def h2d(p):
        with torch.cuda.stream(copy_stream):
            slots[p % 2][:lens[p]].copy_(host[cuts[p]:cuts[p + 1]], non_blocking=True)
            ev[p % 2].record(copy_stream)

    def step():
        h2d(0)
        off = windows = 0
        for p in range(len(lens)):
            if p + 1 < len(lens):
                h2d(p + 1)  # overlaps piece p's parse + sketch
            ev[p % 2].synchronize()
            nb, _ = ctx.fasta_parse_device(slots[p % 2].data_ptr(), lens[p], rec.data_ptr(),
                                           lens[p] + 1)
            ss = ctx.sketch_build(rec.data_ptr(), nb, [0, nb], W, mask, sksffi.SKS_FRAC_MOD,
                                  C3_FRAC)
            sz = int(ss.sizes()[0])
            windows += int(ss.windows()[0])
            assert off + sz <= cat.numel()
            ss.export(cat.data_ptr() + 8 * off, max(sz, 1), sz_tmp.data_ptr())
            off += sz
            del ss
        k = ctx.sketch_union(cat.data_ptr(), off, uni.data_ptr())
        out[:k].copy_(uni[:k])  # pinned D2H
        return k, windows

    k, windows = step()
    got = out[:k].numpy().view(np.uint64)
    assert windows == c3_windows() and np.array_equal(got, ref), "overlapped e2e sketch differs"
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    return {"ms": t * 1e3, "kmers_per_s": c3_windows() / t, "pieces": len(lens),
            "note": "FASTA cut at record starts; H2D of piece p+1 (pinned, own stream) overlaps "
                    "parse + sketch of piece p; union of the piece sketches equals the "
                    "HBM-resident sketch"}


def cpu_baseline_c3(mask, budget_bases):
    """Reference-faithful port, 1 core (the reference sketches one genome on one
    worker, kmer_set.cpp:124), on the first `budget_bases` of contig 0."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    _, _, nrun_off = c3_layout()
    seq = synth.bases(budget_bases, seed=3)
    for o in nrun_off:
        if o < budget_bases:
            seq[o:min(budget_bases, o + C3_NRUN_LEN)] = ord("N")
    runs = pyoracle.cut_runs(seq.tobytes())
    codes = np.frombuffer(b"".join(runs), dtype=np.uint8)
    lens = np.array([len(r) for r in runs], dtype=np.uint64)
    windows = int(sum(max(0, int(L) - W + 1) for L in lens))
    t0 = time.perf_counter()
    s = pyoracle.refport_sketch_codes(codes, lens, W, mask, C3_FRAC, 1, 0)
    dt = time.perf_counter() - t0
    size = s.size()
    del s
    return {"value": windows / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"first {budget_bases / 1e6:.0f} Mb of config-3 contig 0 "
                      f"({windows} windows, FracMinHash 1/{C3_FRAC}, set size {size}), "
                      f"oracle/ref_port.cpp, {dt:.1f} s",
            "host": host_info(1)}


def run_c3_sharded(ctx, world, rank, mask, buf, steps, warmup):
    """Config 3 strong scaling: ONE 3 Gb genome (rank 0's) cut into `world`
    chunks with (w-1)-base halos; each rank sketches its chunk, the chunk sets are
    all-gathered and unioned (sks_sketch_union).  The reference cannot split a
    genome at all (one cilk worker per file, kmer_set.cpp:124).  Rank 0 checks
    the result against its whole-genome sketch."""
    import sks_dist
    g = buf if rank == 0 else make_c3(ctx, seed_base=3)[0]
    _, n_bytes, _ = c3_layout()
    dev = "cuda" if os.environ.get("SKS_BENCH_DEVICE") is None else "cpu"

    def build_chunk(a, b):
        ss = ctx.sketch_build(g.data_ptr() + a, b - a, [0, b - a], W, mask, sksffi.SKS_FRAC_MOD,
                              C3_FRAC)
        k = int(ss.sizes()[0])
        out = torch.empty(max(k, 1), dtype=torch.int64, device="cuda")
        ss.export(out.data_ptr(), max(k, 1), torch.zeros(1, dtype=torch.int32,
                                                         device="cuda").data_ptr())
        nw = int(ss.windows()[0])
        del ss
        return out[:k].to(dev), nw

    def union(t):
        t = t.to("cuda").contiguous()
        out = torch.empty_like(t)
        k = ctx.sketch_union(t.data_ptr(), t.numel(), out.data_ptr())
        return out[:k]

    tot = 0.0
    for it in range(warmup + steps):
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sk, nw = sks_dist.sketch_genome_sharded(n_bytes, W, world, rank, build_chunk, union, dev)
        torch.cuda.synchronize()
        dt = max_over_ranks(time.perf_counter() - t0, world)
        if it >= warmup:
            tot += dt / steps
    assert nw == c3_windows()
    if rank == 0:
        whole = ctx.sketch_build(buf.data_ptr(), n_bytes, [0, n_bytes], W, mask,
                                 sksffi.SKS_FRAC_MOD, C3_FRAC).sketch(0)[:, 0]
        assert np.array_equal(sk.cpu().numpy().view(np.uint64), whole)
    return {"metric": "k-mers hashed/s, one genome", "value": nw / tot, "unit": "k-mers/s",
            "scaling": "strong", "ms_per_genome": tot * 1e3, "sketch_size": int(sk.numel()),
            "config": {"workload": "config3 genome split across ranks ((w-1) halos), union",
                       "collective": "all_gather of chunk sketches + all_reduce of windows"
                       if collective() else "none"},
            "check": "equals the whole-genome sketch (rank 0)"}


def cpu_threads():
    """Host cores this process may use (the GPU box gives a share of a larger
    machine: os.cpu_count() shows all of it), capped at 16 — the share a
    one-GPU box grants (MAX_JOBS / OMP_NUM_THREADS are 16 there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def host_info(threads):
    """What a CPU baseline ran on (cores and CPU model with every result)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = None
    return {"threads_used": threads, "os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "cpu_model": model, "thread_cap": "min(16, affinity): the box's CPU share"}


def _codes_lens(seq_bytes, w=W):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    runs = pyoracle.cut_runs(seq_bytes)
    codes = np.frombuffer(b"".join(runs), dtype=np.uint8)
    lens = np.array([len(r) for r in runs], dtype=np.uint64)
    windows = int(sum(max(0, int(L) - w + 1) for L in lens))
    return codes, lens, windows


def cpu_baseline_c2(host_genome, mask, gpu_sketch):
    """Config 2 on the host: the reference-style port (oracle/ref_port.cpp:
    heap bitsets, per-window kmer, std::function predicate, with the bottom-s
    kept in std::set / unordered_map — the reference has no bottom-s) over the
    whole 5 Mb genome on one core (one genome = one cilk worker,
    kmer_set.cpp:124).  The set is checked equal to the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    codes, lens, windows = _codes_lens(host_genome)
    t0 = time.perf_counter()
    s = pyoracle.refport_bottom_codes(codes, lens, W, mask, C2_S)
    dt = time.perf_counter() - t0
    assert np.array_equal(s.elems(), gpu_sketch), "config-2 CPU set differs from the GPU's"
    return {"value": windows / dt, "unit": "k-mers/s", "cores": 1, "kind": "port",
            "sample": f"the whole config-2 genome ({windows} windows, bottom-s {C2_S}), "
                      f"oracle/ref_port.cpp bottom_runs, {dt:.2f} s; set equal to the GPU's",
            "host": host_info(1)}


def cpu_sketch_many(host_genomes, mask, kind, param, threads, w=W):
    """Reference-style port over genomes, `threads` workers over genomes (the
    reference's cilk_for over files, kmer_set.cpp:112-133). Returns (sets, windows, s)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from concurrent.futures import ThreadPoolExecutor
    prepared = [_codes_lens(g, w) for g in host_genomes]

    def one(i):
        codes, lens, _ = prepared[i]
        if kind == "bottom":
            return pyoracle.refport_bottom_codes(codes, lens, w, mask, param)
        return pyoracle.refport_sketch_codes(codes, lens, w, mask, param)
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        sets = list(ex.map(one, range(len(prepared))))
    dt = time.perf_counter() - t0
    return sets, sum(p[2] for p in prepared), dt


def cpu_crosscheck_c3(ctx, buf, mask, sample_bytes):
    """Optimised multi-core CPU cross-check: the oracle restatement
    (u128 rolling windows, exact hash; oracle/sks_oracle.cpp) on the first
    `sample_bytes` of the config-3 genome, cut into one chunk per thread with
    (w-1)-base halos, the chunk sets unioned.  Checked equal to the GPU sketch of
    the same prefix."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from concurrent.futures import ThreadPoolExecutor
    T = cpu_threads()
    host = buf[:sample_bytes].cpu().numpy().tobytes()
    cuts = [sample_bytes * i // T for i in range(T + 1)]

    def one(i):
        a, b = cuts[i], min(sample_bytes, cuts[i + 1] + W - 1)
        sk, nw = pyoracle.sketch(pyoracle.cut_runs(host[a:b]), W, mask, "frac", C3_FRAC)
        return sk[:, 0], nw
    t0 = time.perf_counter()
    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(one, range(T)))
    union = np.unique(np.concatenate([r[0] for r in res]))
    dt = time.perf_counter() - t0
    windows = sum(r[1] for r in res)
    dev = torch.empty(sample_bytes + 1, dtype=torch.uint8, device="cuda")
    dev[:sample_bytes] = buf[:sample_bytes]
    dev[sample_bytes] = ord("\n")
    gpu = ctx.sketch_build(dev.data_ptr(), sample_bytes + 1, [0, sample_bytes + 1], W, mask,
                           sksffi.SKS_FRAC_MOD, C3_FRAC)
    assert np.array_equal(gpu.sketch(0)[:, 0], union) and int(gpu.windows()[0]) == windows
    return {"value": windows / dt, "unit": "k-mers/s", "cores": T, "kind": "port (optimised)",
            "sample": f"first {sample_bytes / 1e6:.0f} MB of the config-3 genome, {T} chunks with "
                      f"(w-1) halos, oracle/sks_oracle.cpp u128 rolling window, "
                      f"{dt:.1f} s; set equal to the GPU's",
            "host": host_info(T)}


# ---- config 2 ------------------------------------------------------------------------
C2_LEN, C2_SEED, C2_S, C2_BATCH = 5_000_000, 2, 10000, 64


def run_c2(ctx, mask, steps, warmup, inflight=2, cpu=False):
    """Config 2 of BASELINE.json: one 5 Mb bacterial-scale genome (synthetic,
    seed 2), w=31/k=21 spaced seed, bottom-s s=10000.  One such build is
    launch/latency-bound (a metadata upload, the scan, the fused bottom-s
    kernel writing the set's arrays and one read-back: api.cpp
    build_bottom_single), so three numbers are reported, each named for what
    it is:
      * single: K builds one at a time — wall time per build (k-mers/s of a
        complete sks_sketch_build) and the scan kernel's own time (hipEvents)
        with its HBM roofline fraction;
      * inflight: the same single-genome build with `inflight` contexts on their
        own HIP streams and host threads (builds overlap);
      * batched: C2_BATCH distinct 5 Mb genomes (genome 0 = the config-2
        genome) in ONE sks_sketch_build call (the reference's per-file sets,
        kmer_set.cpp:112-133, in one launch sequence).
    Every sketch is checked against the first build (and batch genome 0 equal to
    it); the oracle comparison at this size is tests/test_gpu_parity.py::
    test_config2_5mb_bottom_s."""
    import threading
    seg_len = C2_LEN + 1
    buf = torch.empty(seg_len * C2_BATCH, dtype=torch.uint8, device="cuda")
    for i in range(C2_BATCH):
        ctx.synth_bases(buf.data_ptr() + i * seg_len, C2_LEN, C2_SEED if i == 0 else 2000 + i)
        buf[i * seg_len + C2_LEN] = ord("\n")
    torch.cuda.synchronize()
    windows = C2_LEN - W + 1

    def one(c):
        return c.sketch_build(buf.data_ptr(), seg_len, [0, seg_len], W, mask, sksffi.SKS_BOTTOM_S, C2_S)

    ref = one(ctx).sketch(0)
    for _ in range(warmup):
        del_ = one(ctx)
        del del_
    scan_ms, surv = [], []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ss = one(ctx)
        t = ctx.timings()
        scan_ms.append(t["scan_ms"])
        surv.append(t["survivors"])
        assert int(ss.windows()[0]) == windows
        del ss
    torch.cuda.synchronize()
    t_single = (time.perf_counter() - t0) / steps
    scan = float(np.median(scan_ms))
    # bottom-s candidates are written as (k-mer, k-mer) record pairs: 16 B each
    alg = seg_len + 16 * float(np.mean(surv))
    achieved = alg / (scan * 1e-3) / 1e9

    # in flight: one context + stream + host thread per build in flight
    streams = [torch.cuda.Stream() for _ in range(max(1, inflight))]
    ctxs = [sksffi.Context(torch.cuda.current_device(), st.cuda_stream) for st in streams]
    for c in ctxs:
        assert np.array_equal(one(c).sketch(0), ref)
    errors = []

    def worker(i):
        try:
            for _ in range(i, steps, len(ctxs)):
                ss = one(ctxs[i])
                ss.free(stream=streams[i].cuda_stream)
        except Exception as e:  # surfaced after the join
            errors.append(e)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(len(ctxs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    t_inflight = (time.perf_counter() - t0) / steps
    if errors:
        raise errors[0]

    # batched: C2_BATCH genomes in one build
    seg = [i * seg_len for i in range(C2_BATCH + 1)]
    bs = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, W, mask, sksffi.SKS_BOTTOM_S, C2_S)
    assert np.array_equal(bs.sketch(0), ref) and (bs.sizes() == C2_S).all()
    del bs
    reps = max(2, steps // 4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        bs = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, W, mask, sksffi.SKS_BOTTOM_S, C2_S)
        bt = ctx.timings()
        del bs
    torch.cuda.synchronize()
    t_batch = (time.perf_counter() - t0) / reps
    bscan = bt["scan_ms"]
    balg = seg[-1] + 16 * bt["survivors"]
    cpu_b = None
    if cpu:
        cpu_b = cpu_baseline_c2(buf[:C2_LEN].cpu().numpy().tobytes(), mask, ref)
    del buf
    return {
        "metric": "k-mers hashed/s, config 2", "unit": "k-mers/s", "steps": steps,
        "config": {"workload": "config2: 1x5 Mb genome, spaced seed w=31/k=21 (mask seed 0), "
                               "bottom-s s=10000", "genome_len": C2_LEN, "s": C2_S,
                   "windows_per_genome": windows},
        "single": {"kmers_per_s_build": windows / t_single, "ms_per_build": t_single * 1e3,
                   "scan_kernel_ms": scan, "kmers_per_s_scan": windows / (scan * 1e-3),
                   "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                                "algorithmic_bytes_per_launch": alg},
                   "note": "one complete build at a time, wall clock incl. host syncs; the "
                           "scan kernel alone by hipEvents"},
        "inflight": {"builds_in_flight": len(ctxs), "kmers_per_s": windows / t_inflight,
                     "ms_per_build": t_inflight * 1e3},
        "cpu_baseline": cpu_b,
        "batched": {"genomes_per_build": C2_BATCH, "kmers_per_s": C2_BATCH * windows / t_batch,
                    "ms_per_build": t_batch * 1e3, "scan_kernel_ms": bscan,
                    "scan_roofline_frac": balg / (bscan * 1e-3) / 1e9 / HBM_PEAK_GBS},
    }


# ---- config 4 ------------------------------------------------------------------------
def c4_genome_seeds(g):
    anc = g // (C4_GENOMES // C4_ANCESTORS)
    desc = g % (C4_GENOMES // C4_ANCESTORS)
    return 100 + anc, 1000 + g, desc * 0.001


def cpu_baseline_pairs(ctx, buf, seg, mask, counts, n_sets=100, w=W):
    """Reference-faithful pair phase on the host (oracle/ref_port.cpp: unordered_map
    kmer_sets, probe-the-larger intersection, threads over pairs like the
    reference's cilk_for, kmer_set.cpp:23-41,167-184) over all ordered pairs of
    the first `n_sets` config-4 genomes' sketches (same family: sharing is high).
    Then containment + ANI per ordered pair, serially like the reference's
    loop (kmer-sketching.cpp:195-200, ani_estimation.cpp:24-42), inside the
    clock.  Counts are checked against the GPU matrix."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    T = cpu_threads()
    ss = ctx.sketch_build(buf.data_ptr(), seg[n_sets], seg[:n_sets + 1], w, mask,
                          sksffi.SKS_BOTTOM_S, C4_S)
    sets = [pyoracle.refport_set_from_elems(ss.sketch(i), w, mask) for i in range(n_sets)]
    ones = bin(mask).count("1") // 2
    t0 = time.perf_counter()
    got = pyoracle.refport_all_pairs(sets, threads=T)
    sz = np.diag(got)
    ani = [pyoracle.binomial_estimator(pyoracle.containment(int(got[i, j]), int(sz[i])), ones)
           for i in range(n_sets) for j in range(n_sets)]
    dt = time.perf_counter() - t0
    assert np.array_equal(got, counts[:n_sets, :n_sets])
    del ani
    return {"value": n_sets * n_sets / dt, "unit": "ordered pairs/s (count + containment + ANI)", "cores": T,
            "kind": "port",
            "sample": f"all {n_sets}x{n_sets} ordered pairs of the first {n_sets} genomes "
                      f"(s={C4_S}, w={w}: {'128' if w > 32 else '64'}-bit k-mers in heap bitsets), "
                      f"oracle/ref_port.cpp, {T} threads over pairs + serial ANI, {dt:.2f} s; "
                      f"counts equal the GPU's",
            "host": host_info(T)}


def cpu_baseline_c4_sketch(ctx, buf, seg, mask, w=W):
    """Config 4's sketch phase on the host: the reference-style port over a
    bounded sample of the genomes, one worker thread per host core over genomes
    (the reference's cilk_for over files, kmer_set.cpp:112-133); every sampled
    set is checked equal to the GPU's."""
    T = cpu_threads()
    n = min(len(seg) - 1, 4 * T)
    ss = ctx.sketch_build(buf.data_ptr(), seg[n], seg[:n + 1], w, mask, sksffi.SKS_BOTTOM_S, C4_S)
    host = [buf[seg[i]:seg[i + 1]].cpu().numpy().tobytes() for i in range(n)]
    sets, windows, dt = cpu_sketch_many(host, mask, "bottom", C4_S, T, w=w)
    for i in range(n):
        assert np.array_equal(sets[i].elems(), ss.sketch(i)), f"config-4 CPU set {i} differs"
    return {"value": windows / dt, "unit": "k-mers/s", "cores": T, "kind": "port",
            "sample": f"{n} of the {C4_GENOMES} config-4 genomes (5 Mb each, {windows} windows, "
                      f"w={w}, bottom-s {C4_S}), oracle/ref_port.cpp bottom_runs, {T} threads over "
                      f"genomes, {dt:.2f} s; sets equal to the GPU's",
            "host": host_info(T)}


def run_pairs(ctx, world, rank, mask, steps, warmup, cpu_pairs=False, w=W):
    """Config 4 all-vs-all.  Timed per step: the sketch phase (every rank's
    genomes), then the pair phase = counts for every ordered pair + containment
    and ANI on the device + the ANI copied into pinned host memory (the whole
    "comparison" of kmer-sketching.cpp:185-203).  A second pass times the counts
    alone (layout + join, no ANI) for the fixed-cost figure.  w > 32 (the
    reference sweep's (k+10, k) shapes, kmer-sketching.cpp:228-239) runs the
    same flow on 128-bit k-mers: 16-byte values in the sketches, the layout
    and the join (elem_words 2)."""
    import sks_dist
    _, g0, g1 = sks_dist.block_shard(C4_GENOMES, world, rank)
    n_local = g1 - g0
    seg = [0]
    for _ in range(n_local):
        seg.append(seg[-1] + C4_LEN + 1)
    buf = torch.empty(max(seg[-1], 1), dtype=torch.uint8, device="cuda")
    for i in range(n_local):
        anc_seed, mut_seed, rate = c4_genome_seeds(g0 + i)
        ctx.synth_bases(buf.data_ptr() + seg[i], C4_LEN, anc_seed, mut_seed, rate)
        buf[seg[i] + C4_LEN] = ord("\n")
    torch.cuda.synchronize()
    ones = bin(mask).count("1") // 2
    ops = sks_dist.GpuJoinOps(ctx, ew=2 if w > 32 else 1)
    # one rank without a process group counts every tile of one layout; with one
    # (N > 1, or the world-1 RCCL rehearsal) the cyclic tile plan and the sketch
    # exchange.  Either way the join writes every counted pair's ANI straight
    # into this pinned host matrix (sks_intersect_layout_ani; each rank the cells
    # of its own tiles), so no ANI kernel or device-to-host copy follows the join
    solo = world == 1 and not collective()
    host_ani = sksffi.HostBuffer(C4_GENOMES * C4_GENOMES * 8)
    host_ani.array[:] = 0.0

    def pair_step(ss, with_ani=True):
        return sks_dist.all_vs_all_join(C4_GENOMES, world, rank, sks_dist.sketches_of(ss, ew=ops.ew), ops,
                                        sksffi.join_layout_log_b, device="cuda", dst=None,
                                        ani_ones=ones if with_ani else None,
                                        ani_out=host_ani if with_ani else None,
                                        max_size=int(ss.sizes().max()) if ss is not None and ss.n else None,
                                        size_bound=C4_S, exchange=EXCHANGE, world1_exchange=WORLD1_EXCHANGE,
                                        bounds_mask=mask)

    t_sketch = t_pairs = t_counts = 0.0
    timed = 0
    k_all = []
    res = ss = None
    sizes = np.zeros(0, np.uint32)
    for it in range(warmup + steps):
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ss = None
        if n_local:
            ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, C4_S)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = pair_step(ss)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ts, tp = max_over_ranks(t1 - t0, world), max_over_ranks(t2 - t1, world)
        if it >= warmup:
            t_sketch += ts
            t_pairs += tp
            timed += 1
    sizes = ss.sizes().copy() if ss is not None else sizes
    # counts alone (the fixed-cost figure: pair phase minus the join kernel)
    for it in range(1 + steps):
        barrier(world)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        pair_step(ss, with_ani=False)
        torch.cuda.synchronize()
        tc = max_over_ranks(time.perf_counter() - t1, world)
        if it >= 1:
            t_counts += tc
            # the rank's last join launch: at N = 1 every tile in one launch (the
            # timed steps above count tile-row parts, one launch each)
            k_all.append(ctx.last_intersect_ms())
    k_ms = float(np.mean(k_all)) if k_all else None
    t_sketch /= max(timed, 1)
    t_pairs /= max(timed, 1)
    t_counts /= max(steps, 1)
    res.check_layouts()  # every join layout of the last timed step was valid
    ani = host_ani.array.reshape(C4_GENOMES, C4_GENOMES)
    counts = None
    # the rank's tiles' counts placed in the n x n matrix (zero elsewhere)
    mat = sks_dist.place_tiles(torch.zeros((C4_GENOMES, C4_GENOMES), dtype=torch.int32, device="cuda"),
                               res.tiles, res.counts, C4_GENOMES).cpu().numpy()
    # the fused ANI against the host's (kmer-sketching.cpp:195-200 on the exact
    # counts), on every cell this rank's tiles cover
    covered = np.zeros((C4_GENOMES, C4_GENOMES), bool)
    for I, J in np.asarray(res.tiles).reshape(-1, 2):
        covered[I * 64:(I + 1) * 64, J * 64:(J + 1) * 64] = True
        covered[J * 64:(J + 1) * 64, I * 64:(I + 1) * 64] = True
    all_sizes = np.zeros(C4_GENOMES, np.int64)
    all_sizes[g0:g1] = sizes
    all_sizes = sum_vector_over_ranks(all_sizes, world)
    rows_i = np.nonzero(covered)[0]
    _, h_ani = sksffi.ani_from_counts(mat[covered], all_sizes[rows_i].astype(np.int32), ones)
    ani_err = float(np.abs(ani[covered] - h_ani).max()) if covered.any() else 0.0
    assert ani_err <= 1e-9, ani_err
    ani_mean = sum_over_ranks(float(ani[covered].sum()), world) / (C4_GENOMES * C4_GENOMES)
    if solo:
        counts = mat
        assert (counts == counts.T).all() and counts[0, 1] > 0
        assert (np.diag(counts) == sizes).all()
    cpu = cpu_sk = None
    if cpu_pairs and rank == 0 and solo:
        cpu = cpu_baseline_pairs(ctx, buf, seg, mask, counts, w=w)
        cpu_sk = cpu_baseline_c4_sketch(ctx, buf, seg, mask, w=w)
    ani_bytes = int(covered.sum()) * 8
    return {
        "metric": "genome-pairs ANI/s", "value": C4_GENOMES * C4_GENOMES / t_pairs,
        "unit": "ordered pairs/s (count + containment + ANI, ANI in host memory)", "scaling": "strong",
        "ms_pair_phase": t_pairs * 1e3, "ms_sketch_phase": t_sketch * 1e3,
        "ms_counts_phase": t_counts * 1e3,
        "pair_kernel_ms_rank0": k_ms,
        "pair_kernel_timing": "hipEvents around the k_join launch on the context stream, mean over the counts-only "
                              "steps (one launch for all tiles at N = 1)",
        "fixed_cost_ms": (t_counts * 1e3 - k_ms) if k_ms else None,
        "ani_readback_bytes_rank0": ani_bytes,
        "ani_max_abs_err_vs_host": ani_err,
        # streamed-equivalent bytes of the pair kernel, 8 B per
        # element of both sets + 4 B per count, for every ordered pair this rank's
        # tiles cover; a measure of reuse, not an HBM claim (the join is bound by
        # LDS round trips: see pairs_lds in the round's profile)
        "roofline_streamed_equivalent": {
            "bytes_per_pair": 8 * 2 * C4_S + 4,
            "pairs_this_rank": C4_GENOMES * C4_GENOMES / world,
            "achieved_GBps": (8 * 2 * C4_S + 4) * C4_GENOMES * C4_GENOMES / world / (k_ms * 1e-3) / 1e9
            if k_ms else None},
        "roofline": pairs_lds_roofline(k_ms, "pair_lds.json" if w == W else "pair_lds_wide.json") if solo else None,
        "sketch_kmers_per_s": C4_GENOMES * (C4_LEN - w + 1) / t_sketch,
        "ani_mean_all_pairs": ani_mean,
        "config": {"workload": "config4 all-vs-all", "genomes": C4_GENOMES,
                   "genome_len": C4_LEN, "s": C4_S, "w": w, "k": ones,
                   "kmer_bits": 128 if w > 32 else 64,
                   "pair_sharding": "block-aligned genomes per rank; cyclic tile plan: the rank's own "
                                    "blocks' 64x64 join tiles, then every tile pairing its blocks with "
                                    "ranks r+1 .. r+N/2 (the N/2 pairs split) as their sketches land",
                   "ani": "written by the join (last workgroup of each tile) into pinned host memory",
                   "collective": (f"sketch exchange '{EXCHANGE}' of sketches padded to s ({backend_label()}); "
                                  f"group bounds from the mask on every rank (no broadcast)"
                                  if collective() else "none")},
        "cpu_baseline": cpu,
        "cpu_baseline_sketch_phase": cpu_sk,
        "end_to_end_pairs_per_s": C4_GENOMES * C4_GENOMES / (t_sketch + t_pairs),
        "ms_end_to_end": (t_sketch + t_pairs) * 1e3,
    }


# ---- the reference's own flow: main's 62 (w, k) configurations --------------------------
REF_SWEEP_GENOMES, REF_SWEEP_CPU_GENOMES = 64, 16
REF_SWEEP_CPU_CONFIGS = ((21, 21), (31, 31), (45, 35), (50, 40))


def ref_sweep_configs():
    """kmer-sketching.cpp:218-238: (10,10); (k,k) k = 11..40; (k+10,k) k = 10..40."""
    return [(10, 10)] + [(k, k) for k in range(11, 41)] + [(k + 10, k) for k in range(10, 41)]


def _fasta_files(ctx, n, d):
    """The first n config-4 genomes as FASTA files (80-column lines) in d."""
    files = []
    dev = torch.empty(C4_LEN, dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = c4_genome_seeds(g)
        ctx.synth_bases(dev.data_ptr(), C4_LEN, a, m, r)
        seq = dev.cpu().numpy().tobytes()
        path = os.path.join(d, f"g{g:03d}.fa")
        with open(path, "wb") as f:
            f.write(b">syn_%d_0\n" % g)
            f.write(b"\n".join(seq[i:i + 80] for i in range(0, len(seq), 80)) + b"\n")
        files.append(path)
    return files


def cpu_ref_sweep(files, configs):
    """The reference's per-configuration flow on the host (kmer-sketching.cpp:151-212)
    for a bounded sample: every file parsed again (the reference re-reads its
    files per configuration, :168; oracle/sks_oracle.cpp's restatement of
    fasta_processing.cpp), sketched with sketching_condition (c = 200) by the
    reference-faithful port, threads over files (kmer_set.cpp:112-133); every
    ordered pair counted, threads over pairs (kmer_set.cpp:167-184); ANI serial
    (:195-200).  Returns per-config (sketch s, compare s, windows, counts)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    from concurrent.futures import ThreadPoolExecutor
    T = cpu_threads()
    out = []
    for w, k in configs:
        m = pyoracle.mask(w, k, 0)
        ones = bin(m).count("1") // 2

        def one(path):
            runs = pyoracle.fasta_runs(path)
            codes = np.frombuffer(b"".join(runs), dtype=np.uint8)
            lens = np.array([len(r) for r in runs], dtype=np.uint64)
            nw = int(sum(max(0, int(L) - w + 1) for L in lens))
            return pyoracle.refport_sketch_codes(codes, lens, w, m, 200), nw
        t0 = time.perf_counter()
        with ThreadPoolExecutor(T) as ex:
            res = list(ex.map(one, files))
        t1 = time.perf_counter()
        sets = [r[0] for r in res]
        counts = pyoracle.refport_all_pairs(sets, threads=T)
        sz = np.diag(counts)
        ani = [pyoracle.binomial_estimator(pyoracle.containment(int(counts[i, j]), int(sz[i])), ones)
               for i in range(len(files)) for j in range(len(files))]
        t2 = time.perf_counter()
        out.append({"w": w, "k": k, "sketch_s": t1 - t0, "compare_s": t2 - t1,
                    "windows": sum(r[1] for r in res), "counts": counts, "ani": ani})
    return out, T


def run_ref_sweep(ctx, cpu=False):
    """The reference's own workload (kmer-sketching.cpp:214-239, main): its 62
    (w, k) configurations — 36 of them at w <= 32 (u64 k-mers), 26 at w > 32
    (128-bit) — each sketching every file (FracMinHash c = 200, the reference's
    sketching_condition, :29-34) and comparing all ordered pairs into ANI and
    the CSV, run by this engine's drop-in driver bin/kmer-sketching (the facade:
    sks::genome_batch parses the files once on the device and keeps them in HBM,
    then sketch + all-pairs per configuration) on 64 config-4 genome files.  The
    driver prints the reference's two timing lines per configuration; the CPU
    baseline runs the same flow, reference-style, on the first 16 files for 4
    configurations, and its ANI equals the CSV's for those pairs."""
    import subprocess
    import tempfile
    n = REF_SWEEP_GENOMES
    d = tempfile.mkdtemp(prefix="sks_refsweep_", dir="/tmp")
    try:
        files = _fasta_files(ctx, n, d)
        torch.cuda.synchronize()
        exe = os.path.join(PKG, "bin", "kmer-sketching")
        out_csv = os.path.join(d, "out.csv")
        t0 = time.perf_counter()
        p = subprocess.run([exe, out_csv] + files, capture_output=True, text=True, timeout=900)
        wall = time.perf_counter() - t0
        if p.returncode != 0:
            raise RuntimeError(f"bin/kmer-sketching failed ({p.returncode}): {p.stderr[-2000:]}")
        sk = [float(l.split("=")[1].split()[0]) for l in p.stdout.splitlines() if "Time taken for sketching" in l]
        cp = [float(l.split("=")[1].split()[0]) for l in p.stdout.splitlines() if "Time taken for comparison" in l]
        cfg = ref_sweep_configs()
        assert len(sk) == len(cp) == len(cfg), (len(sk), len(cp))
        rows = sum(1 for _ in open(out_csv)) - 1
        assert rows == len(cfg) * n * n, rows
        narrow = [i for i, (w, _) in enumerate(cfg) if w <= 32]
        wide = [i for i, (w, _) in enumerate(cfg) if w > 32]
        wins = {i: n * (C4_LEN - w + 1) for i, (w, _) in enumerate(cfg)}

        def part(ix):
            s, c = sum(sk[i] for i in ix), sum(cp[i] for i in ix)
            return {"configs": len(ix), "sketch_ms_per_config": s / len(ix), "compare_ms_per_config": c / len(ix),
                    "sketch_ms_median": statistics.median(sk[i] for i in ix),
                    "compare_ms_median": statistics.median(cp[i] for i in ix),
                    "sketch_ms_max": max(sk[i] for i in ix), "compare_ms_max": max(cp[i] for i in ix),
                    "sketch_kmers_per_s": sum(wins[i] for i in ix) / (s * 1e-3),
                    "compare_pairs_per_s": len(ix) * n * n / (c * 1e-3)}
        res = {"metric": "reference sweep (kmer-sketching main), 62 (w, k) configs",
               "per_config_ms": [{"w": w_, "k": k_, "sketch": round(sk[i], 4), "compare": round(cp[i], 4)}
                                 for i, (w_, k_) in enumerate(cfg)],
               "genomes": n, "genome_len": C4_LEN, "pairs_per_config": n * n,
               "driver": "spaced-kmer-sketching_amd/bin/kmer-sketching: this engine's restatement of the reference "
                         "main (apps/kmer_sketching.cpp + cpp/sweep.cpp) - files parsed once and kept in HBM, the "
                         "sketch step with the FracMinHash descriptor on the device (not the reference's "
                         "std::function predicate: that flow is dropin_std_function), all pairs + ANI in one fused "
                         "native call",
               "wall_s": wall, "csv_rows": rows,
               "sketch_ms_total": sum(sk), "compare_ms_total": sum(cp),
               "w_le_32": part(narrow), "w_gt_32": part(wide),
               "note": "per-configuration times are the driver's own 'Time taken for sketching / comparison' "
                       "lines (kmer-sketching.cpp:174-175, 202-203 on the same boundaries); the files are parsed "
                       "once, on the device, before the first configuration (the reference re-parses them per "
                       "configuration); wall_s includes process start, that parse and the CSV writing"}
        res["dropin_std_function"] = run_dropin_flow(files)
        if cpu:
            csel = REF_SWEEP_CPU_CONFIGS
            cres, T = cpu_ref_sweep(files[:REF_SWEEP_CPU_GENOMES], csel)
            # the GPU's CSV values for the same pairs (6 significant digits, the
            # reference's default ostream formatting) equal the CPU's ANI
            vals = {}
            want_rows = {}
            for c in cres:
                ci = cfg.index((c["w"], c["k"]))
                for i in range(REF_SWEEP_CPU_GENOMES):
                    for j in range(REF_SWEEP_CPU_GENOMES):
                        want_rows[1 + ci * n * n + i * n + j] = (c["ani"][i * REF_SWEEP_CPU_GENOMES + j])
            with open(out_csv) as f:
                for ln, line in enumerate(f):
                    if ln in want_rows:
                        vals[ln] = line.split(",")[2]
            bad = [ln for ln, a in want_rows.items() if vals[ln] != f"{a:.6g}"]
            assert not bad, f"{len(bad)} CSV values differ from the CPU flow's, e.g. row {bad[0]}"
            g = REF_SWEEP_CPU_GENOMES
            per = []
            for c in cres:
                ci = cfg.index((c["w"], c["k"]))
                per.append({"w": c["w"], "k": c["k"], "cpu_sketch_ms": c["sketch_s"] * 1e3,
                            "cpu_compare_ms": c["compare_s"] * 1e3,
                            "cpu_sketch_kmers_per_s": c["windows"] / c["sketch_s"],
                            "cpu_compare_pairs_per_s": g * g / c["compare_s"],
                            "gpu_sketch_kmers_per_s": wins[ci] / (sk[ci] * 1e-3),
                            "gpu_compare_pairs_per_s": n * n / (cp[ci] * 1e-3)})
            # projected reference-style host time of the whole sweep on the 64 files,
            # from the sampled rates (sketch per window, compare per pair)
            rk = {32: [], 64: []}
            for x in per:
                rk[32 if x["w"] <= 32 else 64].append(x)
            proj = 0.0
            for i, (w, _) in enumerate(cfg):
                xs = rk[32 if w <= 32 else 64]
                ks = statistics.mean(x["cpu_sketch_kmers_per_s"] for x in xs)
                ps = statistics.mean(x["cpu_compare_pairs_per_s"] for x in xs)
                proj += wins[i] / ks + n * n / ps
            for x in res["dropin_std_function"]["per_config"]:
                c = next((y for y in per if (y["w"], y["k"]) == (x["w"], x["k"])), None)
                if c is not None:  # the reference-style host flow at this file count, from its sampled rate
                    x["cpu_port_sketch_ms_64_files"] = x["windows"] / c["cpu_sketch_kmers_per_s"] * 1e3
                    x["speedup_vs_cpu_port"] = x["cpu_port_sketch_ms_64_files"] / x["std_function_ms"]
            res["cpu_baseline"] = {
                "kind": "port", "cores": T,
                "sample": f"the first {g} of the {n} files, configurations {list(csel)}: per configuration every file "
                          f"parsed again, sketched (oracle/ref_port.cpp, c = 200, {T} threads over files) and every "
                          f"ordered pair counted ({T} threads over pairs) + serial ANI; ANI equal to the GPU CSV's",
                "per_config": per,
                "projected_sweep_s_64_files": proj,
                "gpu_sweep_s_64_files": (sum(sk) + sum(cp)) * 1e-3,
                "host": host_info(T)}
        return res
    finally:
        import shutil
        shutil.rmtree(d, ignore_errors=True)


def run_dropin_flow(files):
    """The reference driver's sketching step as an UNMODIFIED caller runs it
    (kmer-sketching.cpp:165-175): parallel_kmer_sets_from_fasta_files with the
    reference's global-function predicate sketching_condition (:29-34) as a
    std::function — the GPU extracts every window (sks_windows_dense), the
    predicate runs on host threads, one pooled device worker per thread with
    pinned double buffers — beside the same call with the device-side
    descriptor (sketch_policy::frac(200)); bin/dropin-flow asserts the sets are
    equal.  Per configuration: both times, the window rows' device-to-host
    bytes, their copy time and effective rate, the host predicate time, and
    which of the two bounds the flow."""
    import subprocess
    exe = os.path.join(PKG, "bin", "dropin-flow")
    cfg = ",".join(f"{w}:{k}" for w, k in REF_SWEEP_CPU_CONFIGS)
    p = subprocess.run([exe, cfg] + list(files), capture_output=True, text=True, timeout=900)
    if p.returncode != 0:
        raise RuntimeError(f"bin/dropin-flow failed ({p.returncode}): {p.stderr[-2000:]}")
    per = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    for x in per:
        thr = max(1, x["threads"])
        x["d2h_GBps_effective"] = x["d2h_bytes"] / (x["std_function_ms"] * 1e-3) / 1e9
        x["d2h_GBps_copy"] = x["d2h_bytes"] / (x["d2h_ms_sum"] * 1e-3) / 1e9 * thr if x["d2h_ms_sum"] else None
        x["predicate_ms_per_thread"] = x["predicate_ms_sum"] / thr
        x["predicate_ns_per_window"] = x["predicate_ms_sum"] * 1e6 / max(1, x["windows"])
        x["bound"] = ("host predicate" if x["predicate_ms_per_thread"] >= 0.75 * x["std_function_ms"]
                      else "device / PCIe")
        assert x["sets_equal"]
    return {"driver": "spaced-kmer-sketching_amd/bin/dropin-flow (apps/dropin_flow.cpp: the reference's "
                      "sketching_condition passed to parallel_kmer_sets_from_fasta_files unchanged)",
            "files": len(files), "per_config": per,
            "note": "std_function_ms: wall time of the unmodified call; descriptor_ms: the same call with "
                    "sketch_policy::frac(200) (selection on the GPU); d2h_GBps_copy: bytes over the summed "
                    "per-worker copy durations (HIP events) x threads, i.e. the rate while copies run"}


# ---- config 5 ------------------------------------------------------------------------
def cpu_baseline_c5(ctx, buf, seg, masks, ones):
    """Config 5 on the host over a bounded sample: 2 of the 8 seeds x the first
    G genomes; per seed the reference-style port sketches the genomes (threads
    over genomes, kmer_set.cpp:112-133), counts all G x G ordered pairs
    (threads over pairs, kmer_set.cpp:167-184) and computes containment and ANI
    (ani_estimation.cpp:24-42, the oracle's restatement); the timed region is
    the whole per-seed pipeline, like a GPU sweep step.  Seed 0's counts are
    checked against the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    T = cpu_threads()
    G = min(len(seg) - 1, 2 * T)
    seeds = [0, 1]
    host = [buf[seg[i]:seg[i + 1]].cpu().numpy().tobytes() for i in range(G)]
    t_all = 0.0
    windows = 0
    counts0 = None
    for sd in seeds:
        sets, nw, dt = cpu_sketch_many(host, masks[sd], "bottom", C4_S, T)
        t0 = time.perf_counter()
        counts = pyoracle.refport_all_pairs(sets, threads=T)
        sizes = np.diag(counts)
        ani = [pyoracle.binomial_estimator(pyoracle.containment(int(counts[i, j]), int(sizes[i])),
                                           ones[sd]) for i in range(G) for j in range(G)]
        t_all += dt + time.perf_counter() - t0
        windows += nw
        if sd == 0:
            counts0 = counts
        del ani
    seg0 = seg[:G + 1]
    ss = ctx.sketch_build(buf.data_ptr(), seg0[-1], seg0, W, masks[0], sksffi.SKS_BOTTOM_S, C4_S)
    out = torch.zeros((G, G), dtype=torch.int32, device="cuda")
    d, st, sz = ss.device_ptrs()
    ctx.intersect_all(d, st, sz, 1, G, 0, G, out.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), counts0), "config-5 CPU counts differ from the GPU's"
    return {"value": len(seeds) * G * G / t_all, "unit": "ordered (pair, seed) ANIs/s", "cores": T,
            "kind": "port", "sketch_kmers_per_s": windows / t_all,
            "sample": f"{len(seeds)} of the {C5_SEEDS} seeds x the first {G} genomes "
                      f"({G * G} ordered pairs per seed, bottom-s {C4_S}): sketch (threads over "
                      f"genomes) + all pairs (threads over pairs) + containment/ANI, "
                      f"oracle/ref_port.cpp, {t_all:.2f} s; seed-0 counts equal the GPU's",
            "host": host_info(T)}


def run_seed_sweep(ctx, world, rank, steps, warmup, lanes_n=2, cpu=False):
    """Config 5: 8 spaced seeds (w=31/k=21, mask seeds 0..7) over the first 200
    genomes of config 4, bottom-s s=10000; per seed: sketch all genomes, count
    all 200 x 200 ordered pairs (symmetric tiles), containment + ANI on the host
    (bit-exact doubles, kmer-sketching.cpp:195-200); consensus = mean ANI over
    the seeds.  Ranks shard seeds (sks_dist.seed_sweep); one all-reduce of the
    ANI sums.  A step is the whole sweep, consensus included."""
    import sks_dist
    n = C5_GENOMES
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + C4_LEN + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        anc_seed, mut_seed, rate = c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], C4_LEN, anc_seed, mut_seed, rate)
        buf[seg[g] + C4_LEN] = ord("\n")
    torch.cuda.synchronize()
    masks = [sksffi.mask_generate(W, K, s) for s in range(C5_SEEDS)]
    ones = [bin(m).count("1") // 2 for m in masks]
    starts = torch.arange(n, dtype=torch.int64, device="cuda") * C4_S
    n_tiles = sksffi.intersect_sym_tiles(n)
    dev = "cuda" if collective() and os.environ.get("SKS_BENCH_DEVICE") is None else "cpu"

    # seeds are independent: `lanes` seeds run at once, each lane a context on its
    # own HIP stream with its own buffers, driven by its own host thread, so one
    # seed's post-processing, pair counts and host ANI overlap another's scan
    import queue
    from concurrent.futures import ThreadPoolExecutor
    lanes = queue.Queue()
    for _ in range(max(1, lanes_n)):
        st = torch.cuda.Stream()
        lanes.put({"ctx": sksffi.Context(torch.cuda.current_device(), st.cuda_stream),
                   "stream": st.cuda_stream,
                   "padded": torch.full((n, C4_S), -1, dtype=torch.int64, device="cuda"),
                   "sizes": torch.zeros(n, dtype=torch.int32, device="cuda"),
                   "mat": torch.empty((n, n), dtype=torch.int32, device="cuda")})
    pool = ThreadPoolExecutor(max_workers=max(1, lanes_n))

    def seed_job(s):
        lane = lanes.get()
        try:
            c = lane["ctx"]
            ss = c.sketch_build(buf.data_ptr(), seg[-1], seg, W, masks[s], sksffi.SKS_BOTTOM_S, C4_S)
            ss.export(lane["padded"].data_ptr(), C4_S, lane["sizes"].data_ptr())
            c.intersect_sym(lane["padded"].data_ptr(), starts.data_ptr(), lane["sizes"].data_ptr(),
                            1, n, 0, n_tiles, lane["mat"].data_ptr())
            c.synchronize()
            counts = lane["mat"].cpu().numpy()
            ss.free(stream=lane["stream"])  # no device-wide wait (the other lane runs)
        finally:
            lanes.put(lane)
        size_first = np.repeat(np.diag(counts).astype(np.int32), n)
        _, ani = sksffi.ani_from_counts(counts.reshape(-1), size_first, ones[s])
        return torch.from_numpy(ani.reshape(n, n))

    def ani_for_seed(s):
        return pool.submit(seed_job, s)

    total = 0.0
    timed = 0
    for it in range(warmup + steps):
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cons, mine = sks_dist.seed_sweep(C5_SEEDS, world, rank, ani_for_seed, n, device=dev)
        cons = cons.cpu()
        dt = max_over_ranks(time.perf_counter() - t0, world)
        if it >= warmup:
            total += dt
            timed += 1
    pool.shutdown()
    t = total / max(timed, 1)
    c = cons.numpy()
    cpu_b = cpu_baseline_c5(ctx, buf, seg, masks, ones) if cpu else None
    return {
        "metric": "seed-sweep genome-pairs ANI/s", "value": C5_SEEDS * n * n / t,
        "unit": "ordered (pair, seed) ANIs/s", "scaling": "strong", "ms_per_sweep": t * 1e3,
        "sketch_kmers_per_s": C5_SEEDS * n * (C4_LEN - W + 1) / t,
        "consensus_ani_mean": float(c.mean()),
        "consensus_ani_offdiag_min": float((c + np.eye(n) * 2).min()),
        "config": {"workload": "config5 seed sweep", "genomes": n, "genome_len": C4_LEN,
                   "seeds": C5_SEEDS, "s": C4_S, "w": W, "k": K,
                   "sharding": "seeds over ranks", "consensus": "mean ANI over seeds",
                   "seeds_in_flight": max(1, lanes_n),
                   "collective": (f"all_reduce of ANI sums ({backend_label()})"
                                  if collective() else "none")},
        "cpu_baseline": cpu_b,
    }


# LDS: the fastest random-address rate of profiles/r01/lds_atomics_microbench.txt
# (ds_add_u32 random, 9.73 lane-ops/clk/CU at 2.4 GHz = 0.152 wave-instructions
# per clock per CU); ds_cmpst_rtn_b32 (the join's insert) runs 5.66, ds_read_b64
# 9.39.  k_join's mix is reads, compare-swaps and XOR atomics, so this peak is
# an upper bound of what its LDS instructions could reach.
LDS_PEAK_WAVE_INST_PER_CLK_CU = 9.73 / 64
CUS, PEAK_CLK_GHZ, SIMDS = 256, 2.4, 1024


def latest_profile_json(name):
    """profiles/rNN/<name> of the newest round that has one."""
    import glob
    import re
    found = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*", name)):
        m = re.search(r"[/\\]r(\d+)[/\\]" + re.escape(name) + "$", f)
        if m:
            found.append((int(m.group(1)), f))
    return max(found)[1] if found else ""


def scan_valu_roofline(kernel_ms):
    """The scan's VALU issue bound (the bound it is on): counted
    VALU wave-instructions per launch (PMC, profiles/rNN/scan_valu.json) over
    the live kernel time, against 1024 SIMDs issuing the hot block's mix at the
    measured per-instruction rates (tools/valu_mix.py).  Null when the profile
    was measured on other scan sources."""
    import srchash
    path = latest_profile_json("scan_valu.json")
    if not path:
        return {"note": "no profiles/rNN/scan_valu.json"}
    t = json.load(open(path))
    src = os.path.relpath(path, ROOT)
    if t.get("scan_source_hash") != srchash.scan_hash() or not t.get("sq_insts_valu_per_launch"):
        return {"note": f"stale: {src} measured on scan sources {t.get('scan_source_hash')}, "
                        f"these are {srchash.scan_hash()}", "source": src}
    insts = t["sq_insts_valu_per_launch"]
    achieved = insts / (kernel_ms * 1e-3)
    peak = SIMDS / (t["mean_ns_per_valu_per_simd"] * 1e-9)
    hw = t.get("valu_inst_per_simd_cycle")
    return {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "VALU wave-instructions/s",
            "frac": achieved / peak, "valu_per_window": t["valu_per_window"],
            # the hardware's count: VALU instructions issued per SIMD per cycle of the
            # profiled launch (SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM cycles)); a
            # wave64 VALU op holds its SIMD 2 (add/xor) to 4+ (64-bit mul/shift) cycles
            "hw_valu_inst_per_simd_cycle": hw,
            "hw_valu_busy_at_mix": hw * t["mean_cycles_per_valu"] if hw else None,
            "hot_block_valu": t["hot_block_valu"], "mean_cycles_per_valu": t["mean_cycles_per_valu"],
            "source": src,
            "note": "SQ_INSTS_VALU per launch (PMC) / live kernel time, against 1024 SIMDs at the hot "
                    "block's cycle-weighted mix (profiles/r01/isa_rates_microbench.txt)"}


def pairs_lds_roofline(kernel_ms, name="pair_lds.json"):
    """k_join's LDS roofline from the hardware's own busy counter: LDS-array
    cycles per all-pairs call (SQ_LDS_IDX_ACTIVE, PMC, profiles/rNN/<name>;
    summed over the CUs, bank-conflict cycles included) over the live kernel
    time, against every CU's LDS busy every cycle (256 CUs x the clock measured
    in the same profile, GRBM_GUI_ACTIVE / 8 XCDs / profiled time).  Beside it:
    LDS wave-instructions per call and the conflict share.  Null when the
    profile was measured on other join sources."""
    import srchash
    path = latest_profile_json(name)
    if not path or not kernel_ms:
        return {"note": f"no profiles/rNN/{name}"}
    t = json.load(open(path))
    src = os.path.relpath(path, ROOT)
    if t.get("join_source_hash") != srchash.join_hash() or not t.get("sq_lds_idx_active_per_call"):
        return {"note": f"stale: {src} measured on join sources {t.get('join_source_hash')}, "
                        f"these are {srchash.join_hash()}", "source": src}
    act = t["sq_lds_idx_active_per_call"]
    clk = t["grbm_gui_active_per_call"] / 8 / (t["profiled_ms"] * 1e-3)  # Hz under the profiled load
    achieved = act / (kernel_ms * 1e-3)
    peak = CUS * clk
    conf = t.get("sq_lds_bank_conflict_per_call")
    return {"bound": "lds", "achieved": achieved, "peak": peak, "unit": "LDS-array cycles/s",
            "frac": achieved / peak, "lds_insts_per_call": t.get("sq_insts_lds_per_call"),
            "bank_conflict_frac_of_lds_active": (conf / act) if conf and act else None,
            "wave_cycles_waiting_frac": (t["sq_wait_any_per_call"] / t["sq_wave_cycles_per_call"])
            if t.get("sq_wait_any_per_call") and t.get("sq_wave_cycles_per_call") else None,
            "clock_ghz": clk / 1e9, "kernel": t.get("kernel"), "source": src,
            "peak_note": "every CU's LDS array busy every cycle (SQ_LDS_IDX_ACTIVE counts LDS-array "
                         "cycles per CU, MI355X_MICROARCH.md LDS section); clock from GRBM_GUI_ACTIVE"}


def latest_traffic_json():
    """profiles/rNN/traffic.json of the newest round that has one: written by
    tools/profile_round.sh from rocprofv3 PMC passes over this same bench command
    (FETCH_SIZE and WRITE_SIZE cannot share a pass), per timed launch."""
    import glob
    import re
    found = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")):
        m = re.search(r"[/\\]r(\d+)[/\\]traffic\.json$", f)
        if m:
            found.append((int(m.group(1)), f))
    return max(found)[1] if found else ""


def traffic_for_current_scan(path):
    """(bytes per launch, source file, note): the PMC traffic of a profile only
    while it was measured on the scan kernel's current sources; else None with
    the reason."""
    import srchash
    if not path or not os.path.exists(path):
        return None, None, "no profiles/rNN/traffic.json"
    src = os.path.relpath(path, ROOT)
    with open(path) as f:
        t = json.load(f)
    want, got = srchash.scan_hash(), t.get("scan_source_hash")
    if got != want:
        return None, src, (f"stale: measured on scan sources {got}, these are {want} "
                           "(re-run tools/profile_round.sh)")
    return t.get("scan_hbm_bytes_per_launch"), src, f"PMC on scan sources {want}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-sample-mb", type=int, default=125)  # ~10 s of 1-core work
    ap.add_argument("--cpu-crosscheck-mb", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pairs", action="store_true")
    ap.add_argument("--no-pairs-wide", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-c3-sharded", action="store_true")
    ap.add_argument("--no-c2", action="store_true")
    ap.add_argument("--no-ref-sweep", action="store_true",
                    help="skip the reference main's 62-config sweep (bin/kmer-sketching on 64 files)")
    ap.add_argument("--sweep-inflight", type=int, default=2,
                    help="config-5 seeds in flight (one context + HIP stream each)")
    ap.add_argument("--inflight", type=int, default=3,
                    help="config-3 builds in flight (one context + HIP stream each)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--exchange", default="p2p", choices=["p2p", "allgather", "broadcast"],
                    help="config-4 sketch exchange between ranks (sks_dist.all_vs_all_join)")
    ap.add_argument("--world1-exchange", action="store_true",
                    help="with --dist-rehearsal: config 4 at world 1 takes the multi-rank exchange path "
                         "(own layout + tile list + the exchange calls, which move nothing) instead of "
                         "the one-call native path, to measure that path's fixed cost")
    ap.add_argument("--dist-rehearsal", action="store_true",
                    help="start the process group at world 1 too (under torchrun), so the "
                         "collective paths run on the backend")
    ap.add_argument("--traffic-json", default=latest_traffic_json(),
                    help="PMC HBM traffic of the scan launches this command times "
                         "(tools/profile_round.sh; default: the newest profiles/rNN)")
    args = ap.parse_args()
    global EXCHANGE, WORLD1_EXCHANGE
    EXCHANGE = args.exchange
    WORLD1_EXCHANGE = args.world1_exchange

    world, rank, local = dist_setup(args.gpus, args.dist_backend, args.dist_rehearsal)
    ctx = sksffi.Context(local)
    mask = sksffi.mask_generate(W, K, MASK_SEED)

    buf, n_bytes = make_c3(ctx, seed_base=3 + 1000 * rank)
    log(f"[rank {rank}] config 3 genome resident: {n_bytes / 1e9:.2f} GB")

    def step():
        return ctx.sketch_build(buf.data_ptr(), n_bytes, [0, n_bytes], W, mask,
                                sksffi.SKS_FRAC_MOD, C3_FRAC)

    for _ in range(args.warmup):
        ss = step()
        del ss
    # serial pass: one build at a time on the null stream; gives the scan
    # kernel's own duration for the roofline and the unpipelined step time
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    scan_ms, survivors, windows, sizes = [], [], 0, []
    for _ in range(args.steps):
        ss = step()
        t = ctx.timings()
        scan_ms.append(t["scan_ms"])
        survivors.append(t["survivors"])
        windows += int(ss.windows()[0])
        sizes.append(int(ss.sizes()[0]))
        del ss
    torch.cuda.synchronize()
    barrier(world)
    elapsed_serial = max_over_ranks(time.perf_counter() - t0, world)
    sum_windows_serial = sum_over_ranks(windows, world)
    assert windows == args.steps * c3_windows(), (windows, c3_windows())

    # headline pass: `inflight` builds at once (host threads, one context per
    # HIP stream), so one build's sort / unique / host syncs run under the next
    # build's scan. Each build is complete when sks_sketch_build returns; its
    # set is then freed in stream order (sks_sketch_set_free_on_stream).
    value, elapsed, inflight_sizes = run_c3_inflight(local, buf, n_bytes, mask, args.steps,
                                                     args.inflight, world)
    assert inflight_sizes == {sizes[0]}, (inflight_sizes, sizes[0])

    # roofline of the dominant kernel (fused scan): algorithmic bytes per launch
    # = input bytes read (1 B per sequence byte incl. separators) + 8 B per record written
    scan_avg_ms = float(np.mean(scan_ms))
    alg_bytes = n_bytes + 8 * float(np.mean(survivors))
    achieved = alg_bytes / (scan_avg_ms * 1e-3) / 1e9
    traffic, traffic_src, traffic_note = traffic_for_current_scan(args.traffic_json)

    c2 = None
    if not args.no_c2:
        c2 = run_c2(ctx, mask, steps=max(4, args.steps), warmup=2, inflight=args.inflight,
                    cpu=rank == 0 and world == 1 and not args.no_cpu_baseline)

    pairs = None
    if not args.no_pairs:
        pairs = run_pairs(ctx, world, rank, mask, steps=max(1, min(args.steps, 10)),
                          warmup=1, cpu_pairs=not args.no_cpu_baseline)

    pairs_wide = None
    if not args.no_pairs and not args.no_pairs_wide:
        pairs_wide = run_pairs(ctx, world, rank, sksffi.mask_generate(C4W_W, C4W_K, MASK_SEED),
                               steps=max(1, min(args.steps, 10)), warmup=1, w=C4W_W,
                               cpu_pairs=not args.no_cpu_baseline)

    c3s = None
    if not args.no_c3_sharded:
        c3s = run_c3_sharded(ctx, world, rank, mask, buf, steps=3, warmup=1)

    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = run_end_to_end(ctx, mask, buf, steps=2)

    sweep = None
    if not args.no_sweep:
        sweep = run_seed_sweep(ctx, world, rank, steps=max(1, min(args.steps, 2)), warmup=1,
                               lanes_n=args.sweep_inflight,
                               cpu=rank == 0 and world == 1 and not args.no_cpu_baseline)

    ref_sweep = None
    if rank == 0 and world == 1 and not args.no_ref_sweep:
        ref_sweep = run_ref_sweep(ctx, cpu=not args.no_cpu_baseline)

    cpu = cpu_x = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_c3(mask, args.cpu_sample_mb * 1_000_000)
        cpu_x = cpu_crosscheck_c3(ctx, buf, mask, args.cpu_crosscheck_mb * 1_000_000)

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "k-mers/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "ms_per_step_serial": elapsed_serial / args.steps * 1e3,
            "value_serial": sum_windows_serial / elapsed_serial,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (device splitmix64 generator, resident in HBM)",
            "config": {"workload": "config3: 1x3 Gb multi-contig genome per GPU, spaced seed "
                                   "w=31/k=21 (mask seed 0), FracMinHash 1/1000",
                       "builds_in_flight": args.inflight,
                       "genome_bytes": n_bytes, "windows_per_genome": c3_windows(),
                       "sketch_size": sizes[0], "parallelism": f"genome-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "scan_kernel<frac, boost-mix, pre-filter>", "kernel_ms": scan_avg_ms,
                         "kernel_ms_median": float(np.median(scan_ms)),
                         "algorithmic_bytes_per_launch": alg_bytes,
                         "traffic_source": traffic_src, "traffic_note": traffic_note,
                         "valu": scan_valu_roofline(scan_avg_ms),
                         "timing": "hipEvents around each scan launch of the serial pass "
                                   "(the --steps builds after --warmup)"},
            "cpu_baseline": cpu,
            "cpu_crosscheck": cpu_x,
            "config2": c2,
            "pairs": pairs,
            "pairs_wide": pairs_wide,
            "seed_sweep": sweep,
            "reference_sweep": ref_sweep,
            "end_to_end": e2e,
            "c3_one_genome_sharded": c3s,
        }
        print(json.dumps(line), flush=True)
    if collective():
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
