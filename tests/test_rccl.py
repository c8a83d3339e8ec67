"""The multi-GPU orchestration on RCCL, on one GPU.

The driver runs N > 1 (one process per GPU); a 1-GPU box cannot.  Here a
process group of size 1 on the "nccl" backend (RCCL) is started, so
sks_dist takes its collective path (`_solo` is False) and every exchange the
N > 1 runs make — the per-source broadcasts of int64 sketches and int32 sizes,
the bounds broadcast, the metadata gather and the packed tile gather of
all_vs_all_join, all_gather_into_tensor of padded sketches and chunk sketches,
all_reduce of the count matrix, of the ANI sums and of scalars — runs through
RCCL on device memory.  Each result is
compared with the same computation without a process group, and with the
oracle (oracle/sks_oracle.cpp) where that is cheap.  Reference semantics:
kmer_set.cpp:23-41 (set intersection), kmer-sketching.cpp:185-200 (ANI).
"""
import socket

import numpy as np
import pytest

import pyoracle as O
import sksffi
import synth

pytestmark = pytest.mark.gpu

W, K = 31, 21


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def env():
    import torch
    import torch.distributed as dist
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    torch.cuda.set_device(0)
    ctx = sksffi.Context(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    yield torch, dist, ctx
    dist.destroy_process_group()
    ctx.close()


def _family(n, length, families):
    gen = [synth.bases(length, seed=500 + i % families, mut_seed=9000 + i,
                       mut_rate=0.002 * (i // families % 8)).tobytes() for i in range(n)]
    return gen


def _upload(torch, genomes):
    stream = b"".join(g + b"\n" for g in genomes)
    seg = [0]
    for g in genomes:
        seg.append(seg[-1] + len(g) + 1)
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to("cuda:0")
    return d, seg


def _merge_counts(sk):
    n = len(sk)
    return np.array([[len(np.intersect1d(sk[i], sk[j], assume_unique=True)) for j in range(n)]
                     for i in range(n)], dtype=np.int64)


@pytest.mark.parametrize("side_stream,w,bound", [(False, W, True), (True, W, False), (False, 45, True)])
def test_join_layout_all_vs_all_on_rccl(env, side_stream, w, bound):
    """sks_dist.all_vs_all_join through the collective branch on RCCL: the size
    all-reduce (without a size bound), the packed tile gather to rank 0
    (dist.gather), the matrix assembly and the ANI the join writes into pinned
    host memory — 130 genomes (3 blocks, a ragged last one, an empty sketch),
    u64 and (w = 45) 128-bit k-mers.  With side_stream the context's kernels
    run on a non-default HIP stream: GpuJoinOps orders it against torch's
    stream both ways."""
    torch, dist, ctx = env
    import sks_dist
    n, s = 130, 600
    genomes = _family(n, 30_000, 9)
    genomes[40] = b""
    d, seg = _upload(torch, genomes)
    k = K if w == W else 30
    mask = sksffi.mask_generate(w, k, 0)
    ss = ctx.sketch_build(d.data_ptr(), seg[-1], seg, w, mask, sksffi.SKS_BOTTOM_S, s)
    sizes = ss.sizes().copy()
    sk = [ss.sketch(i) for i in range(n)]
    for g in (0, 64, 129):
        want, _ = O.sketch(O.cut_runs(genomes[g]), w, mask, "bottom", s)
        assert np.array_equal(ss.sketch(g), want)
    want = np.array([[O.intersect(sk[i], sk[j]) for j in range(n)] for i in range(n)], dtype=np.int64)
    assert want[0, 9] > 0 and want[40].sum() == 0
    stream = torch.cuda.Stream() if side_stream else None
    cctx = sksffi.Context(0, stream.cuda_stream) if side_stream else ctx
    ops = sks_dist.GpuJoinOps(cctx, ss.elem_words)
    hb = sksffi.HostBuffer(n * n * 8)
    res = sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), ops, sksffi.join_layout_log_b,
                                   device="cuda", dst=0, ani_ones=k, ani_out=hb,
                                   size_bound=s if bound else None, world1_exchange=True)
    torch.cuda.synchronize()
    res.check_layouts()
    assert np.array_equal(res.matrix.cpu().numpy().astype(np.int64), want), side_stream
    # every ordered pair's ANI against the host formula on the oracle counts
    size_first = np.repeat(sizes.astype(np.int32), n)
    _, want_ani = sksffi.ani_from_counts(want.reshape(-1).astype(np.int32), size_first, k)
    assert np.abs(hb.array - want_ani).max() <= 1e-9
    hb.free()
    if side_stream:
        cctx.close()


def test_padded_sketch_all_vs_all_on_rccl(env):
    """sks_dist.all_vs_all (padded int64 sketches + int32 sizes gathered, symmetric
    tiles, count all_reduce), equal to the oracle's merge counts."""
    torch, dist, ctx = env
    import sks_dist
    n, s = 70, 400
    genomes = _family(n, 12_000, 5)
    d, seg = _upload(torch, genomes)
    mask = sksffi.mask_generate(W, K, 3)
    ss = ctx.sketch_build(d.data_ptr(), seg[-1], seg, W, mask, sksffi.SKS_BOTTOM_S, s)
    padded = torch.full((n, s), -1, dtype=torch.int64, device="cuda")
    psz = torch.zeros(n, dtype=torch.int32, device="cuda")
    ss.export(padded.data_ptr(), s, psz.data_ptr())
    starts = torch.arange(n, dtype=torch.int64, device="cuda") * s

    def count_sym(src, src_sz, nn, t0, t1, out):
        ctx.intersect_sym(src.data_ptr(), starts.data_ptr(), src_sz.data_ptr(), 1, nn, t0, t1,
                          out.data_ptr())
        torch.cuda.synchronize()

    got = sks_dist.all_vs_all(padded, psz, n, 1, 0, count_sym).cpu().numpy()
    assert np.array_equal(got.astype(np.int64), _merge_counts([ss.sketch(i)[:, 0] for i in range(n)]))


@pytest.mark.parametrize("w,k", [(W, K), (45, 30)])
def test_one_genome_sharded_on_rccl(env, w, k):
    """sks_dist.sketch_genome_sharded's exchange (scalar all_reduce MAX, padded
    chunk-sketch gather, size gather, window-count all_reduce) over RCCL, with the
    GPU union (sks_sketch_union / _wide): equal to the oracle's whole-genome
    sketch, and the windows add up."""
    torch, dist, ctx = env
    import sks_dist
    g = synth.bases(1_500_000, seed=17)
    g[700_000:700_050] = ord("N")
    g = g.tobytes()
    d, _ = _upload(torch, [g])
    m = O.mask(w, k, 0)
    ew = 2 if w > 32 else 1

    def build_chunk(a, b):
        ss = ctx.sketch_build(d.data_ptr() + a, b - a, [0, b - a], w, m, sksffi.SKS_FRAC_MOD, 100)
        kk = int(ss.sizes()[0])
        out = torch.empty(max(kk, 1) * ew, dtype=torch.int64, device="cuda")
        ss.export(out.data_ptr(), max(kk, 1),
                  torch.zeros(1, dtype=torch.int32, device="cuda").data_ptr())
        nw = int(ss.windows()[0])
        v = out[: kk * ew]
        return (v.view(kk, 2) if ew == 2 else v), nw

    def union(t):
        t = t.to("cuda").contiguous()
        out = torch.empty_like(t)
        kk = ctx.sketch_union(t.data_ptr(), t.shape[0], out.data_ptr(), elem_words=ew)
        return out[:kk]

    sk, nw = sks_dist.sketch_genome_sharded(len(g), w, 1, 0, build_chunk, union, "cuda")
    want, wnw = O.sketch(O.cut_runs(g), w, m, "frac", 100)
    got = sk.cpu().numpy().view(np.uint64)
    assert nw == wnw
    assert np.array_equal(got.reshape(-1, 2) if ew == 2 else got, want if ew == 2 else want[:, 0])


def test_seed_sweep_on_rccl(env):
    """sks_dist.seed_sweep with the ANI sums all-reduced on the device (float64
    over RCCL), equal to the mean of per-seed host ANI."""
    torch, dist, ctx = env
    import sks_dist
    n, s, seeds = 40, 300, 3
    genomes = _family(n, 10_000, 4)
    d, seg = _upload(torch, genomes)
    per_seed = []

    def ani_for_seed(k):
        m = sksffi.mask_generate(W, K, k)
        ss = ctx.sketch_build(d.data_ptr(), seg[-1], seg, W, m, sksffi.SKS_BOTTOM_S, s)
        counts = _merge_counts([ss.sketch(i)[:, 0] for i in range(n)])
        size_first = np.repeat(np.diag(counts).astype(np.int32), n)
        _, ani = sksffi.ani_from_counts(counts.reshape(-1).astype(np.int32), size_first,
                                        bin(m).count("1") // 2)
        per_seed.append(ani.reshape(n, n))
        return torch.from_numpy(ani.reshape(n, n))

    cons, mine = sks_dist.seed_sweep(seeds, 1, 0, ani_for_seed, n, device="cuda")
    assert mine == list(range(seeds)) and cons.is_cuda
    want = sum(per_seed) / seeds
    assert np.allclose(cons.cpu().numpy(), want, rtol=0, atol=1e-15)
