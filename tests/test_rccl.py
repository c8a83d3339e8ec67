"""The multi-GPU orchestration on RCCL, on one GPU.

The driver runs N > 1 (one process per GPU); a 1-GPU box cannot.  Here a
process group of size 1 on the "nccl" backend (RCCL) is started, so
sks_dist takes its collective path (`_solo` is False) and every exchange the
N > 1 runs make — all_gather_into_tensor of int64 / uint8 / int32 join layouts,
of padded sketches and chunk sketches, all_reduce of the count matrix, of the
ANI sums and of scalars — runs through RCCL on device memory.  Each result is
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


@pytest.mark.parametrize("side_stream", [False, True])
def test_join_layout_all_vs_all_on_rccl(env, side_stream):
    """sks_dist.all_vs_all_join through the collective branch on RCCL: the
    all_reduce MAX of (largest sketch, element total), the padded layout gathers
    (int64 data, uint8 ids, int32 bucket starts, int64 block starts), queued on
    the collective stream while the rank's own tiles are counted, the packed
    tile gather to rank 0 (dist.gather) and the matrix assembly — 130 genomes
    (3 blocks, a ragged last one, an empty sketch).  With side_stream the
    context's kernels run on a non-default HIP stream: join_layout_fns orders it
    against torch's stream both ways."""
    torch, dist, ctx = env
    import sks_dist
    n, s = 130, 600
    genomes = _family(n, 30_000, 9)
    genomes[40] = b""
    d, seg = _upload(torch, genomes)
    mask = sksffi.mask_generate(W, K, 0)
    ss = ctx.sketch_build(d.data_ptr(), seg[-1], seg, W, mask, sksffi.SKS_BOTTOM_S, s)
    sizes = ss.sizes().copy()
    sk = [ss.sketch(i)[:, 0].copy() for i in range(n)]
    for g in (0, 64, 129):
        want, _ = O.sketch(O.cut_runs(genomes[g]), W, mask, "bottom", s)
        assert np.array_equal(ss.sketch(g), want)
    want = _merge_counts(sk)
    assert want[0, 9] > 0 and want[40].sum() == 0
    stream = torch.cuda.Stream() if side_stream else None
    cctx = sksffi.Context(0, stream.cuda_stream) if side_stream else ctx
    build, count, bounds = sks_dist.join_layout_fns(cctx, ss, sizes, device="cuda")
    out = torch.full((n, n), -5, dtype=torch.int32, device="cuda")
    mat = sks_dist.all_vs_all_join(n, 1, 0, int(sizes.max()), int(sizes.astype(np.int64).sum()),
                                   sksffi.join_layout_log_b, build, count, device="cuda", out=out,
                                   bounds=bounds)
    torch.cuda.synchronize()
    assert np.array_equal(mat.cpu().numpy().astype(np.int64), want), side_stream
    if side_stream:
        cctx.close()


def test_padded_sketch_all_vs_all_and_rows_on_rccl(env):
    """sks_dist.all_vs_all (padded int64 sketches + int32 sizes gathered, symmetric
    tiles, count all_reduce) and all_vs_all_rows at w = 45 ((lo, hi) pairs, row
    blocks gathered as flat int32), both equal to the oracle's merge counts."""
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

    w, k, c = 45, 30, 15
    m = O.mask(w, k, 2)
    ssw = ctx.sketch_build(d.data_ptr(), seg[-1], seg, w, m, sksffi.SKS_FRAC_MOD, c)
    skw = [O.sketch(O.cut_runs(g), w, m, "frac", c)[0] for g in genomes]
    stride = max(len(x) for x in skw) + 1
    pw = torch.full((n, 2 * stride), -1, dtype=torch.int64, device="cuda")
    pwsz = torch.zeros(n, dtype=torch.int32, device="cuda")
    ssw.export(pw.data_ptr(), stride, pwsz.data_ptr())
    st2 = torch.arange(n, dtype=torch.int64, device="cuda") * stride

    def count_rows(src, sizes, nn, r0, r1, out):
        ctx.intersect_all(src.data_ptr(), st2.data_ptr(), sizes.data_ptr(), 2, nn, r0, r1,
                          out.data_ptr())
        torch.cuda.synchronize()

    got = sks_dist.all_vs_all_rows(pw, pwsz, n, 1, 0, count_rows).cpu().numpy()
    want = np.array([[O.intersect(skw[i], skw[j]) for j in range(n)] for i in range(n)])
    assert want[0, 5] > 0
    assert np.array_equal(got, want)


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
