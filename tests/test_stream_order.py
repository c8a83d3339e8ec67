"""Stream-ordered reuse of device memory ("stream-ordered release").

A sketch set freed with sks_sketch_set_free_on_stream, and a context scratch
buffer that grows, go back to the process's block cache ordered after their
stream's queued work.  The cache must not hand such a block to another build
until that work has completed: round 2's hipMallocAsync experiment read back
all-zero sketches when memory changed hands between streams without an
ordering.  Here stream A is held busy by a bounded sleep kernel (about 0.1 s)
while the block is released on it, so the release is certainly pending when
the other context allocates; the other context must get a different block, and
every sketch must equal the oracle's."""
import numpy as np
import pytest

import pyoracle as O
import sksffi
import synth

pytestmark = pytest.mark.gpu

W, MASK_SEED = 31, 0


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _upload(torch, genomes):
    stream = b"".join(g + b"\n" for g in genomes)
    offs = np.cumsum([0] + [len(g) + 1 for g in genomes]).tolist()
    d = torch.frombuffer(bytearray(stream), dtype=torch.uint8).to("cuda:0")
    torch.cuda.synchronize()
    return d, len(stream), offs


def _check(ss, genomes, m, param):
    for i, g in enumerate(genomes):
        want, nw = O.sketch(O.cut_runs(g), W, m, "frac", param)
        assert np.array_equal(ss.sketch(i), want), i
        assert int(ss.windows()[i]) == nw


def test_pending_stream_release_is_not_reused(torch_cuda):
    torch = torch_cuda
    m = O.mask(W, 21, MASK_SEED)
    genomes = [synth.bases(400_000, seed=3, mut_seed=80 + i, mut_rate=0.01 * i).tobytes()
               for i in range(4)]
    d, n, offs = _upload(torch, genomes)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ca, cb = sksffi.Context(0, sa.cuda_stream), sksffi.Context(0, sb.cuda_stream)
    try:
        s1 = ca.sketch_build(d.data_ptr(), n, offs, W, m, sksffi.SKS_FRAC_MOD, 20)
        _check(s1, genomes, m, 20)
        p1 = s1.device_ptrs()[0]
        with torch.cuda.stream(sa):
            torch.cuda._sleep(200_000_000)  # ~0.1 s of stream A, bounded
        s1.free(stream=sa.cuda_stream)  # released after the sleep: still pending
        # the same-size allocation on stream B must not get the pending block
        s2 = cb.sketch_build(d.data_ptr(), n, offs, W, m, sksffi.SKS_FRAC_MOD, 20)
        assert s2.device_ptrs()[0] != p1
        # context A's scratch grows while its stream is still busy: the old
        # blocks go back ordered after the sleep, nothing waits for the device
        big = [synth.bases(3_000_000, seed=5, mut_seed=90 + i, mut_rate=0.0).tobytes()
               for i in range(2)]
        db, nb, ob = _upload(torch, big)
        with torch.cuda.stream(sa):
            torch.cuda._sleep(200_000_000)
        s3 = ca.sketch_build(db.data_ptr(), nb, ob, W, m, sksffi.SKS_FRAC_MOD, 200)
        s4 = cb.sketch_build(d.data_ptr(), n, offs, W, m, sksffi.SKS_FRAC_MOD, 20)
        torch.cuda.synchronize()
        _check(s2, genomes, m, 20)
        _check(s4, genomes, m, 20)
        _check(s3, big, m, 200)
    finally:
        ca.close()
        cb.close()
