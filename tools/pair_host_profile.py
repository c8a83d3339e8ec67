"""Host-side cost of the bench's config-4 pair step (N = 1): cProfile over
`reps` calls of the step as bench.py issues it (sketches_of + all_vs_all_join,
counts only and with the fused ANI into pinned host memory), each followed by
a device sync, and the wall time per call.
    python tools/pair_host_profile.py [reps]"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
sys.path.insert(0, ROOT)
import sksffi  # noqa: E402
import sks_dist  # noqa: E402
import bench  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    n, L = bench.C4_GENOMES, bench.C4_LEN
    ctx = sksffi.Context(0)
    seg = [0]
    for _ in range(n):
        seg.append(seg[-1] + L + 1)
    buf = torch.empty(seg[-1], dtype=torch.uint8, device="cuda")
    for g in range(n):
        a, m, r = bench.c4_genome_seeds(g)
        ctx.synth_bases(buf.data_ptr() + seg[g], L, a, m, r)
        buf[seg[g] + L] = ord("\n")
    mask = sksffi.mask_generate(31, 21, 0)
    ones = bin(mask).count("1") // 2
    ss = ctx.sketch_build(buf.data_ptr(), seg[-1], seg, 31, mask, sksffi.SKS_BOTTOM_S, bench.C4_S)
    ops = sks_dist.GpuJoinOps(ctx)
    hb = sksffi.HostBuffer(n * n * 8)

    def step(ani):
        return sks_dist.all_vs_all_join(n, 1, 0, sks_dist.sketches_of(ss), ops, sksffi.join_layout_log_b,
                                        device="cuda", dst=None, ani_ones=ones if ani else None,
                                        ani_out=hb if ani else None, max_size=int(ss.sizes().max()),
                                        size_bound=bench.C4_S)
    for ani in (False, True):
        for _ in range(3):
            step(ani)
        torch.cuda.synchronize()
        ms, host = [], []
        pr = cProfile.Profile()
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            pr.enable()
            step(ani)
            pr.disable()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
            host.append((t1 - t0) * 1e3)
        ms.sort()
        host.sort()
        print(f"ani={ani}: call median {ms[len(ms) // 2]:.3f} ms, host part (until the call returns) median "
              f"{host[len(host) // 2]:.3f} ms", flush=True)
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(14)
        print(s.getvalue()[-3500:], flush=True)


if __name__ == "__main__":
    main()
