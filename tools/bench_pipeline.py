"""Config-3 builds with D builds in flight: D host threads, each with its own
context on its own HIP stream, sharing the resident genome.  Measures whether
one build's post-processing (sort / unique / host syncs, ~0.45 ms) hides under
the next build's scan.  Sets are kept until the timed region ends (freeing one
synchronises the device, as hipFree does).

    python tools/bench_pipeline.py --depth 2 --steps 12
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "spaced-kmer-sketching_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import sksffi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    streams = [torch.cuda.Stream() for _ in range(a.depth)]
    ctxs = [sksffi.Context(0, s.cuda_stream) for s in streams]
    mask = sksffi.mask_generate(bench.W, bench.K, bench.MASK_SEED)
    buf, n_bytes = bench.make_c3(ctxs[0], seed_base=3)
    torch.cuda.synchronize()

    def build(ctx):
        return ctx.sketch_build(buf.data_ptr(), n_bytes, [0, n_bytes], bench.W, mask,
                                sksffi.SKS_FRAC_MOD, bench.C3_FRAC)

    ref = build(ctxs[0])
    ref_vals = ref.to_numpy()[0] if hasattr(ref, "to_numpy") else None
    for _ in range(a.warmup):
        for c in ctxs:
            del_ = build(c)
            del del_
    torch.cuda.synchronize()
    kept = [[] for _ in ctxs]

    def worker(i):
        for s in range(i, a.steps, a.depth):
            kept[i].append(build(ctxs[i]))

    t0 = time.perf_counter()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(a.depth)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    sizes = {int(s.sizes()[0]) for k in kept for s in k}
    ok = sizes == {int(ref.sizes()[0])}
    print(json.dumps({"depth": a.depth, "steps": a.steps, "ms_per_step": el / a.steps * 1e3,
                      "kmers_per_s": a.steps * bench.c3_windows() / el, "sizes_equal": ok,
                      "ref_checked": ref_vals is not None}), flush=True)


if __name__ == "__main__":
    main()
