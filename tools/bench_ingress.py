"""Device FASTA ingress throughput (sks_fasta_parse_device) on a synthetic
multi-record FASTA file held in HBM: 80-column lines, a header every
`rec_mb` MB, a few N runs.  Prints raw GB/s of input parsed and the phases'
device time (hipEvents around the call)."""
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
import sksffi  # noqa: E402


def synth_fasta(n_bases, rec_mb=125, width=80, seed=1):
    rng = np.random.default_rng(seed)
    seq = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n_bases, dtype=np.uint8)]
    parts = []
    rec = int(rec_mb * 1_000_000)
    for r0 in range(0, n_bases, rec):
        body = seq[r0:r0 + rec]
        n_lines = (len(body) + width - 1) // width
        pad = n_lines * width - len(body)
        lines = np.concatenate([body, np.full(pad, 10, np.uint8)]).reshape(n_lines, width)
        lines = np.concatenate([lines, np.full((n_lines, 1), 10, np.uint8)], 1).ravel()
        if pad:
            lines = lines[:-pad]  # last line shorter, keep its newline
            lines[-1] = 10
        parts.append(np.frombuffer(f">contig_{r0 // rec} synthetic\n".encode(), np.uint8))
        parts.append(lines)
    return np.concatenate(parts)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    t0 = time.time()
    raw = synth_fasta(n)
    print(f"host synth {len(raw) / 1e9:.2f} GB in {time.time() - t0:.1f}s", flush=True)
    ctx = sksffi.Context(0)
    d = torch.from_numpy(raw).to("cuda:0")
    nb, nr = ctx.fasta_parse_device(d.data_ptr(), len(raw))
    out = torch.empty(nb, dtype=torch.uint8, device="cuda:0")
    ms = []
    for _ in range(reps):
        ctx.fasta_parse_device(d.data_ptr(), len(raw), out.data_ptr(), nb)
        ms.append(ctx.last_ingress_ms())
    med = statistics.median(ms)
    ok = nb == n + nr  # every base kept plus one separator per record
    print(f"ingress: {len(raw)} raw bytes -> {nb} stream bytes, {nr} records; "
          f"median {med:.2f} ms, min {min(ms):.2f} ms = {len(raw) / med / 1e6:.1f} GB/s raw; "
          f"size check {'ok' if ok else 'BAD'}", flush=True)


if __name__ == "__main__":
    main()
