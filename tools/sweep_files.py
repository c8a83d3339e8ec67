"""Writes the first n config-4 genomes as FASTA files (80-column lines, the
bench's reference_sweep inputs) into a directory, plus list.txt naming them.
    python tools/sweep_files.py <dir> [n]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "spaced-kmer-sketching_amd"))
import bench  # noqa: E402
import sksffi  # noqa: E402


def main():
    d = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.REF_SWEEP_GENOMES
    os.makedirs(d, exist_ok=True)
    files = bench._fasta_files(sksffi.Context(0), n, d)
    with open(os.path.join(d, "list.txt"), "w") as f:
        f.write(" ".join(files) + "\n")
    print(f"{len(files)} files in {d}")


if __name__ == "__main__":
    main()
