set -e
cd /root/repo
for lib in spaced-kmer-sketching_amd/lib/libsks.so variants/libsks_mw8.so; do
  SKS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_scan.py 5000000000 5 1000
  SKS_LIB=$PWD/$lib timeout -k 10 120 python3 tools/bench_scan.py 3000000000 5 1
done
