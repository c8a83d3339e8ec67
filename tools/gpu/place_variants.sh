# k_gl_place / k_join kernel time per library variant (kernel trace of tools/bench_pairs.py, 2 reps):
#   bash tools/gpu/place_variants.sh base diag2 ...
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/var
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for tag in "$@"; do
  if [ "$tag" = base ]; then L=$R/spaced-kmer-sketching_amd/lib/libsks.so; else L=$R/variants/libsks_$tag.so; fi
  for m in family indep; do
    SKS_LIB=$L SKS_BENCH_KERNELS=join timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_${tag}_$m -o run -- python3 $R/tools/bench_pairs.py 1000 2 $m > $O/$tag.$m.log 2>&1 || exit 1
    python3 - $O/t_${tag}_$m $tag $m >> $O/summary.txt <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    m = re.search(r"(k_\w+)", r["Name"])
    if m and m.group(1).startswith(("k_gl_place", "k_join", "k_gl_pos", "k_gl_prep")):
        print(sys.argv[2], sys.argv[3], m.group(1), round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
    rm -rf $O/t_${tag}_$m
  done
done
echo done
