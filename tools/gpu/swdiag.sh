set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/swdiag; mkdir -p $O; cd $R
timeout -k 10 300 python3 tools/sweep_files.py /tmp/sf 64 > $O/files.log 2>&1 || exit 1
LD_LIBRARY_PATH=$R/variants/lstamps_lib timeout -k 10 300 $R/spaced-kmer-sketching_amd/bin/kmer-sketching /tmp/o.csv $(cat /tmp/sf/list.txt) > $O/stamps_run.log 2> $O/stamps.err || { tail $O/stamps.err; exit 1; }
echo stamps done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/t -o run -- $R/spaced-kmer-sketching_amd/bin/kmer-sketching /tmp/o2.csv $(cat /tmp/sf/list.txt) > $O/trace_run.log 2>&1 || { tail $O/trace_run.log; exit 1; }
f=$(find $O/t -name '*kernel_trace.csv' | head -1); gzip -c $f > $O/kernel_trace.csv.gz; rm -rf $O/t
echo trace done
