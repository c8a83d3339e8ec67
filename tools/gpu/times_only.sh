# whole-call and kernel times per library variant, no tests: times_only.sh tag ...
R=${GRAFT_REPO_ROOT:-/root/repo}
rm -rf $R/gpurun_out/var
bash $R/tools/gpu/pairs_times.sh "$@"
