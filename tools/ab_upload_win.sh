# Window width of the full-width windowed upload (configs[1]): alternating
# host-timed runs of tools/msm_only.py with the default build (c = 20) and
# variant builds var_wc<c> (tools/build_variant.sh wc<c> - -DZK_UPLOAD_WIN_C=<c>).
#   bash tools/ab_upload_win.sh OUT 17 18 19 21
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
out=$1; shift
: > $out
for rep in 1 2 3; do
  for v in base "$@"; do
    lib=""; [ $v != base ] && lib=$R/zero-knowledge-proofs_amd/var_wc$v/libzkp_amd.so
    echo "c=$v $(ZK_AMD_LIB=$lib timeout -k 10 120 python -u tools/msm_only.py 20 20 2>/dev/null)" >> $out
  done
done
cat $out
