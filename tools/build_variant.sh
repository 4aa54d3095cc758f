# Build a variant libzkp_amd.so for A/B runs (tools/ab_prove.sh):
#   bash tools/build_variant.sh NAME [GIT_REV|-] [EXTRA HIPFLAGS...]
# GIT_REV: build that commit's sources (a temporary git worktree); "-": this
# tree.  Output: zero-knowledge-proofs_amd/var_NAME/libzkp_amd.so (loaded via
# ZK_AMD_LIB by the A/B tools; never by the product).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=${2:--}; shift; shift || true
out=$R/zero-knowledge-proofs_amd/var_$name
mkdir -p $out; rm -rf /tmp/zk_build_$name   # flags are not tracked by make: always a clean build
if [ "$rev" = "-" ]; then
  src=$R
else
  src=/tmp/zk_wt_$name
  rm -rf $src; git -C $R worktree prune
  git -C $R worktree add --detach $src $rev > /dev/null
fi
make -C $src/zero-knowledge-proofs_amd/csrc -j8 BUILD=/tmp/zk_build_$name OUT=$out/libzkp_amd.so ZK_EXTRA="$*" > /tmp/zk_build_$name.log 2>&1
if [ "$rev" != "-" ]; then git -C $R worktree remove --force $src; fi
echo "built $out/libzkp_amd.so ($rev $*)"
