# Per-kernel A/B under rocprofv3 --stats: the same workload with the default
# library and each variant (zero-knowledge-proofs_amd/var_<name>/libzkp_amd.so).
#   bash tools/ab_kernels.sh "WORKLOAD ARGS" VARIANT...
#   e.g. bash tools/ab_kernels.sh "tools/msm_only.py 20 20" prev
set -e
R=$GRAFT_REPO_ROOT
work=$1; shift
cd /tmp && export TMPDIR=/tmp
for v in base "$@"; do
  lib=""; [ $v != base ] && lib=$R/zero-knowledge-proofs_amd/var_$v/libzkp_amd.so
  rm -rf $R/gpurun_out/abk_$v
  ZK_AMD_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abk_$v -o run -- python3 $R/$work > $R/gpurun_out/abk_$v.log 2>&1
  (cd $R && python3 tools/prof_summary.py stats gpurun_out/abk_$v/run_kernel_stats.csv gpurun_out/abk_$v.md > /dev/null)
done
cd $R
python3 - "$@" <<'PY'
import sys
rows = {}
for v in ["base"] + sys.argv[1:]:
    for ln in open(f"gpurun_out/abk_{v}.md").read().splitlines()[2:]:
        c = [x.strip() for x in ln.strip("|").split("|")]
        rows.setdefault(c[0], {})[v] = (int(c[1]), float(c[3]))
vs = ["base"] + sys.argv[1:]
print("kernel".ljust(44) + "".join(f"{v:>22s}" for v in vs))
for k, d in sorted(rows.items(), key=lambda kv: -max(n * a for n, a in kv[1].values())):
    print(k[:44].ljust(44) + "".join((f"{d[v][0]:>6d} x {d[v][1]:>9.1f} us" if v in d else " " * 22) for v in vs))
PY
