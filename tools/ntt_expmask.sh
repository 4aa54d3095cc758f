# 2^22 / 2^20 API NTT with the HBM indices confined to a cache-resident
# prefix (ZK_NTT_EXPMASK, wrong results): how much of a pass is HBM latency.
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
for i in 1 2 3; do
  for m in none 0xfff 0x3ffff; do
    for L in 22 20; do
      if [ $m = none ]; then r=$(timeout -k 10 60 python3 $R/tools/ntt_only.py $L 20 2>/dev/null | head -1)
      else r=$(ZK_NTT_EXPMASK=$m timeout -k 10 60 python3 $R/tools/ntt_only.py $L 20 2>/dev/null | head -1); fi
      echo "mask=$m $r"
    done
  done
done
