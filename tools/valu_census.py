"""Static instruction census of the accumulate kernels' hot loops.

Compile msm.hip to gfx950 assembly (device only) and count, inside the
loop of each accumulate kernel that holds the most v_mad_u64_u32, every
instruction by class.  The per-add issue of `profiles/r03_accum_valu_issue.json`
(SQ_INSTS_VALU per mixed add, hardware counters) says how many VALU
instructions an add costs; this says which ones.
Usage: valu_census.py [msm.s] > profiles/r06_accum_census.json
(without an argument it runs hipcc -S itself into /tmp)."""
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"k_msm_accum<G1>": "_ZN2zk11k_msm_accumINS_2G1EEEvNS_8SegBasesINT_1AEEEjPKjS7_S7_jjPNS3_1XES9_",
           "k_msm_accum_pair (G2)": "_ZN2zk16k_msm_accum_pairENS_8SegBasesI6AffineI3Fq2EEEjPKjS6_S6_jjP4XYZZIS2_ES9_"}

CLASSES = [
    ("v_mad_u64_u32 (limb products)", r"^v_mad_u64_u32"),
    ("v_add/sub with carry (co/ci)", r"^v_(add|sub|subrev)_co|^v_(add|sub|subrev)c_co|^v_addc|^v_subb"),
    ("v_add/sub u32 (no carry)", r"^v_(add|sub|subrev)_(nc_)?u32|^v_add3_u32|^v_(add|sub)_i32"),
    ("v_cndmask (selects)", r"^v_cndmask"),
    ("v_cmp (compares)", r"^v_cmp"),
    ("shifts / masks / bitfield", r"^v_(lshl|lshr|ashr|alignbit|and|or|xor|bfe|bfi|lshl_add|lshl_or|and_or|or3|xad|perm)"),
    ("v_mul_lo/hi / mad_u32_u24", r"^v_mul|^v_mad_u32|^v_mad_i32"),
    ("v_mov (register moves)", r"^v_mov"),
    ("v_readlane / permlane / dpp", r"^v_(readlane|readfirstlane|writelane|permlane)|dpp"),
    ("other VALU", r"^v_"),
    ("LDS", r"^ds_"),
    ("global / buffer memory", r"^(global|buffer|flat|scratch)_"),
    ("scalar", r"^s_(?!waitcnt|nop|cbranch|branch)"),
    ("waitcnt / nop", r"^s_(waitcnt|nop)"),
    ("branches", r"^s_(cbranch|branch)"),
]


def classify(op):
    for name, rx in CLASSES:
        if re.search(rx, op):
            return name
    return "other"


def function_lines(asm, sym):
    start = asm.index(f"\n{sym}:") + 1
    end = asm.index(".Lfunc_end", start)
    return asm[start:end].splitlines()


def hot_loop(lines):
    """(first, last) line of the backward-branch loop with the most v_mad."""
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
    best, best_n = None, -1
    for i, ln in enumerate(lines):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            a = labels[m.group(2)]
            n = sum(1 for x in lines[a:i] if "v_mad_u64_u32" in x)
            if n > best_n:
                best, best_n = (a, i), n
    return best


def census(lines):
    c = collections.Counter()
    for ln in lines:
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        c[classify(s.split()[0])] += 1
    return c


def blocks(lines, a, b):
    """[(label, first, last)] basic blocks (by label) of lines[a..b]."""
    out, cur = [], None
    for i in range(a, b + 1):
        m = re.match(r"^(\.LBB\w+):", lines[i])
        if m or cur is None:
            if cur:
                out.append((cur[0], cur[1], i - 1))
            cur = (m.group(1) if m else "head", i)
    out.append((cur[0], cur[1], b))
    return out


NON_VALU = ("LDS", "global / buffer memory", "scalar", "waitcnt / nop", "branches", "other")


def summary(c):
    valu = sum(v for k, v in c.items() if k not in NON_VALU)
    return {"valu": valu, "v_mad_share": round(c["v_mad_u64_u32 (limb products)"] / max(valu, 1), 4),
            "classes": dict(sorted(c.items(), key=lambda kv: -kv[1]))}


def main():
    if len(sys.argv) > 1:
        asm_path = sys.argv[1]
    else:
        asm_path = "/tmp/census/msm.s"
        os.makedirs("/tmp/census", exist_ok=True)
        src = os.path.join(ROOT, "zero-knowledge-proofs_amd", "csrc")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", os.path.join(src, "msm.hip"), "-I", src, "-o", asm_path], check=True,
                       stderr=subprocess.DEVNULL)
    asm = open(asm_path).read()
    out = {}
    for name, sym in KERNELS.items():
        lines = function_lines(asm, sym)
        a, b = hot_loop(lines)
        bl = blocks(lines, a, b)
        mads = [sum(1 for x in lines[f:l + 1] if "v_mad_u64_u32" in x) for _, f, l in bl]
        order = sorted(range(len(bl)), key=lambda i: -mads[i])
        body, dbl = order[0], order[1]   # the mixed add's main path; the P == 0 doubling branch
        rest = collections.Counter()
        for i, (_, f, l) in enumerate(bl):
            if i not in (body, dbl):
                rest += census(lines[f:l + 1])
        out[name] = {"mixed_add_main_path": summary(census(lines[bl[body][1]:bl[body][2] + 1])),
                     "per_entry_loop_overhead": summary(rest),
                     "doubling_branch_rare": summary(census(lines[bl[dbl][1]:bl[dbl][2] + 1])),
                     "blocks": {lbl: m for (lbl, _, _), m in zip(bl, mads)}}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
