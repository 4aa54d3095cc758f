"""Debug: zk_qap_evaluate_at vs big-int Lagrange on small synthetic cases."""
import importlib, sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import binding as o
zkp = importlib.import_module("zero-knowledge-proofs_amd")
R = zkp.R
ctx = zkp.Context(0)
for log_n, nc in ((1, 2), (2, 4), (3, 8), (3, 5), (4, 16), (6, 64)):
    n = 1 << log_n
    z = o.synthetic_witness(n, 0x55 + log_n); zi = o.fr_ints(z)
    rp = np.arange(nc + 1, dtype=np.uint64); j = np.arange(nc, dtype=np.uint32)
    qap = zkp.QAP(zkp.CSRMatrices(nc, 3 * n + 1, [(rp, (1 + 3 * j).astype(np.uint32), None), (rp, (2 + 3 * j).astype(np.uint32), None), (rp, (3 + 3 * j).astype(np.uint32), None)]))
    w = o.fr_root_of_unity(log_n)
    for t in (0, 1, 2, w, 0x1234567890ABCDEF, R - 1, 12345678901234567890123456789):
        tn1 = (pow(t, n, R) - 1) % R
        if tn1:
            L = [pow(w, k, R) * tn1 * pow(n * (t - pow(w, k, R)), R - 2, R) % R for k in range(n)]
        else:
            L = [1 if pow(w, k, R) == t % R else 0 for k in range(n)]
        want = [sum(zi[c + 3 * k] * L[k] for k in range(nc)) % R for c in (1, 2, 3)]
        ev = qap.evaluate_at(t, z, ctx)
        got = [ev.a_val, ev.b_val, ev.c_val]
        ok = got == want and ev.z_val == tn1
        print(f"log_n={log_n} nc={nc} t={t:#x} ok={ok}" + ("" if ok else f"\n  got {[hex(x) for x in got]} z {hex(ev.z_val)}\n want {[hex(x) for x in want]} z {hex(tn1)}"), flush=True)
