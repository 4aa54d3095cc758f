"""The reference's own quotient scaling: the literal dense
restatement of QAP::from_r1cs + compute_quotient_polynomial
(crates/groth16-qap/src/lib.rs:95-187, 225-271: per-variable interpolants of
the dense 3 x n x V matrices, dense products, long division) against the
O(n log n) sparse quotient, both on one host thread, on the synthetic
circuit at n = 2^6 .. 2^12 (the dense form is infeasible beyond).  Both are
oracle/ C restatements (test infrastructure); they must return the same H.

  python tools/dense_scaling.py [max_log_n]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import binding as oracle  # noqa: E402


def main():
    top = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    oracle.set_threads(1)
    rows = []
    for log_n in range(6, top + 1):
        n = 1 << log_n
        csr = oracle.CSR.synthetic(n)
        z = oracle.synthetic_witness(n, 77 + log_n)
        t0 = time.perf_counter()
        rc_d, h_d = oracle.quotient(csr, z, dense=True)
        t_d = time.perf_counter() - t0
        t0 = time.perf_counter()
        rc_s, h_s = oracle.quotient(csr, z)
        t_s = time.perf_counter() - t0
        rows.append({"log_n": log_n, "V": 3 * n + 1, "dense_s": round(t_d, 4), "sparse_s": round(t_s, 5),
                     "ratio": round(t_d / max(t_s, 1e-9), 1),
                     "same_h": bool(rc_d == rc_s == 0 and np.array_equal(h_d, h_s))})
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({"dense_vs_sparse": rows}))


if __name__ == "__main__":
    main()
