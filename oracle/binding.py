"""ctypes binding for oracle/liboracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
Layouts: canonical little-endian u64 limbs; G1 = 13 words, G2 = 25 words
(see oracle/zk_oracle.h and include/zkp.h).
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

U64P = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
U32P = np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS")

OR_OK, OR_ERR_MSM_LEN, OR_ERR_INVALID_WITNESS, OR_ERR_QAP_DIVISION, OR_ERR_DOMAIN, OR_ERR_SETUP_PARAMS = range(6)


class OrR1CS(C.Structure):
    _fields_ = [("num_constraints", C.c_uint64), ("num_variables", C.c_uint64)] + [
        (f"{m}_{f}", t) for m in "abc" for f, t in
        (("rowptr", C.c_void_p), ("col", C.c_void_p), ("val", C.c_void_p))]


class OrPK(C.Structure):
    _fields_ = [("alpha_g1", C.c_uint64 * 13), ("beta_g1", C.c_uint64 * 13),
                ("delta_g1", C.c_uint64 * 13), ("beta_g2", C.c_uint64 * 25),
                ("delta_g2", C.c_uint64 * 25),
                ("a_g1", C.c_void_p), ("a_len", C.c_uint64),
                ("b_g1", C.c_void_p), ("b_len", C.c_uint64),
                ("b_g2", C.c_void_p), ("b2_len", C.c_uint64),
                ("ic_g1", C.c_void_p), ("ic_len", C.c_uint64),
                ("h_g1", C.c_void_p), ("h_len", C.c_uint64),
                ("num_public", C.c_uint64)]


class OrVK(C.Structure):
    _fields_ = [("alpha_g1", C.c_uint64 * 13), ("beta_g2", C.c_uint64 * 25),
                ("gamma_g2", C.c_uint64 * 25), ("delta_g2", C.c_uint64 * 25),
                ("ic_g1", C.c_void_p), ("ic_len", C.c_uint64), ("num_public", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        L.or_init()
        L.or_domain_size.restype = C.c_uint64
        L.or_splitmix64.restype = C.c_uint64
        L.or_set_threads(C.c_int(default_threads()))
        _lib = L
    return _lib


def default_threads():
    """ZK_ORACLE_THREADS, else OMP_NUM_THREADS (16 on the GPU box), else
    min(16, cpu_count): the oracle is a checker, parallel by default."""
    for k in ("ZK_ORACLE_THREADS", "OMP_NUM_THREADS"):
        if os.environ.get(k, "").isdigit():
            return max(1, int(os.environ[k]))
    return max(1, min(16, os.cpu_count() or 1))


def set_threads(n):
    """1 = the reference's single-threaded arkworks build (Cargo.lock:101-113)."""
    lib().or_set_threads(C.c_int(int(n)))


def get_threads():
    return int(lib().or_get_threads())


def g1_lin_bases(a, b, n):
    """(a + i b) G1 for i < n, (n, 13) words."""
    out = np.zeros((n, 13), dtype=np.uint64)
    lib().or_g1_lin_bases(_p(out), _p(np.array(int_to_limbs(a, 4), dtype=np.uint64)),
                          _p(np.array(int_to_limbs(b, 4), dtype=np.uint64)), C.c_uint64(n))
    return out


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


# ----------------------------------------------------------- conversions --
def int_to_limbs(v, k):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(k)]


def limbs_to_int(a):
    return sum(int(x) << (64 * i) for i, x in enumerate(a))


def fr_array(vals):
    return np.array([int_to_limbs(v, 4) for v in vals], dtype=np.uint64).reshape(-1, 4)


def fr_ints(arr):
    return [limbs_to_int(r) for r in np.asarray(arr).reshape(-1, 4)]


# --------------------------------------------------------------- R1CS -----
class CSR:
    """CSR form of an R1CS.  Keeps numpy buffers alive for the C struct."""

    def __init__(self, num_constraints, num_variables, mats):
        # mats: 3 x (rowptr u64[nc+1], col u32[nnz], val u64[nnz,4] or None)
        self.num_constraints, self.num_variables = num_constraints, num_variables
        self.mats = mats
        self.s = OrR1CS()
        self.s.num_constraints, self.s.num_variables = num_constraints, num_variables
        for m, (rp, col, val) in zip("abc", mats):
            setattr(self.s, f"{m}_rowptr", _p(rp))
            setattr(self.s, f"{m}_col", _p(col))
            setattr(self.s, f"{m}_val", _p(val) if val is not None else None)

    @classmethod
    def from_constraints(cls, constraints, num_variables):
        """constraints: list of (a, b, c) dicts var -> int coefficient."""
        mats = []
        for m in range(3):
            rp, cols, vals = [0], [], []
            for abc in constraints:
                for var in sorted(abc[m]):
                    cols.append(var)
                    vals.append(int_to_limbs(abc[m][var], 4))
                rp.append(len(cols))
            mats.append((np.array(rp, dtype=np.uint64), np.array(cols, dtype=np.uint32),
                         np.array(vals, dtype=np.uint64).reshape(-1, 4)))
        return cls(len(constraints), num_variables, mats)

    @classmethod
    def synthetic(cls, n):
        L = lib()
        rp = np.zeros(n + 1, dtype=np.uint64)
        cols = [np.zeros(max(n, 1), dtype=np.uint32) for _ in range(3)]
        L.or_synthetic_circuit(C.c_uint64(n), _p(rp), _p(cols[0]), _p(cols[1]), _p(cols[2]), None)
        return cls(n, 3 * n + 1, [(rp, cols[i], None) for i in range(3)])


def synthetic_witness(n, seed):
    z = np.zeros((3 * n + 1, 4), dtype=np.uint64)
    lib().or_synthetic_witness(C.c_uint64(n), C.c_uint64(seed), _p(z))
    return z


def random_fr(count, seed):
    out = np.zeros((count, 4), dtype=np.uint64)
    lib().or_random_fr(_p(out), C.c_uint64(count), C.c_uint64(seed))
    return out


def domain_size(nc):
    return int(lib().or_domain_size(C.c_uint64(nc)))


# ------------------------------------------------------------- calls ------
def msm_g1(bases, scalars):
    out = np.zeros(13, dtype=np.uint64)
    n = len(scalars)
    rc = lib().or_msm_g1(_p(out), _p(np.ascontiguousarray(bases, dtype=np.uint64)),
                         _p(np.ascontiguousarray(scalars, dtype=np.uint64)), C.c_uint64(n))
    assert rc == OR_OK
    return out


def msm_g2(bases, scalars):
    out = np.zeros(25, dtype=np.uint64)
    n = len(scalars)
    rc = lib().or_msm_g2(_p(out), _p(np.ascontiguousarray(bases, dtype=np.uint64)),
                         _p(np.ascontiguousarray(scalars, dtype=np.uint64)), C.c_uint64(n))
    assert rc == OR_OK
    return out


def fft(data, inverse=False):
    a = np.ascontiguousarray(data, dtype=np.uint64).copy()
    log_n = int(a.shape[0]).bit_length() - 1
    lib().or_fft(_p(a), C.c_uint32(log_n), C.c_int(int(inverse)))
    return a


def coset_fft(data, g, inverse=False):
    a = np.ascontiguousarray(data, dtype=np.uint64).copy()
    log_n = int(a.shape[0]).bit_length() - 1
    lib().or_coset_fft(_p(a), C.c_uint32(log_n), C.c_int(int(inverse)),
                       _p(np.array(int_to_limbs(g, 4), dtype=np.uint64)))
    return a


def quotient(csr, z, dense=False):
    n = domain_size(csr.num_constraints)
    h = np.zeros((n, 4), dtype=np.uint64)
    f = lib().or_quotient_dense if dense else lib().or_quotient
    rc = f(C.byref(csr.s), _p(np.ascontiguousarray(z, dtype=np.uint64)), _p(h))
    return rc, h


def validate(csr, z):
    return lib().or_validate(C.byref(csr.s), _p(np.ascontiguousarray(z, dtype=np.uint64)),
                             C.c_uint64(len(z)))


class PK:
    def __init__(self, V, n, num_public):
        self.a_g1 = np.zeros((V, 13), dtype=np.uint64)
        self.b_g1 = np.zeros((V, 13), dtype=np.uint64)
        self.b_g2 = np.zeros((V, 25), dtype=np.uint64)
        self.ic_g1 = np.zeros((max(V - num_public - 1, 1), 13), dtype=np.uint64)
        self.h_g1 = np.zeros((n, 13), dtype=np.uint64)
        self.s = OrPK()
        self.s.a_g1, self.s.b_g1, self.s.b_g2 = _p(self.a_g1), _p(self.b_g1), _p(self.b_g2)
        self.s.ic_g1, self.s.h_g1 = _p(self.ic_g1), _p(self.h_g1)

    def field(self, name):
        return np.array(getattr(self.s, name), dtype=np.uint64)


class VK:
    def __init__(self, num_public):
        self.ic_g1 = np.zeros((num_public + 1, 13), dtype=np.uint64)
        self.s = OrVK()
        self.s.ic_g1 = _p(self.ic_g1)

    def field(self, name):
        return np.array(getattr(self.s, name), dtype=np.uint64)


def setup(csr, params, num_public, nthreads=1):
    """params: 5 ints (alpha, beta, gamma, delta, tau). Returns (rc, pk, vk)."""
    V, n = csr.num_variables, domain_size(csr.num_constraints)
    pk, vk = PK(V, n, num_public), VK(num_public)
    par = np.array([int_to_limbs(p, 4) for p in params], dtype=np.uint64).reshape(-1)
    rc = lib().or_setup(C.byref(csr.s), _p(par), C.c_uint64(num_public), C.byref(pk.s),
                        C.byref(vk.s), C.c_int(nthreads))
    return rc, pk, vk


def setup_sample(csr, params, num_public, vars, hidx):
    """Sampled key entries by or_setup's arithmetic: {a_g1, b_g1, b_g2, ic}
    for the variables in vars (ic: pk ic_g1[v - num_public - 1] for v >
    num_public) and h_g1 for the coefficient indices in hidx."""
    vars = np.ascontiguousarray(vars, dtype=np.uint64)
    hidx = np.ascontiguousarray(hidx, dtype=np.uint64)
    out = {"a_g1": np.zeros((len(vars), 13), dtype=np.uint64), "b_g1": np.zeros((len(vars), 13), dtype=np.uint64),
           "b_g2": np.zeros((len(vars), 25), dtype=np.uint64), "ic": np.zeros((len(vars), 13), dtype=np.uint64),
           "h_g1": np.zeros((len(hidx), 13), dtype=np.uint64)}
    par = np.array([int_to_limbs(p, 4) for p in params], dtype=np.uint64).reshape(-1)
    rc = lib().or_setup_sample(C.byref(csr.s), _p(par), C.c_uint64(num_public), _p(vars), C.c_uint64(len(vars)),
                               _p(hidx), C.c_uint64(len(hidx)), _p(out["a_g1"]), _p(out["b_g1"]),
                               _p(out["b_g2"]), _p(out["ic"]), _p(out["h_g1"]))
    return rc, out


def prove(pk, csr, z, num_public, r, s):
    """Returns (rc, proof words[51])."""
    proof = np.zeros(51, dtype=np.uint64)
    rr = np.array(int_to_limbs(r, 4), dtype=np.uint64)
    ss = np.array(int_to_limbs(s, 4), dtype=np.uint64)
    z = np.ascontiguousarray(z, dtype=np.uint64)
    rc = lib().or_prove(C.byref(pk.s), C.byref(csr.s), _p(z), C.c_uint64(len(z)),
                        C.c_uint64(num_public), _p(rr), _p(ss), _p(proof))
    return rc, proof


def g1_generator():
    out = np.zeros(13, dtype=np.uint64)
    lib().or_g1_generator(_p(out))
    return out


def g2_generator():
    out = np.zeros(25, dtype=np.uint64)
    lib().or_g2_generator(_p(out))
    return out


def g1_mul(p, k):
    out = np.zeros(13, dtype=np.uint64)
    lib().or_g1_mul(_p(out), _p(np.ascontiguousarray(p, dtype=np.uint64)),
                    _p(np.array(int_to_limbs(k, 4), dtype=np.uint64)))
    return out


def g2_mul(p, k):
    out = np.zeros(25, dtype=np.uint64)
    lib().or_g2_mul(_p(out), _p(np.ascontiguousarray(p, dtype=np.uint64)),
                    _p(np.array(int_to_limbs(k, 4), dtype=np.uint64)))
    return out


def g1_add(a, b):
    out = np.zeros(13, dtype=np.uint64)
    lib().or_g1_add(_p(out), _p(np.ascontiguousarray(a, dtype=np.uint64)),
                    _p(np.ascontiguousarray(b, dtype=np.uint64)))
    return out


def g1_on_curve(p):
    return bool(lib().or_g1_on_curve(_p(np.ascontiguousarray(p, dtype=np.uint64))))


def g2_on_curve(p):
    return bool(lib().or_g2_on_curve(_p(np.ascontiguousarray(p, dtype=np.uint64))))


def g1_compress(p):
    out = (C.c_uint8 * 48)()
    lib().or_g1_compress(out, _p(np.ascontiguousarray(p, dtype=np.uint64)))
    return bytes(out)


def g2_compress(p):
    out = (C.c_uint8 * 96)()
    lib().or_g2_compress(out, _p(np.ascontiguousarray(p, dtype=np.uint64)))
    return bytes(out)


def proof_compress(proof):
    return g1_compress(proof[:13]) + g2_compress(proof[13:38]) + g1_compress(proof[38:51])


def fr_root_of_unity(log_n):
    out = np.zeros(4, dtype=np.uint64)
    lib().or_fr_root_of_unity(_p(out), C.c_uint32(log_n))
    return limbs_to_int(out)
