"""zero-knowledge-proofs_amd -- MI355X-native Groth16 prover hot path.

Python mirror of the reference's prover/setup interface (vats98754/
zero-knowledge-proofs, Rust) over the C ABI of include/zkp.h, which is
implemented by libzkp_amd.so (hand-written gfx950 HIP kernels).  Names,
argument meaning and error behaviour follow the reference crates:

  R1CS / LinearCombination / Variable  crates/groth16-r1cs/src/lib.rs:16-358
  QAP.from_r1cs / degree               crates/groth16-qap/src/lib.rs:95-187, 285-294
  SetupParams / CRS.generate_from_qap  crates/groth16-setup/src/lib.rs:82-278
  Witness / Prover.prove / Proof       crates/groth16-core/src/lib.rs:27-272
  Verifier / BatchVerifier             crates/groth16-core/src/lib.rs:303-432
  GrothError kinds                     crates/groth16-core/src/lib.rs:47-77

There is no CPU fallback: every compute call goes through libzkp_amd.so on a
GPU, and loading fails loudly when the library (or a GPU) is missing.
The package directory name contains hyphens; import it with
importlib.import_module("zero-knowledge-proofs_amd").
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# ZK_AMD_LIB: an alternative build of the same library (tooling: A/B runs of
# variant builds; the library itself reads no environment variables)
LIB_PATH = os.environ.get("ZK_AMD_LIB") or os.path.join(_HERE, "libzkp_amd.so")
# the GPU tests' diagnostic hooks (include/zkp_test.h), built on top of
# libzkp_amd.so; the product path never loads it
TEST_LIB_PATH = os.path.join(os.path.dirname(LIB_PATH), "libzkp_amd_test.so")

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001  # Fr modulus

ZK_OK, ZK_ERR_MSM_LEN, ZK_ERR_INVALID_WITNESS, ZK_ERR_QAP_DIVISION, ZK_ERR_DOMAIN, \
    ZK_ERR_SETUP_PARAMS, ZK_ERR_DEVICE, ZK_ERR_RCCL, ZK_ERR_ARG, ZK_ERR_DIMENSION = range(10)
G1_WORDS, G2_WORDS = 13, 25
PARTIAL_BYTES = 1536

# C-ABI symbols declared in include/zkp.h (checked by tests/test_capi.py)
EXPORTS = (
    "zk_ctx_create", "zk_ctx_destroy", "zk_last_error", "zk_ctx_synchronize",
    "zk_ctx_profile", "zk_ctx_profile_read",
    "zk_msm_g1", "zk_msm_g2", "zk_msm_g1_upload", "zk_msm_g2_upload", "zk_msm_bases_free",
    "zk_msm_g1_dev", "zk_msm_g2_dev", "zk_ntt_fr", "zk_ntt_fr_dev",
    "zk_groth16_setup", "zk_groth16_setup_dev", "zk_pk_upload", "zk_pk_free",
    "zk_groth16_prove", "zk_groth16_prove_dev", "zk_pk_upload_shard",
    "zk_groth16_setup_dev_shard", "zk_groth16_prove_partial", "zk_groth16_prove_combine",
    "zk_proof_serialize_compressed", "zk_rccl_unique_id", "zk_ctx_attach_rccl",
    "zk_proof_deserialize_compressed", "zk_groth16_verify",
    "zk_groth16_verify_batch", "zk_pairing_product_is_one", "zk_msm_g1_upload_windows",
    "zk_msm_g2_upload_windows", "zk_build_id", "zk_ctx_set_schedule", "zk_qap_evaluate_at",
    "zk_poly_evaluate_batch", "zk_synthetic_witness_dev", "zk_ctx_set_option", "zk_ctx_timeline_read",
    "zk_ctx_attach_exchange", "zk_groth16_witness_ranges", "zk_groth16_prove_partial_host",
    "zk_ctx_detach_exchange",
)
# include/zkp_test.h (libzkp_amd_test.so)
TEST_EXPORTS = ("zk_test_prove_virtual_shards", "zk_test_exchange", "zk_test_fault_after_exchange",
                "zk_test_pk_bases", "zk_test_pk_info")
ZK_OPT_QUOTIENT_PATH, ZK_OPT_PROVE_WIN_C, ZK_OPT_EXCHANGE_TIMEOUT_MS, ZK_OPT_DIST_QUOTIENT = 1, 2, 3, 5
ZK_OPT_EXCHANGE_FIRST = 6
CSRC = os.path.join(_HERE, "csrc")


# ------------------------------------------------------------- errors ----
class GrothError(Exception):
    """crates/groth16-core/src/lib.rs:47-77"""


class InvalidWitness(GrothError):
    pass


class MSMError(GrothError):
    pass


class QAPError(GrothError):
    """crates/groth16-qap/src/lib.rs:63-86"""


class PolynomialDivisionFailed(QAPError):
    pass


class DomainTooSmall(QAPError):
    pass


class DimensionMismatch(QAPError):
    """QAPError::FieldError(FieldError::DimensionMismatch), qap:191-198"""


class SetupError(GrothError):
    """crates/groth16-setup/src/lib.rs:95-113 (InvalidParams)"""


class DeviceError(GrothError):
    pass


class ExchangeError(DeviceError):
    """ZK_ERR_RCCL: the multi-GPU exchange (RCCL or host-staged) failed or was aborted."""


_STATUS = {ZK_ERR_MSM_LEN: MSMError, ZK_ERR_INVALID_WITNESS: InvalidWitness,
           ZK_ERR_QAP_DIVISION: PolynomialDivisionFailed, ZK_ERR_DOMAIN: DomainTooSmall,
           ZK_ERR_SETUP_PARAMS: SetupError, ZK_ERR_DEVICE: DeviceError,
           ZK_ERR_RCCL: ExchangeError, ZK_ERR_ARG: ValueError, ZK_ERR_DIMENSION: DimensionMismatch}


# ---------------------------------------------------------- C structs ----
_A2A_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
_AMAX_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)
_ABORT_FN = C.CFUNCTYPE(None, C.c_void_p)


class _ExchangeOps(C.Structure):
    _fields_ = [("all_to_all", _A2A_FN), ("all_reduce_max", _AMAX_FN), ("abort", _ABORT_FN), ("user", C.c_void_p)]


class _Fr(C.Structure):
    _fields_ = [("l", C.c_uint64 * 4)]


class _G1(C.Structure):
    _fields_ = [("w", C.c_uint64 * G1_WORDS)]


class _G2(C.Structure):
    _fields_ = [("w", C.c_uint64 * G2_WORDS)]


class _Proof(C.Structure):
    _fields_ = [("a", _G1), ("b", _G2), ("c", _G1)]


class _CSR(C.Structure):
    _fields_ = [("num_constraints", C.c_uint64), ("num_variables", C.c_uint64)] + [
        (f"{m}_{f}", C.c_void_p) for m in "abc" for f in ("rowptr", "col", "val")]


class _SetupParams(C.Structure):
    _fields_ = [(k, _Fr) for k in ("alpha", "beta", "gamma", "delta", "tau")]


class _PK(C.Structure):
    _fields_ = [("alpha_g1", _G1), ("beta_g1", _G1), ("delta_g1", _G1),
                ("beta_g2", _G2), ("delta_g2", _G2),
                ("a_g1", C.c_void_p), ("a_len", C.c_uint64),
                ("b_g1", C.c_void_p), ("b_len", C.c_uint64),
                ("b_g2", C.c_void_p), ("b2_len", C.c_uint64),
                ("ic_g1", C.c_void_p), ("ic_len", C.c_uint64),
                ("h_g1", C.c_void_p), ("h_len", C.c_uint64),
                ("num_public", C.c_uint64)]


class _VK(C.Structure):
    _fields_ = [("alpha_g1", _G1), ("beta_g2", _G2), ("gamma_g2", _G2), ("delta_g2", _G2),
                ("ic_g1", C.c_void_p), ("ic_len", C.c_uint64), ("num_public", C.c_uint64)]


_lib = None


def lib():
    """Load libzkp_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C zero-knowledge-proofs_amd/csrc`")
        # One HIP runtime per process: torch bundles its own libamdhip64
        # (SONAME libamdhip64.so.7).  Loading torch first makes our DT_NEEDED
        # bind to that copy, so torch device memory, streams and RCCL
        # (torch.distributed) share the runtime with our kernels.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        L.zk_ctx_create.restype = C.c_void_p
        L.zk_ctx_create.argtypes = [C.c_int]
        L.zk_ctx_destroy.argtypes = [C.c_void_p]
        L.zk_last_error.restype = C.c_char_p
        L.zk_last_error.argtypes = [C.c_void_p]
        L.zk_build_id.restype = C.c_char_p
        for name in EXPORTS:
            # an A/B build of an older revision (ZK_AMD_LIB, tooling only) may
            # lack entry points added since; the product library must have all
            f = getattr(L, name, None)
            if f is None:
                if os.environ.get("ZK_AMD_LIB"):
                    continue
                raise ImportError(f"{LIB_PATH} does not export {name}")
            if name not in ("zk_ctx_create", "zk_ctx_destroy", "zk_last_error",
                            "zk_msm_bases_free", "zk_pk_free", "zk_build_id"):
                f.restype = C.c_int
        L.zk_msm_bases_free.argtypes = [C.c_void_p]
        L.zk_pk_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


_test_lib = None


def test_lib():
    """Load libzkp_amd_test.so (include/zkp_test.h: virtual ranks, the bare
    exchange, fault injection) on top of libzkp_amd.so -- tests only."""
    global _test_lib
    if _test_lib is None:
        lib()
        if not os.path.exists(TEST_LIB_PATH):
            raise ImportError(f"{TEST_LIB_PATH} not built: run `make -C zero-knowledge-proofs_amd/csrc`")
        T = C.CDLL(TEST_LIB_PATH)
        for name in TEST_EXPORTS:
            getattr(T, name).restype = C.c_int
        _test_lib = T
    return _test_lib


def _p(a):
    return C.c_void_p(a.ctypes.data)


def build_id():
    """zk_build_id(): '<git HEAD>[-dirty] src:<source hash>' of the loaded library."""
    return lib().zk_build_id().decode()


def source_hash():
    """sha256 (16 hex) over csrc/*.hip and *.hpp (sorted) + include/zkp.h of THIS
    tree -- what the Makefile embeds in zk_build_id()."""
    import hashlib
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp")))
    h = hashlib.sha256()
    for f in names:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    for hdr in ("zkp.h", "zkp_test.h"):
        with open(os.path.join(os.path.dirname(_HERE), "include", hdr), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check_build():
    """Raise unless the loaded libzkp_amd.so was built from this tree's sources."""
    bid = build_id()
    want = source_hash()
    if not bid.endswith("src:" + want):
        raise ImportError(f"libzkp_amd.so build id {bid!r} does not match the sources (src:{want}); rebuild it")
    return bid


def _check(rc, ctx=None, what=""):
    if rc == ZK_OK:
        return
    detail = ""
    if ctx is not None:
        msg = lib().zk_last_error(ctx._h)
        detail = msg.decode() if msg else ""
    raise _STATUS.get(rc, GrothError)(f"{what} failed ({rc}) {detail}".strip())


# ------------------------------------------------------------ helpers ----
def to_limbs(v, k=4):
    v = int(v)
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(k)]


def from_limbs(a):
    return sum(int(x) << (64 * i) for i, x in enumerate(np.asarray(a).reshape(-1)))


def fr_array(values):
    """ints (reduced mod r) -> (n, 4) uint64 canonical limbs."""
    values = [int(v) % R for v in values]
    out = np.zeros((len(values), 4), dtype=np.uint64)
    for i, v in enumerate(values):
        out[i] = to_limbs(v)
    return out


def _fr(v):
    f = _Fr()
    for i, x in enumerate(to_limbs(int(v) % R)):
        f.l[i] = x
    return f


# ------------------------------------------------------------ context ----
class Context:
    """One GPU (zk_ctx): streams, cached NTT domains, MSM workspaces."""

    def __init__(self, device=0):
        self._h = lib().zk_ctx_create(int(device))
        if not self._h:
            raise DeviceError(f"zk_ctx_create({device}) failed: no usable GPU")
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            lib().zk_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- RCCL communicator for the distributed quotient of sharded keys ----
    @staticmethod
    def rccl_unique_id():
        buf = (C.c_uint8 * 128)()
        _check(lib().zk_rccl_unique_id(buf), None, "zk_rccl_unique_id")
        return bytes(buf)

    def attach_rccl(self, unique_id, rank, world):
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        _check(lib().zk_ctx_attach_rccl(C.c_void_p(self._h), buf, C.c_int(rank), C.c_int(world)), self,
               "zk_ctx_attach_rccl")

    def detach_exchange(self):
        """zk_ctx_detach_exchange: drop the attached exchange (RCCL: a local
        ncclCommAbort); sharded keys then compute the whole quotient on every
        rank.  Every rank of the job detaches together."""
        _check(lib().zk_ctx_detach_exchange(C.c_void_p(self._h)), self, "zk_ctx_detach_exchange")
        self._exchange_refs = None

    def test_exchange(self, chunk_bytes, status):
        """zk_test_exchange: one all-to-all and one status agreement on the
        attached exchange (RCCL or host-staged); returns the agreed max,
        raises ExchangeError when a received chunk is wrong."""
        out = C.c_int32()
        _check(test_lib().zk_test_exchange(C.c_void_p(self._h), C.c_size_t(chunk_bytes), C.c_int32(status),
                                           C.byref(out)), self, "zk_test_exchange")
        return out.value

    def test_fault_after_exchange(self, k):
        """zk_test_fault_after_exchange: the next distributed-quotient proof
        on this ctx fails right after its k-th all-to-all (tests only)."""
        _check(test_lib().zk_test_fault_after_exchange(C.c_void_p(self._h), C.c_int(int(k))), self,
               "zk_test_fault_after_exchange")

    def attach_exchange(self, exchange, rank, world):
        """zk_ctx_attach_exchange: the distributed quotient of sharded keys
        over a host-staged transport.  `exchange` has all_to_all(send_ptr,
        recv_ptr, chunk_bytes), all_reduce_max(int) -> int and abort()
        (e.g. TorchExchange over a gloo process group)."""
        def a2a(_u, send, recv, chunk):
            try:
                exchange.all_to_all(send, recv, chunk)
                return 0
            except Exception:
                return 1

        def amax(_u, pv):
            try:
                p = C.cast(pv, C.POINTER(C.c_int32))
                p[0] = int(exchange.all_reduce_max(int(p[0])))
                return 0
            except Exception:
                return 1

        def abort(_u):
            try:
                exchange.abort()
            except Exception:
                pass
        ops = _ExchangeOps(_A2A_FN(a2a), _AMAX_FN(amax), _ABORT_FN(abort), None)
        self._exchange_refs = (ops, exchange)   # the callbacks must outlive the attachment
        _check(lib().zk_ctx_attach_exchange(C.c_void_p(self._h), C.byref(ops), C.c_int(rank), C.c_int(world)), self,
               "zk_ctx_attach_exchange")

    def set_schedule(self, schedule=-1):
        """zk_ctx_set_schedule: -1 / 0 overlapped streams (default), 3 every
        prove kernel in order on one stream (isolated kernel durations)."""
        _check(lib().zk_ctx_set_schedule(C.c_void_p(self._h), C.c_int(int(schedule))), self, "zk_ctx_set_schedule")

    def set_option(self, option, value):
        """zk_ctx_set_option: ZK_OPT_QUOTIENT_PATH (-1 by size, 0 small-domain,
        1 large-domain), ZK_OPT_PROVE_WIN_C (0 by size, 16, 22; keys made
        afterwards), ZK_OPT_EXCHANGE_TIMEOUT_MS (>= 1), ZK_OPT_DIST_QUOTIENT
        (-1 distributed when an exchange of the key's shape is attached, 0
        replicated) or ZK_OPT_EXCHANGE_FIRST (0 MSMs start with the witness, 1
        they wait for the distributed quotient).  Explicit path choices for
        tests and A/B runs."""
        _check(lib().zk_ctx_set_option(C.c_void_p(self._h), C.c_int(int(option)), C.c_int64(int(value))), self,
               "zk_ctx_set_option")

    def timeline_read(self):
        """The per-launch stream timeline recorded under profile(2), as text."""
        n = C.c_size_t()
        _check(lib().zk_ctx_timeline_read(C.c_void_p(self._h), None, C.c_size_t(0), C.byref(n)), self, "timeline")
        buf = C.create_string_buffer(n.value + 1)
        _check(lib().zk_ctx_timeline_read(C.c_void_p(self._h), buf, C.c_size_t(n.value + 1), C.byref(n)), self,
               "timeline")
        return buf.value.decode()

    def synthetic_witness(self, n, seed):
        """The groth16-cli circuit's witness z (3n+1 canonical Fr) generated
        on this GPU -> torch int64 tensor (3n+1, 4) on its device."""
        import torch
        z = torch.empty((3 * n + 1, 4), dtype=torch.int64, device=f"cuda:{self.device}")
        _check(lib().zk_synthetic_witness_dev(C.c_void_p(self._h), C.c_uint64(n), C.c_uint64(seed),
                                              C.c_void_p(z.data_ptr())), self, "zk_synthetic_witness_dev")
        return z

    # ---- live kernel timing (HIP events on the launching stream) ----
    def profile(self, enable=True):
        """0/False off, 1/True per-phase kernel times, 2 also the stream timeline."""
        _check(lib().zk_ctx_profile(C.c_void_p(self._h), C.c_int(int(enable))), self, "zk_ctx_profile")

    def profile_read(self):
        """{phase: {"ms": total device ms, "launches": n, "units": work units}}"""
        cap, k = 4096, 64
        names = C.create_string_buffer(cap)
        ms = (C.c_double * k)()
        la = (C.c_uint64 * k)()
        un = (C.c_uint64 * k)()
        n = C.c_size_t()
        _check(lib().zk_ctx_profile_read(C.c_void_p(self._h), names, C.c_size_t(cap), ms, la, un,
                                         C.c_size_t(k), C.byref(n)), self, "zk_ctx_profile_read")
        keys = names.raw.split(b"\0")[:n.value]
        return {kk.decode(): {"ms": ms[i], "launches": la[i], "units": un[i]} for i, kk in enumerate(keys)}

    # ---- MSM (crates/groth16-core/src/lib.rs:275-300) ----
    def msm_g1(self, bases, scalars, scalar_bits=255):
        """bases: (n, 13) uint64 canonical affine; scalars: (n, 4) uint64 canonical Fr."""
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, G1_WORDS)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(G1_WORDS, dtype=np.uint64)
        rc = lib().zk_msm_g1(C.c_void_p(self._h), _p(bases), C.c_size_t(len(bases)), _p(scalars),
                             C.c_size_t(len(scalars)), C.c_uint32(scalar_bits), _p(out))
        _check(rc, self, "zk_msm_g1")
        return out

    def msm_g2(self, bases, scalars, scalar_bits=255):
        bases = np.ascontiguousarray(bases, dtype=np.uint64).reshape(-1, G2_WORDS)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
        out = np.zeros(G2_WORDS, dtype=np.uint64)
        rc = lib().zk_msm_g2(C.c_void_p(self._h), _p(bases), C.c_size_t(len(bases)), _p(scalars),
                             C.c_size_t(len(scalars)), C.c_uint32(scalar_bits), _p(out))
        _check(rc, self, "zk_msm_g2")
        return out

    # ---- NTT (ark-poly Radix2EvaluationDomain fft / ifft / coset) ----
    def ntt(self, data, inverse=False, coset=None):
        a = np.ascontiguousarray(data, dtype=np.uint64).reshape(-1, 4).copy()
        n = len(a)
        log_n = n.bit_length() - 1
        if n == 0 or (1 << log_n) != n:
            raise DomainTooSmall(f"NTT size {n} is not a power of two")
        g = C.byref(_fr(coset)) if coset is not None else None
        rc = lib().zk_ntt_fr(C.c_void_p(self._h), _p(a), C.c_uint32(log_n),
                             C.c_int(-1 if inverse else 1), g)
        _check(rc, self, "zk_ntt_fr")
        return a


# --------------------------------------------------------------- R1CS ----
class Variable(int):
    """crates/groth16-r1cs/src/lib.rs:20-35; Variable.ONE = 0."""

    def index(self):
        return int(self)


Variable.ONE = Variable(0)


class LinearCombination:
    """Sparse sum of coeff * var (crates/groth16-r1cs/src/lib.rs:46-118)."""

    def __init__(self, terms=None):
        self.terms = {}
        for v, c in (terms or {}).items():
            self.add_term(v, c)

    @classmethod
    def from_variable(cls, var):
        return cls({Variable(var): 1})

    @classmethod
    def from_constant(cls, c):
        return cls({Variable.ONE: c} if int(c) % R else {})

    def add_term(self, var, coeff):
        coeff = int(coeff) % R
        if coeff == 0:
            return
        var = Variable(var)
        v = (self.terms.get(var, 0) + coeff) % R
        if v:
            self.terms[var] = v
        else:
            self.terms.pop(var, None)

    def sub_lc(self, other):
        for v, c in other.terms.items():
            self.add_term(v, -c)


class R1CS:
    """crates/groth16-r1cs/src/lib.rs:229-358 (the builder subset on the path)."""

    def __init__(self, num_public_inputs=0):
        self.constraints = []
        self.num_public_inputs = num_public_inputs
        self.num_variables = 1 + num_public_inputs

    def allocate_variable(self):
        v = Variable(self.num_variables)
        self.num_variables += 1
        return v

    def add_constraint(self, a, b, c):
        self.constraints.append((a, b, c))

    def enforce_multiplication(self, a, b, c):
        self.add_constraint(a, b, c)

    def enforce_equal(self, left, right):
        diff = LinearCombination(dict(left.terms))
        diff.sub_lc(right)
        self.add_constraint(diff, LinearCombination.from_constant(1), LinearCombination())

    def num_constraints(self):
        return len(self.constraints)

    def is_satisfied(self, z):
        z = [int(x) % R for x in z]
        for a, b, c in self.constraints:
            ev = [sum(z[v] * k for v, k in lc.terms.items() if v < len(z)) % R for lc in (a, b, c)]
            if ev[0] * ev[1] % R != ev[2]:
                return False
        return True


class CSRMatrices:
    """The constraint matrices in CSR (zk_r1cs_csr); keeps the buffers alive."""

    def __init__(self, num_constraints, num_variables, mats):
        self.num_constraints, self.num_variables = int(num_constraints), int(num_variables)
        self.mats = mats  # 3 x (rowptr u64[nc+1], col u32[nnz], val u64[nnz,4] or None)
        self.s = _CSR()
        self.s.num_constraints, self.s.num_variables = self.num_constraints, self.num_variables
        for m, (rp, col, val) in zip("abc", mats):
            setattr(self.s, f"{m}_rowptr", rp.ctypes.data)
            setattr(self.s, f"{m}_col", col.ctypes.data)
            setattr(self.s, f"{m}_val", val.ctypes.data if val is not None else None)

    @classmethod
    def from_r1cs(cls, cs):
        mats = []
        for m in range(3):
            rp, cols, vals = [0], [], []
            for con in cs.constraints:
                for var in sorted(con[m].terms):
                    cols.append(int(var))
                    vals.append(to_limbs(con[m].terms[var]))
                rp.append(len(cols))
            mats.append((np.array(rp, dtype=np.uint64), np.array(cols, dtype=np.uint32),
                         np.array(vals, dtype=np.uint64).reshape(-1, 4)))
        return cls(cs.num_constraints(), cs.num_variables, mats)

    @classmethod
    def synthetic(cls, n):
        """groth16-cli generate_crs circuit (crates/groth16-cli/src/lib.rs:57-70):
        n x (x_j * y_j = z_j), variables x_j = 1+3j, y_j = 2+3j, z_j = 3+3j,
        unit coefficients (val = NULL)."""
        rp = np.arange(n + 1, dtype=np.uint64)
        j = np.arange(n, dtype=np.uint32)
        mats = [(rp, (1 + 3 * j).astype(np.uint32), None), (rp, (2 + 3 * j).astype(np.uint32), None),
                (rp, (3 + 3 * j).astype(np.uint32), None)]
        return cls(n, 3 * n + 1, mats)


class QAP:
    """crates/groth16-qap/src/lib.rs:31-46 in sparse form: the constraint
    matrices plus the radix-2 domain; the per-variable polynomials of the
    reference are never materialised (they are implied by the matrices)."""

    def __init__(self, csr):
        self.csr = csr
        self.num_variables = csr.num_variables
        self.num_constraints = csr.num_constraints
        n = 1
        while n < self.num_constraints:
            n <<= 1
        if n.bit_length() - 1 > 32:
            raise DomainTooSmall(f"domain {n} exceeds 2^32")
        self.domain_size = n

    @classmethod
    def from_r1cs(cls, cs):
        return cls(CSRMatrices.from_r1cs(cs))

    def degree(self):
        """max(per-variable degree < n, deg Z = n) = n (qap:285-294)."""
        return self.domain_size

    def evaluate_at(self, point, assignment, ctx=None):
        """QAP::evaluate_at (qap:190-220) on the GPU -> QAPEvaluation with
        A(point), B(point), C(point) = sum_i z_i A_i(point) ..., Z(point)."""
        ctx = ctx or default_context()
        z = _fr_rows(assignment)
        out = (_Fr * 4)()
        rc = lib().zk_qap_evaluate_at(C.c_void_p(ctx._h), C.byref(self.csr.s), C.byref(_fr(point)),
                                      _p(z) if len(z) else None, C.c_size_t(len(z)), out)
        _check(rc, ctx, "zk_qap_evaluate_at")
        a, b, c, zv = (sum(int(x) << (64 * i) for i, x in enumerate(o.l)) for o in out)
        return QAPEvaluation(a, b, c, zv)

    @staticmethod
    def verify_evaluation(ev):
        """QAP::verify_evaluation (qap:274-282)."""
        if ev.h_val is not None:
            return (ev.a_val * ev.b_val - ev.c_val) % R == ev.h_val * ev.z_val % R
        return ev.a_val * ev.b_val % R == ev.c_val


class QAPEvaluation:
    """QAPEvaluation (crates/groth16-qap/src/lib.rs:49-57): field values as ints."""

    def __init__(self, a_val, b_val, c_val, z_val, h_val=None):
        self.a_val, self.b_val, self.c_val, self.z_val, self.h_val = a_val, b_val, c_val, z_val, h_val


def batch_evaluate(polynomials, point, ctx=None):
    """qap utils::batch_evaluate (qap:315-322) on the GPU: each polynomial is
    a coefficient list (lowest degree first) of Fr ints or an (m, 4) array."""
    ctx = ctx or default_context()
    rows = [_fr_rows(p) if len(p) else np.zeros((0, 4), dtype=np.uint64) for p in polynomials]
    offs = np.zeros(len(rows) + 1, dtype=np.uint64)
    for i, r in enumerate(rows):
        offs[i + 1] = offs[i] + len(r)
    flat = np.ascontiguousarray(np.concatenate(rows) if rows else np.zeros((0, 4), dtype=np.uint64))
    out = np.zeros((max(len(rows), 1), 4), dtype=np.uint64)
    rc = lib().zk_poly_evaluate_batch(C.c_void_p(ctx._h), _p(flat) if len(flat) else None, _p(offs),
                                      C.c_size_t(len(rows)), C.byref(_fr(point)), _p(out))
    _check(rc, ctx, "zk_poly_evaluate_batch")
    return [from_limbs(o) for o in out[:len(rows)]]


_default_ctx = None


def default_context():
    """Context(0), created on first use (for reference-shaped calls that take no ctx)."""
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# -------------------------------------------------------------- setup ----
class SetupParams:
    """crates/groth16-setup/src/lib.rs:82-136 (`s` is tau)."""

    def __init__(self, alpha, beta, gamma, delta, s):
        self.alpha, self.beta, self.gamma, self.delta, self.s = (int(x) % R for x in (alpha, beta, gamma, delta, s))

    @classmethod
    def random(cls, rng):
        """rng: callable returning a uniform Fr int (e.g. SplitMix64.fr)."""
        return cls(rng(), rng(), rng(), rng(), rng())

    def validate(self):
        if 0 in (self.alpha, self.beta, self.gamma, self.delta):
            raise SetupError("Setup parameters must be non-zero")

    def _c(self):
        p = _SetupParams()
        for k, v in (("alpha", self.alpha), ("beta", self.beta), ("gamma", self.gamma),
                     ("delta", self.delta), ("tau", self.s)):
            setattr(p, k, _fr(v))
        return p


class ProvingKey:
    """crates/groth16-setup/src/lib.rs:27-52 (host arrays, canonical affine)."""

    def __init__(self, V, n, num_public, qap):
        self.a_g1 = np.zeros((V, G1_WORDS), dtype=np.uint64)
        self.b_g1 = np.zeros((V, G1_WORDS), dtype=np.uint64)
        self.b_g2 = np.zeros((V, G2_WORDS), dtype=np.uint64)
        self.ic_g1 = np.zeros((max(V - num_public - 1, 0), G1_WORDS), dtype=np.uint64)
        self.h_g1 = np.zeros((n, G1_WORDS), dtype=np.uint64)
        self.num_public = num_public
        self.qap = qap
        self.s = _PK()

    def _bind(self):
        s = self.s
        s.a_g1, s.a_len = self.a_g1.ctypes.data, len(self.a_g1)
        s.b_g1, s.b_len = self.b_g1.ctypes.data, len(self.b_g1)
        s.b_g2, s.b2_len = self.b_g2.ctypes.data, len(self.b_g2)
        s.ic_g1, s.ic_len = (self.ic_g1.ctypes.data if len(self.ic_g1) else None), len(self.ic_g1)
        s.h_g1, s.h_len = self.h_g1.ctypes.data, len(self.h_g1)
        s.num_public = self.num_public
        return s

    def point(self, name):
        """alpha_g1 / beta_g1 / delta_g1 / beta_g2 / delta_g2 as uint64 words."""
        return np.array(getattr(self.s, name).w, dtype=np.uint64)

    def upload(self, ctx, shard=0, nshards=1):
        return DeviceProvingKey.upload(ctx, self, shard, nshards)


class VerificationKey:
    """crates/groth16-setup/src/lib.rs:56-69"""

    def __init__(self, num_public):
        self.ic_g1 = np.zeros((num_public + 1, G1_WORDS), dtype=np.uint64)
        self.num_public = num_public
        self.s = _VK()
        self.s.ic_g1 = self.ic_g1.ctypes.data
        self.s.ic_len = num_public + 1
        self.s.num_public = num_public

    @classmethod
    def from_points(cls, alpha_g1, beta_g2, gamma_g2, delta_g2, ic_g1):
        """Build from canonical affine words (13 per G1, 25 per G2 point)."""
        ic = np.asarray(ic_g1, dtype=np.uint64).reshape(-1, G1_WORDS)
        vk = cls(len(ic) - 1)
        vk.ic_g1[:] = ic
        for name, words in (("alpha_g1", alpha_g1), ("beta_g2", beta_g2), ("gamma_g2", gamma_g2),
                            ("delta_g2", delta_g2)):
            field = getattr(vk.s, name)
            for i, w in enumerate(np.asarray(words, dtype=np.uint64).reshape(-1)):
                field.w[i] = int(w)
        return vk

    def point(self, name):
        return np.array(getattr(self.s, name).w, dtype=np.uint64)


class DeviceProvingKey:
    """A proving key resident in HBM (zk_pk_dev)."""

    def __init__(self, ctx, handle, qap):
        self.ctx, self._h, self.qap = ctx, handle, qap

    @classmethod
    def upload(cls, ctx, pk, shard=0, nshards=1):
        h = C.c_void_p()
        s = pk._bind()
        if nshards == 1:
            rc = lib().zk_pk_upload(C.c_void_p(ctx._h), C.byref(s), C.byref(pk.qap.csr.s), C.byref(h))
        else:
            rc = lib().zk_pk_upload_shard(C.c_void_p(ctx._h), C.byref(s), C.byref(pk.qap.csr.s),
                                          C.c_uint32(shard), C.c_uint32(nshards), C.byref(h))
        _check(rc, ctx, "zk_pk_upload")
        return cls(ctx, h.value, pk.qap)

    def witness_ranges(self):
        """zk_groth16_witness_ranges: (k, 2) array of the [lo, hi) witness
        index ranges this shard reads on its ctx."""
        n = C.c_size_t()
        _check(lib().zk_groth16_witness_ranges(C.c_void_p(self.ctx._h), C.c_void_p(self._h), None, C.c_size_t(0),
                                               C.byref(n)), self.ctx, "zk_groth16_witness_ranges")
        out = np.zeros((max(n.value, 1), 2), dtype=np.uint64)
        _check(lib().zk_groth16_witness_ranges(C.c_void_p(self.ctx._h), C.c_void_p(self._h), _p(out),
                                               C.c_size_t(n.value), C.byref(n)), self.ctx, "zk_groth16_witness_ranges")
        return out[:n.value]

    def test_info(self):
        """zk_test_pk_info (test library): (win, win_c, shard, nshards)."""
        v = [C.c_uint32() for _ in range(4)]
        _check(test_lib().zk_test_pk_info(C.c_void_p(self._h), *[C.byref(x) for x in v]), None, "zk_test_pk_info")
        return tuple(x.value for x in v)

    def test_bases(self, slot, window=0):
        """zk_test_pk_bases (test library): (variable / coefficient index per
        compacted base, canonical words of the compacted bases + extras,
        number of extras) of one MSM slot's window copy."""
        cnt, nex = C.c_size_t(), C.c_size_t()
        _check(test_lib().zk_test_pk_bases(C.c_void_p(self.ctx._h), C.c_void_p(self._h), C.c_int(slot),
                                           C.c_int(window), None, None, C.c_size_t(0), C.byref(cnt), C.byref(nex)),
               self.ctx, "zk_test_pk_bases")
        tot = cnt.value + nex.value
        words = G2_WORDS if slot == 1 else G1_WORDS
        idx = np.zeros(max(cnt.value, 1), dtype=np.uint32)
        out = np.zeros((max(tot, 1), words), dtype=np.uint64)
        _check(test_lib().zk_test_pk_bases(C.c_void_p(self.ctx._h), C.c_void_p(self._h), C.c_int(slot),
                                           C.c_int(window), _p(idx), _p(out), C.c_size_t(max(tot, 1)),
                                           C.byref(cnt), C.byref(nex)), self.ctx, "zk_test_pk_bases")
        return idx[:cnt.value], out[:tot], nex.value

    def witness_slice(self, assignment):
        """This shard's part of a full witness (rows of every witness range, in order)."""
        a = np.asarray(assignment, dtype=np.uint64).reshape(-1, 4)
        rs = self.witness_ranges()
        return np.ascontiguousarray(np.concatenate([a[int(lo):int(hi)] for lo, hi in rs]) if len(rs)
                                    else np.zeros((0, 4), dtype=np.uint64))

    def free(self):
        if getattr(self, "_h", None):
            lib().zk_pk_free(C.c_void_p(self._h))
            self._h = None

    def __del__(self):
        self.free()


class CRS:
    """crates/groth16-setup/src/lib.rs:72-78, 139-278 (GPU setup)."""

    def __init__(self, pk, vk):
        self.pk, self.vk = pk, vk

    @classmethod
    def generate_from_qap(cls, ctx, qap, params, num_public):
        params.validate()
        if num_public >= qap.num_variables:
            raise SetupError("Number of public inputs must be less than total variables")
        pk = ProvingKey(qap.num_variables, qap.domain_size, num_public, qap)
        vk = VerificationKey(num_public)
        s = pk._bind()
        rc = lib().zk_groth16_setup(C.c_void_p(ctx._h), C.byref(qap.csr.s), C.byref(params._c()),
                                    C.c_uint64(num_public), C.byref(s), C.byref(vk.s))
        _check(rc, ctx, "zk_groth16_setup")
        return cls(pk, vk)

    @classmethod
    def generate_random(cls, ctx, qap, num_public, rng):
        return cls.generate_from_qap(ctx, qap, SetupParams.random(rng), num_public)

    @staticmethod
    def generate_device(ctx, qap, params, num_public, shard=0, nshards=1):
        """Setup straight into HBM (no host round trip) -> DeviceProvingKey."""
        h = C.c_void_p()
        if nshards == 1:
            rc = lib().zk_groth16_setup_dev(C.c_void_p(ctx._h), C.byref(qap.csr.s), C.byref(params._c()),
                                            C.c_uint64(num_public), C.byref(h), None)
        else:
            rc = lib().zk_groth16_setup_dev_shard(C.c_void_p(ctx._h), C.byref(qap.csr.s),
                                                  C.byref(params._c()), C.c_uint64(num_public),
                                                  C.c_uint32(shard), C.c_uint32(nshards), C.byref(h))
        _check(rc, ctx, "zk_groth16_setup_dev")
        return DeviceProvingKey(ctx, h.value, qap)


# -------------------------------------------------------------- prove ----
class Witness:
    """crates/groth16-core/src/lib.rs:40-131"""

    def __init__(self, assignment, num_public):
        a = assignment
        if not isinstance(a, np.ndarray):
            a = fr_array(a)
        a = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 4)
        if not fr_rows_canonical(a):
            raise ValueError("assignment holds a value >= r (not a canonical Fr)")
        if num_public >= len(a):
            raise InvalidWitness("Number of public inputs must be less than total assignment length")
        if len(a) == 0 or not (a[0, 0] == 1 and not a[0, 1:].any()):
            raise InvalidWitness("First element of assignment must be 1 (constant)")
        self.assignment = a
        self.num_public = num_public

    def public_inputs(self):
        """core:101-104"""
        return self.assignment[1:self.num_public + 1]

    def private_inputs(self):
        """core:106-109"""
        return self.assignment[self.num_public + 1:]


_R_LIMBS = np.array([(R >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)


def fr_rows_canonical(a):
    """Every row (4 little-endian u64 limbs) < r, vectorised."""
    a = np.asarray(a, dtype=np.uint64).reshape(-1, 4)
    lt = np.zeros(len(a), dtype=bool)
    eq = np.ones(len(a), dtype=bool)
    for i in (3, 2, 1, 0):
        lt |= eq & (a[:, i] < _R_LIMBS[i])
        eq &= a[:, i] == _R_LIMBS[i]
    return bool(lt.all())


class Proof:
    """crates/groth16-core/src/lib.rs:27-36 (a: G1, b: G2, c: G1)."""

    def __init__(self, words):
        self.words = np.asarray(words, dtype=np.uint64).reshape(-1)
        self.a = self.words[:G1_WORDS]
        self.b = self.words[G1_WORDS:G1_WORDS + G2_WORDS]
        self.c = self.words[G1_WORDS + G2_WORDS:]

    @classmethod
    def _from_c(cls, p):
        return cls(list(p.a.w) + list(p.b.w) + list(p.c.w))

    def _c(self):
        p = _Proof()
        for i in range(G1_WORDS):
            p.a.w[i] = int(self.a[i])
            p.c.w[i] = int(self.c[i])
        for i in range(G2_WORDS):
            p.b.w[i] = int(self.b[i])
        return p

    def serialize_compressed(self):
        """ark CanonicalSerialize (compressed) of Proof: 48 + 96 + 48 bytes."""
        out = (C.c_uint8 * 192)()
        _check(lib().zk_proof_serialize_compressed(C.byref(self._c()), out), None, "serialize")
        return bytes(out)

    @classmethod
    def deserialize_compressed(cls, data):
        """ark CanonicalDeserialize (compressed, validated); ValueError on bad bytes."""
        data = bytes(data)
        if len(data) != 192:
            raise ValueError("a compressed Proof is 192 bytes")
        buf = (C.c_uint8 * 192).from_buffer_copy(data)
        out = _Proof()
        _check(lib().zk_proof_deserialize_compressed(buf, C.byref(out)), None, "deserialize")
        return cls._from_c(out)

    def __eq__(self, other):
        return isinstance(other, Proof) and np.array_equal(self.words, other.words)


class Prover:
    """Prover::prove (crates/groth16-core/src/lib.rs:139-272).  `r` and `s`
    are the two Fr::rand draws of core:152-153; pass them explicitly (or an
    `rng` callable returning Fr ints, drawn r then s)."""

    @staticmethod
    def prove(dpk, witness, r=None, s=None, rng=None):
        if r is None or s is None:
            if rng is None:
                raise ValueError("pass r and s, or an rng")
            r, s = rng(), rng()
        ctx = dpk.ctx
        out = _Proof()
        z = witness.assignment
        rc = lib().zk_groth16_prove(C.c_void_p(ctx._h), C.c_void_p(dpk._h), _p(z), C.c_size_t(len(z)),
                                    C.c_size_t(witness.num_public), C.byref(_fr(r)), C.byref(_fr(s)),
                                    C.byref(out))
        _check(rc, ctx, "zk_groth16_prove")
        return Proof._from_c(out)

    @staticmethod
    def prove_device(dpk, d_z_ptr, zlen, num_public, r, s):
        """z already in HBM (canonical zk_fr array at device pointer d_z_ptr)."""
        ctx = dpk.ctx
        out = _Proof()
        rc = lib().zk_groth16_prove_dev(C.c_void_p(ctx._h), C.c_void_p(dpk._h), C.c_void_p(d_z_ptr),
                                        C.c_size_t(zlen), C.c_size_t(num_public), C.byref(_fr(r)),
                                        C.byref(_fr(s)), C.byref(out))
        _check(rc, ctx, "zk_groth16_prove_dev")
        return Proof._from_c(out)

    @staticmethod
    def prove_partial(dpk, d_z_ptr, zlen, num_public, r, s):
        """This GPU's shard of the MSMs -> opaque bytes for the all-gather."""
        ctx = dpk.ctx
        buf = (C.c_uint8 * PARTIAL_BYTES)()
        rc = lib().zk_groth16_prove_partial(C.c_void_p(ctx._h), C.c_void_p(dpk._h), C.c_void_p(d_z_ptr),
                                            C.c_size_t(zlen), C.c_size_t(num_public), C.byref(_fr(r)),
                                            C.byref(_fr(s)), buf)
        _check(rc, ctx, "zk_groth16_prove_partial")
        return bytes(buf)

    @staticmethod
    def prove_partial_host(dpk, z_slice, zlen, num_public, r, s):
        """This GPU's shard of the proof from a HOST witness slice (only the
        entries of dpk.witness_ranges(), concatenated: dpk.witness_slice(z));
        zlen = length of the whole witness."""
        ctx = dpk.ctx
        zs = np.ascontiguousarray(z_slice, dtype=np.uint64).reshape(-1, 4)
        buf = (C.c_uint8 * PARTIAL_BYTES)()
        rc = lib().zk_groth16_prove_partial_host(C.c_void_p(ctx._h), C.c_void_p(dpk._h), _p(zs) if len(zs) else None,
                                                 C.c_size_t(len(zs)), C.c_size_t(zlen), C.c_size_t(num_public),
                                                 C.byref(_fr(r)), C.byref(_fr(s)), buf)
        _check(rc, ctx, "zk_groth16_prove_partial_host")
        return bytes(buf)

    @staticmethod
    def prove_virtual_shards(dpks, d_z_ptr, zlen, num_public, r, s):
        """Diagnostic: the distributed quotient + sharded MSMs of len(dpks)
        virtual ranks on one device (zk_test_prove_virtual_shards)."""
        ctx = dpks[0].ctx
        arr = (C.c_void_p * len(dpks))(*[C.c_void_p(d._h) for d in dpks])
        out = _Proof()
        rc = test_lib().zk_test_prove_virtual_shards(C.c_void_p(ctx._h), arr, C.c_uint32(len(dpks)),
                                                C.c_void_p(d_z_ptr), C.c_size_t(zlen), C.c_size_t(num_public),
                                                C.byref(_fr(r)), C.byref(_fr(s)), C.byref(out))
        _check(rc, ctx, "zk_test_prove_virtual_shards")
        return Proof._from_c(out)

    @staticmethod
    def combine(partials, r, s):
        k = len(partials)
        arr = (C.c_uint8 * (PARTIAL_BYTES * k)).from_buffer_copy(b"".join(partials))
        out = _Proof()
        rc = lib().zk_groth16_prove_combine(arr, C.c_size_t(k), C.byref(_fr(r)), C.byref(_fr(s)),
                                            C.byref(out))
        _check(rc, None, "zk_groth16_prove_combine")
        return Proof._from_c(out)


class TorchExchange:
    """Host-staged exchange over a torch.distributed process group (CPU
    tensors: gloo), for Context.attach_exchange: the distributed quotient's
    three all-to-alls as all_to_all_single, the status agreement as a MAX
    all-reduce.  abort() tears the group down (the default group unless one
    is given), so peers blocked in a transfer with this rank fail instead of
    waiting out the group's timeout."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group, self.dead = dist, group, False

    def all_to_all(self, send_ptr, recv_ptr, chunk_bytes):
        import torch
        if self.dead:
            raise ExchangeError("TorchExchange: aborted")
        nbytes = chunk_bytes * self.dist.get_world_size(self.group)
        send = torch.frombuffer((C.c_uint8 * nbytes).from_address(send_ptr), dtype=torch.uint8)
        recv = torch.frombuffer((C.c_uint8 * nbytes).from_address(recv_ptr), dtype=torch.uint8)
        self.dist.all_to_all_single(recv, send, group=self.group)

    def all_reduce_max(self, value):
        import torch
        if self.dead:
            raise ExchangeError("TorchExchange: aborted")
        t = torch.tensor([value], dtype=torch.int64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def abort(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group(self.group)
        self.group, self.dead = None, True   # the last reference: the group's connections close with it


# ------------------------------------------------------------- verify ----
def _fr_rows(values):
    a = values if isinstance(values, np.ndarray) else fr_array(values)
    return np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 4)


def pairing_product_is_one(g1_points, g2_points):
    """prod e(P_i, Q_i) == 1 (Bls12_381::multi_pairing(..).is_zero(), core:352)."""
    a = np.ascontiguousarray(g1_points, dtype=np.uint64).reshape(-1, G1_WORDS)
    b = np.ascontiguousarray(g2_points, dtype=np.uint64).reshape(-1, G2_WORDS)
    if len(a) != len(b):
        raise ValueError("as many G1 as G2 points")
    out = C.c_int(0)
    _check(lib().zk_pairing_product_is_one(_p(a), _p(b), C.c_size_t(len(a)), C.byref(out)), None, "pairing")
    return bool(out.value)


class Verifier:
    """Verifier::verify (crates/groth16-core/src/lib.rs:308-355), on the host."""

    @staticmethod
    def verify(vk, proof, public_inputs):
        inp = _fr_rows(public_inputs)
        valid = C.c_int(0)
        rc = lib().zk_groth16_verify(C.byref(vk.s), C.byref(proof._c()), _p(inp) if len(inp) else None,
                                     C.c_size_t(len(inp)), C.byref(valid))
        _check(rc, None, "zk_groth16_verify")
        return bool(valid.value)


class BatchVerifier:
    """BatchVerifier::verify_batch (core:360-432).  The reference draws one
    Fr::rand coefficient per proof; pass them as `coeffs` (or an `rng`
    callable returning Fr ints)."""

    @staticmethod
    def verify_batch(vk, proofs_and_inputs, coeffs=None, rng=None):
        k = len(proofs_and_inputs)
        if coeffs is None:
            if k and rng is None:
                raise ValueError("pass coeffs, or an rng")
            coeffs = [rng() for _ in range(k)]
        proofs = (_Proof * max(k, 1))()
        rows = [_fr_rows(inp) for _, inp in proofs_and_inputs]
        ptrs = (C.c_void_p * max(k, 1))(*[C.c_void_p(r.ctypes.data) for r in rows])
        lens = (C.c_size_t * max(k, 1))(*[len(r) for r in rows])
        for i, (pr, _) in enumerate(proofs_and_inputs):
            proofs[i] = pr._c()
        co = _fr_rows(coeffs) if k else np.zeros((1, 4), dtype=np.uint64)
        valid = C.c_int(0)
        rc = lib().zk_groth16_verify_batch(C.byref(vk.s), proofs, ptrs, lens, C.c_size_t(k), _p(co),
                                           C.byref(valid))
        _check(rc, None, "zk_groth16_verify_batch")
        return bool(valid.value)


# ------------------------------------------------------- file formats ----
# Binary key files (the reference's CLI writes JSON placeholders instead:
# crates/groth16-cli/src/lib.rs:157-219).  Little-endian, canonical affine
# words exactly as they cross the C ABI (13 u64 per G1, 25 per G2), so a
# 2^24-constraint key (~24 GB) streams through numpy without conversion.
#   proving key:  b"ZKAMDPK1", u64 x 9 (V, n, num_public, num_constraints,
#                 a_len, b_len, b2_len, ic_len, h_len), alpha_g1, beta_g1,
#                 delta_g1, beta_g2, delta_g2, the five base vectors, then the
#                 QAP (setup:51) as CSR: per matrix u64 nnz, u64 has_val,
#                 rowptr[nc+1] u64, col[nnz] u32 (+4 pad bytes if nnz odd),
#                 val[nnz x 4] u64 when has_val
#   verification key: b"ZKAMDVK1", u64 num_public, ic_len, alpha_g1,
#                 beta_g2, gamma_g2, delta_g2, ic_g1[ic_len]
#   proof:        the 192-byte ark compressed encoding (Proof::serialize_compressed)
_PK_MAGIC, _VK_MAGIC = b"ZKAMDPK1", b"ZKAMDVK1"


def _u64s(f, k):
    a = np.fromfile(f, dtype="<u8", count=k)
    if len(a) != k:
        raise ValueError("truncated key file")
    return a


def save_proving_key(pk, path):
    with open(path, "wb") as f:
        f.write(_PK_MAGIC)
        csr = pk.qap.csr
        np.array([pk.qap.num_variables, pk.qap.domain_size, pk.num_public, csr.num_constraints,
                  len(pk.a_g1), len(pk.b_g1), len(pk.b_g2), len(pk.ic_g1), len(pk.h_g1)], dtype="<u8").tofile(f)
        for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
            pk.point(nm).astype("<u8").tofile(f)
        for arr in (pk.a_g1, pk.b_g1, pk.b_g2, pk.ic_g1, pk.h_g1):
            np.ascontiguousarray(arr, dtype="<u8").tofile(f)
        for rp, col, val in csr.mats:
            nnz = len(col)
            np.array([nnz, val is not None], dtype="<u8").tofile(f)
            np.ascontiguousarray(rp, dtype="<u8").tofile(f)
            np.ascontiguousarray(col, dtype="<u4").tofile(f)
            if nnz & 1:
                f.write(b"\0" * 4)
            if val is not None:
                np.ascontiguousarray(val, dtype="<u8").tofile(f)


def load_proving_key(path):
    with open(path, "rb") as f:
        if f.read(8) != _PK_MAGIC:
            raise ValueError(f"{path}: not a proving key file")
        V, n, npub, nc, la, lb, lb2, lic, lh = (int(x) for x in _u64s(f, 9))
        pts = [_u64s(f, G1_WORDS) for _ in range(3)] + [_u64s(f, G2_WORDS) for _ in range(2)]
        arrs = [_u64s(f, k * w).reshape(k, w) for k, w in
                ((la, G1_WORDS), (lb, G1_WORDS), (lb2, G2_WORDS), (lic, G1_WORDS), (lh, G1_WORDS))]
        mats = []
        for _ in range(3):
            nnz, has_val = (int(x) for x in _u64s(f, 2))
            rp = _u64s(f, nc + 1).astype(np.uint64)
            col = np.fromfile(f, dtype="<u4", count=nnz).astype(np.uint32)
            if len(col) != nnz:
                raise ValueError("truncated key file")
            if nnz & 1:
                f.read(4)
            val = _u64s(f, 4 * nnz).reshape(nnz, 4).astype(np.uint64) if has_val else None
            mats.append((rp, col, val))
    qap = QAP(CSRMatrices(nc, V, mats))
    if qap.domain_size != n:
        raise ValueError("key domain does not match its constraint system")
    pk = ProvingKey(0, 0, npub, qap)
    pk.a_g1, pk.b_g1, pk.b_g2, pk.ic_g1, pk.h_g1 = (np.ascontiguousarray(a, dtype=np.uint64) for a in arrs)
    for nm, words in zip(("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"), pts):
        field = getattr(pk.s, nm)
        for i, w in enumerate(words):
            field.w[i] = int(w)
    return pk


def save_verification_key(vk, path):
    with open(path, "wb") as f:
        f.write(_VK_MAGIC)
        np.array([vk.num_public, len(vk.ic_g1)], dtype="<u8").tofile(f)
        for nm in ("alpha_g1", "beta_g2", "gamma_g2", "delta_g2"):
            vk.point(nm).astype("<u8").tofile(f)
        np.ascontiguousarray(vk.ic_g1, dtype="<u8").tofile(f)


def load_verification_key(path):
    with open(path, "rb") as f:
        if f.read(8) != _VK_MAGIC:
            raise ValueError(f"{path}: not a verification key file")
        npub, lic = (int(x) for x in _u64s(f, 2))
        pts = [_u64s(f, G1_WORDS)] + [_u64s(f, G2_WORDS) for _ in range(3)]
        ic = _u64s(f, lic * G1_WORDS).reshape(lic, G1_WORDS)
    vk = VerificationKey.from_points(*pts, ic)
    vk.num_public = vk.s.num_public = npub
    return vk


# The reference CLI's serde JSON shapes (crates/groth16-cli/src/lib.rs:16-51):
# coefficients and values are hex strings ("0x" optional).
def _hex(v):
    return int(v, 16) % R


def r1cs_from_circuit_json(doc):
    """CircuitDescription {num_variables (without the constant), num_public,
    constraints: [{a, b, c: [[var, coeff_hex], ...]}]} -> R1CS."""
    cs = R1CS(int(doc["num_public"]))
    while cs.num_variables < int(doc["num_variables"]) + 1:
        cs.allocate_variable()
    for con in doc["constraints"]:
        lcs = [LinearCombination({int(v): _hex(c) for v, c in con[m]}) for m in "abc"]
        cs.enforce_multiplication(*lcs)
    return cs


def witness_from_json(doc):
    """WitnessData {assignment: [hex], num_public} -> Witness."""
    return Witness([_hex(x) for x in doc["assignment"]], int(doc["num_public"]))


def public_inputs_from_json(doc):
    """PublicInputs {inputs: [hex]} -> list of ints."""
    return [_hex(x) for x in doc["inputs"]]
