"""pyref -- independent pure-Python big-integer restatement of the reference
Groth16 path, following the reference's LITERAL (dense, O(V*n)) algorithm.

TEST INFRASTRUCTURE ONLY: used in this container to generate the golden
fixtures under tests/golden/ (tests/golden/gen_golden.py) and by CPU tests as
a second, independent checker of oracle/zk_oracle.c.  Never imported by the
product package, bench.py's timed region or the GPU path.

It shares no code with zk_oracle.c: affine-coordinate group law with explicit
inversions (instead of Jacobian), naive double-and-add MSM (instead of the ark
Pippenger), dense per-variable interpolation, Horner evaluation and schoolbook
polynomial arithmetic (instead of the sparse Lagrange / coset-FFT quotient).

Restated reference items (file:line under /root/reference):
  R1CS / LinearCombination      crates/groth16-r1cs/src/lib.rs:16-358
  QAP::from_r1cs                crates/groth16-qap/src/lib.rs:95-187
  QAP::evaluate_at              crates/groth16-qap/src/lib.rs:190-220
  compute_quotient_polynomial   crates/groth16-qap/src/lib.rs:225-271
  verify_evaluation / degree    crates/groth16-qap/src/lib.rs:274-294
  CRS::generate_from_qap        crates/groth16-setup/src/lib.rs:141-268
  Witness::new / validate       crates/groth16-core/src/lib.rs:81-131
  Prover::prove                 crates/groth16-core/src/lib.rs:139-272
Upstream arkworks 0.4 semantics (not vendored; published algorithm):
  Radix2EvaluationDomain (group_gen = 7^((r-1)/2^32) ^ (2^(32-log n))),
  lo64 = Fr::from(x.into_bigint().as_ref()[0]), zcash compressed encoding.
Parity status: partially pinned (see oracle/zk_oracle.h header).
"""

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
FR_GENERATOR = 7
TWO_ADICITY = 32

G1_GEN = (
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
)
G2_GEN = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)
INF = None  # point at infinity


def lo64(x):
    """Fr::from(x.into_bigint().as_ref()[0])  (core:156-161 and friends)."""
    return x & 0xFFFFFFFFFFFFFFFF


def fr_inv(a):
    return pow(a % R, R - 2, R)


def root_of_unity(n):
    """ark get_root_of_unity for a power-of-two n."""
    log_n = n.bit_length() - 1
    assert 1 << log_n == n and log_n <= TWO_ADICITY
    w = pow(FR_GENERATOR, (R - 1) >> TWO_ADICITY, R)
    return pow(w, 1 << (TWO_ADICITY - log_n), R)


# ---------------------------------------------------------------- Fq2 ----
class Fq2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0, c1=0):
        self.c0 = c0 % P
        self.c1 = c1 % P

    def __add__(self, o):
        o = _f2(o)
        return Fq2(self.c0 + o.c0, self.c1 + o.c1)

    __radd__ = __add__

    def __sub__(self, o):
        o = _f2(o)
        return Fq2(self.c0 - o.c0, self.c1 - o.c1)

    def __rsub__(self, o):
        return _f2(o) - self

    def __neg__(self):
        return Fq2(-self.c0, -self.c1)

    def __mul__(self, o):
        o = _f2(o)
        return Fq2(self.c0 * o.c0 - self.c1 * o.c1, self.c0 * o.c1 + self.c1 * o.c0)

    __rmul__ = __mul__

    def inv(self):
        n = pow(self.c0 * self.c0 + self.c1 * self.c1, P - 2, P)
        return Fq2(self.c0 * n, -self.c1 * n)

    def __eq__(self, o):
        o = _f2(o)
        return self.c0 == o.c0 and self.c1 == o.c1

    def __hash__(self):
        return hash((self.c0, self.c1))

    def is_zero(self):
        return self.c0 == 0 and self.c1 == 0


def _f2(x):
    return x if isinstance(x, Fq2) else Fq2(x)


class Fq1:
    """Prime field Fq with the same interface as Fq2 (for the shared group law)."""
    __slots__ = ("v",)

    def __init__(self, v):
        self.v = v % P

    def __add__(self, o):
        return Fq1(self.v + _v(o))

    __radd__ = __add__

    def __sub__(self, o):
        return Fq1(self.v - _v(o))

    def __rsub__(self, o):
        return Fq1(_v(o) - self.v)

    def __neg__(self):
        return Fq1(-self.v)

    def __mul__(self, o):
        return Fq1(self.v * _v(o))

    __rmul__ = __mul__

    def inv(self):
        return Fq1(pow(self.v, P - 2, P))

    def __eq__(self, o):
        return self.v == _v(o)

    def __hash__(self):
        return hash(self.v)

    def is_zero(self):
        return self.v == 0


def _v(x):
    return x.v if isinstance(x, Fq1) else x


# ------------------------------------------------------- affine group ----
class Curve:
    def __init__(self, b, gen):
        self.b = b
        self.gen = gen

    def on_curve(self, p):
        if p is INF:
            return True
        x, y = p
        return y * y == x * x * x + self.b

    def neg(self, p):
        return INF if p is INF else (p[0], -p[1])

    def add(self, p, q):
        if p is INF:
            return q
        if q is INF:
            return p
        x1, y1 = p
        x2, y2 = q
        if x1 == x2:
            if (y1 + y2).is_zero():
                return INF
            lam = (x1 * x1 * 3) * (y1 * 2).inv()
        else:
            lam = (y2 - y1) * (x2 - x1).inv()
        x3 = lam * lam - x1 - x2
        return (x3, lam * (x1 - x3) - y1)

    def mul(self, p, k):
        acc = INF
        for bit in bin(k)[2:] if k > 0 else "":
            acc = self.add(acc, acc)
            if bit == "1":
                acc = self.add(acc, p)
        return acc

    def msm(self, pairs):
        """Sum k_i P_i; the result is a unique group element, so the naive
        evaluation equals ark's Pippenger bit for bit after normalisation."""
        acc = INF
        for k, pt in pairs:
            acc = self.add(acc, self.mul(pt, k))
        return acc


G1 = Curve(Fq1(4), (Fq1(G1_GEN[0]), Fq1(G1_GEN[1])))
G2 = Curve(Fq2(4, 4), (Fq2(*G2_GEN[0]), Fq2(*G2_GEN[1])))


# ------------------------------------------------------------- R1CS ----
class R1CS:
    """crates/groth16-r1cs/src/lib.rs:229-358 (builder subset on the path)."""

    def __init__(self, num_public_inputs=0):
        self.constraints = []               # (a, b, c) dicts var -> coeff
        self.num_public_inputs = num_public_inputs
        self.num_variables = 1 + num_public_inputs

    def allocate_variable(self):
        v = self.num_variables
        self.num_variables += 1
        return v

    def enforce_multiplication(self, a, b, c):
        self.constraints.append(({k: v % R for k, v in a.items() if v % R},
                                 {k: v % R for k, v in b.items() if v % R},
                                 {k: v % R for k, v in c.items() if v % R}))

    def num_constraints(self):
        return len(self.constraints)


def synthetic_r1cs(n):
    """crates/groth16-cli/src/lib.rs:57-70: n x (x*y=z), R1CS::new(0)."""
    cs = R1CS(0)
    for _ in range(n):
        x, y, z = cs.allocate_variable(), cs.allocate_variable(), cs.allocate_variable()
        cs.enforce_multiplication({x: 1}, {y: 1}, {z: 1})
    return cs


# -------------------------------------------------------------- FFT ----
def dft(vals, n, inverse=False):
    """Naive O(n^2) DFT over the size-n domain (ark fft / ifft semantics)."""
    w = root_of_unity(n)
    if inverse:
        w = fr_inv(w)
    vals = list(vals) + [0] * (n - len(vals))
    out = []
    for k in range(n):
        wk = pow(w, k, R)
        acc, p = 0, 1
        for j in range(n):
            acc = (acc + vals[j] * p) % R
            p = p * wk % R
        out.append(acc)
    if inverse:
        ninv = fr_inv(n)
        out = [x * ninv % R for x in out]
    return out


def trim(coeffs):
    c = list(coeffs)
    while c and c[-1] == 0:
        c.pop()
    return c


def poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R
    return acc


def poly_mul(a, b):
    if not a or not b:
        return []
    out = [0] * (len(a) + len(b) - 1)
    for i, x in enumerate(a):
        if x:
            for j, y in enumerate(b):
                out[i + j] = (out[i + j] + x * y) % R
    return trim(out)


# -------------------------------------------------------------- QAP ----
class QAPError(Exception):
    pass


class QAP:
    """crates/groth16-qap/src/lib.rs:31-46, literal dense form."""

    def __init__(self, cs):
        nc, V = cs.num_constraints(), cs.num_variables
        n = 1
        while n < nc:
            n <<= 1
        self.n = n
        self.omega = root_of_unity(n)
        self.num_variables, self.num_constraints = V, nc
        dense = [[[0] * V for _ in range(nc)] for _ in range(3)]
        for ci, abc in enumerate(cs.constraints):
            for m in range(3):
                for var, coeff in abc[m].items():
                    if var < V:                       # qap:122
                        dense[m][ci][var] = coeff
        self.polys = [[], [], []]
        for m in range(3):
            for var in range(V):
                col = [dense[m][ci][var] for ci in range(nc)]
                self.polys[m].append(trim(dft(col, n, inverse=True)))

    def degree(self):
        """qap:285-294: max poly degree vs Z = x^n - 1 -> n."""
        d = 0
        for m in range(3):
            for p in self.polys[m]:
                d = max(d, max(len(p) - 1, 0))
        return max(d, self.n)

    def evaluate_at(self, x, z):
        if len(z) != self.num_variables:
            raise QAPError("dimension mismatch")
        vals = [0, 0, 0]
        for m in range(3):
            for i, zi in enumerate(z):
                vals[m] = (vals[m] + zi * poly_eval(self.polys[m][i], x)) % R
        return vals

    def verify_evaluation(self, vals):
        a, b, c = vals
        return a * b % R == c

    def compute_quotient_polynomial(self, z):
        if len(z) != self.num_variables:
            raise QAPError("dimension mismatch")
        acc = [[0] * self.n for _ in range(3)]
        for m in range(3):
            for i, zi in enumerate(z):
                if zi % R == 0:
                    continue
                for k, c in enumerate(self.polys[m][i]):
                    acc[m][k] = (acc[m][k] + c * zi) % R
        a, b, c = (trim(x) for x in acc)
        num = poly_mul(a, b)
        num = num + [0] * max(0, len(c) - len(num))
        for k, x in enumerate(c):
            num[k] = (num[k] - x) % R
        num = trim(num)
        # divide by x^n - 1
        n = self.n
        if len(num) <= n:
            q, rem = [], num
        else:
            rem = list(num)
            q = [0] * (len(rem) - n)
            for i in range(len(rem) - 1, n - 1, -1):
                q[i - n] = rem[i]
                rem[i - n] = (rem[i - n] + rem[i]) % R
                rem[i] = 0
            rem = trim(rem)
        if trim(rem):
            raise QAPError("PolynomialDivisionFailed")
        return trim(q)


# ------------------------------------------------------------ setup ----
class SetupError(Exception):
    pass


def generate_from_qap(qap, params, num_public):
    """crates/groth16-setup/src/lib.rs:141-268.  params = (alpha, beta,
    gamma, delta, tau) full Fr values; returns (pk, vk) dicts of affine points."""
    alpha, beta, gamma, delta, tau = (x % R for x in params)
    if 0 in (alpha, beta, gamma, delta):
        raise SetupError("Setup parameters must be non-zero")
    V = qap.num_variables
    if num_public >= V:
        raise SetupError("num_public")
    al, be, ga, de, ta = (lo64(x) for x in (alpha, beta, gamma, delta, tau))
    if de == 0 or ga == 0:
        raise SetupError("truncated delta/gamma not invertible (reference panics)")
    g1, g2 = G1.gen, G2.gen
    av = [poly_eval(p, ta) for p in qap.polys[0]]
    bv = [poly_eval(p, ta) for p in qap.polys[1]]
    cv = [poly_eval(p, ta) for p in qap.polys[2]]
    dinv, ginv = fr_inv(de), fr_inv(ga)
    pk = {
        "alpha_g1": G1.mul(g1, alpha), "beta_g1": G1.mul(g1, beta),
        "beta_g2": G2.mul(g2, beta), "delta_g1": G1.mul(g1, delta),
        "delta_g2": G2.mul(g2, delta),
        "a_g1": [G1.mul(g1, lo64(a)) for a in av],
        "b_g1": [G1.mul(g1, lo64(b)) for b in bv],
        "b_g2": [G2.mul(g2, lo64(b)) for b in bv],
        "ic_g1": [G1.mul(g1, lo64((be * av[i] + al * bv[i] + cv[i]) * dinv % R))
                  for i in range(num_public + 1, V)],
        "h_g1": [G1.mul(g1, lo64(pow(ta, i, R) * dinv % R)) for i in range(qap.degree())],
        "num_public": num_public,
    }
    vk = {
        "alpha_g1": pk["alpha_g1"], "beta_g2": pk["beta_g2"],
        "gamma_g2": G2.mul(g2, gamma), "delta_g2": pk["delta_g2"],
        "ic_g1": [G1.mul(g1, lo64((be * av[i] + al * bv[i] + cv[i]) * ginv % R))
                  for i in range(0, num_public + 1)],
        "num_public": num_public,
    }
    return pk, vk


# ------------------------------------------------------------ prove ----
class GrothError(Exception):
    pass


def prove(pk, qap, z, num_public, r, s):
    """crates/groth16-core/src/lib.rs:81-131 (Witness) + 139-272 (prove)."""
    z = [x % R for x in z]
    if num_public >= len(z) or z[0] != 1:
        raise GrothError("InvalidWitness")
    if len(z) != qap.num_variables:
        raise GrothError("InvalidWitness")
    if not qap.verify_evaluation(qap.evaluate_at(qap.omega, z)):
        raise GrothError("InvalidWitness")
    w = [lo64(x) for x in z]
    a_terms = [(1, pk["alpha_g1"])] + [(wi, pk["a_g1"][i]) for i, wi in enumerate(w)
                                       if wi and i < len(pk["a_g1"])] + [(r, pk["delta_g1"])]
    pi_a = G1.msm(a_terms)
    b_terms = [(1, pk["beta_g2"])] + [(wi, pk["b_g2"][i]) for i, wi in enumerate(w)
                                      if wi and i < len(pk["b_g2"])] + [(s, pk["delta_g2"])]
    pi_b = G2.msm(b_terms)
    try:
        h = qap.compute_quotient_polynomial(z)
    except QAPError as e:
        raise GrothError("QAPError") from e
    h_terms = [(lo64(c), p) for c, p in zip(h, pk["h_g1"]) if lo64(c)]
    h1 = G1.msm(h_terms)
    npub = pk["num_public"]
    c_terms = [(w[i], pk["ic_g1"][i - npub - 1]) for i in range(npub + 1, len(w))
               if w[i] and i - npub - 1 < len(pk["ic_g1"])]
    if h1 is not INF:
        c_terms.append((1, h1))
    if pi_a is not INF:
        c_terms.append((s, pi_a))
    b1 = G1.msm([(1, pk["beta_g1"])] + [(wi, pk["b_g1"][i]) for i, wi in enumerate(w)
                                        if wi and i < len(pk["b_g1"])])
    if b1 is not INF:
        c_terms.append((r, b1))
    pi_c = G1.msm(c_terms)
    return pi_a, pi_b, pi_c


# ------------------------------------------------------- encodings ----
def g1_words(p):
    """13-word canonical little-endian layout (include/zkp.h zk_g1_affine)."""
    if p is INF:
        return [0] * 12 + [1]
    return _limbs(p[0].v, 6) + _limbs(p[1].v, 6) + [0]


def g2_words(p):
    if p is INF:
        return [0] * 24 + [1]
    x, y = p
    return _limbs(x.c0, 6) + _limbs(x.c1, 6) + _limbs(y.c0, 6) + _limbs(y.c1, 6) + [0]


def _limbs(v, k):
    return [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(k)]


def _largest(v):
    return v > (P - 1) // 2


def g1_compress(p):
    if p is INF:
        return bytes([0xC0]) + bytes(47)
    out = bytearray(p[0].v.to_bytes(48, "big"))
    out[0] |= 0x80 | (0x20 if _largest(p[1].v) else 0)
    return bytes(out)


def g2_compress(p):
    if p is INF:
        return bytes([0xC0]) + bytes(95)
    x, y = p
    out = bytearray(x.c1.to_bytes(48, "big") + x.c0.to_bytes(48, "big"))
    big = _largest(y.c1) if y.c1 else _largest(y.c0)
    out[0] |= 0x80 | (0x20 if big else 0)
    return bytes(out)


# ------------------------------------------------- deterministic rng ----
MASK64 = 0xFFFFFFFFFFFFFFFF


class SplitMix64:
    """Same generator as or_splitmix64 (oracle/zk_oracle.c)."""

    def __init__(self, seed):
        self.state = seed & MASK64

    def next(self):
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def fr(self):
        while True:
            limbs = [self.next() for _ in range(4)]
            limbs[3] &= 0x7FFFFFFFFFFFFFFF
            v = sum(l << (64 * i) for i, l in enumerate(limbs))
            if v < R:
                return v


def synthetic_witness(n, seed):
    rng = SplitMix64(seed)
    z = [1]
    for _ in range(n):
        x = rng.fr()
        y = rng.fr()
        z += [x, y, x * y % R]
    return z
