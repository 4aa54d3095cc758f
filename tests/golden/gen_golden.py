"""Generate tests/golden/*.json with oracle/pyref.py -- the independent
pure-Python restatement of the reference's LITERAL dense algorithm
(QAP::from_r1cs per-variable iFFT, dense quotient, Horner setup, naive MSM).
The reference itself (Rust + arkworks) cannot be built or run in this image,
so these vectors pin the C oracle and the GPU path to a second, independent
restatement.  Run from the repo root:  python tests/golden/gen_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import pyref as P  # noqa: E402


def hx(v):
    return "%x" % v


def g1(p):
    return None if p is P.INF else [hx(p[0].v), hx(p[1].v)]


def g2(p):
    return None if p is P.INF else [hx(p[0].c0), hx(p[0].c1), hx(p[1].c0), hx(p[1].c1)]


def circuit_json(cs):
    return [[{str(k): hx(v) for k, v in lc.items()} for lc in con] for con in cs.constraints]


def prove_case(name, cs, z, num_public, seed):
    rng = P.SplitMix64(seed)
    params = [rng.fr() for _ in range(5)]
    r, s = rng.fr(), rng.fr()
    qap = P.QAP(cs)
    pk, vk = P.generate_from_qap(qap, params, num_public)
    case = {"name": name, "num_variables": cs.num_variables, "constraints": circuit_json(cs),
            "num_public": num_public, "params": [hx(x) for x in params], "r": hx(r), "s": hx(s),
            "z": [hx(x) for x in z], "domain": qap.n}
    try:
        h = qap.compute_quotient_polynomial(z)
        case["h"] = [hx(x) for x in h]
    except P.QAPError:
        case["h"] = None
    try:
        pa, pb, pc = P.prove(pk, qap, z, num_public, r, s)
        case["proof"] = {"a": g1(pa), "b": g2(pb), "c": g1(pc)}
        case["proof_compressed"] = (P.g1_compress(pa) + P.g2_compress(pb) + P.g1_compress(pc)).hex()
        case["error"] = None
    except P.GrothError as e:
        case["proof"] = None
        case["error"] = str(e)
    case["pk"] = {"alpha_g1": g1(pk["alpha_g1"]), "beta_g1": g1(pk["beta_g1"]),
                  "delta_g1": g1(pk["delta_g1"]), "beta_g2": g2(pk["beta_g2"]),
                  "delta_g2": g2(pk["delta_g2"]),
                  "a_g1": [g1(p) for p in pk["a_g1"]], "b_g1": [g1(p) for p in pk["b_g1"]],
                  "b_g2": [g2(p) for p in pk["b_g2"]], "ic_g1": [g1(p) for p in pk["ic_g1"]],
                  "h_g1": [g1(p) for p in pk["h_g1"]]}
    case["vk"] = {"gamma_g2": g2(vk["gamma_g2"]), "ic_g1": [g1(p) for p in vk["ic_g1"]]}
    return case


def random_circuit(nc, nvar_extra, num_public, seed):
    rng = P.SplitMix64(seed)
    cs = P.R1CS(num_public)
    for _ in range(nvar_extra):
        cs.allocate_variable()
    V = cs.num_variables
    z = [1] + [rng.fr() for _ in range(V - 1)]
    # constraints a*b = c where c's last term is solved for satisfiability
    for k in range(nc):
        def lc(m):
            d = {}
            for _ in range(m):
                v = rng.next() % V
                d[v] = rng.fr() if rng.next() & 1 else 1
            return d
        a, b = lc(2), lc(2)
        av = sum(z[v] * c for v, c in a.items()) % P.R
        bv = sum(z[v] * c for v, c in b.items()) % P.R
        tgt = 1 + (k % (V - 1))
        c = {v: co for v, co in lc(1).items() if v != tgt}
        rest = sum(z[v] * co for v, co in c.items()) % P.R
        # c_tgt * z_tgt = av*bv - rest
        c[tgt] = (av * bv - rest) * pow(z[tgt], P.R - 2, P.R) % P.R
        cs.enforce_multiplication(a, b, c)
    return cs, z


def main():
    cases = []
    # config 1: the toy x*y=z of crates/groth16-core/src/lib.rs:445-481
    cs = P.R1CS(0)
    x, y, zv = cs.allocate_variable(), cs.allocate_variable(), cs.allocate_variable()
    cs.enforce_multiplication({x: 1}, {y: 1}, {zv: 1})
    cases.append(prove_case("toy_xyz", cs, [1, 3, 4, 12], 1, 0x70F))
    cases.append(prove_case("toy_xyz_invalid", cs, [1, 3, 4, 13], 1, 0x70F))
    for n in (2, 4, 8):
        cs = P.synthetic_r1cs(n)
        cases.append(prove_case(f"synthetic_{n}", cs, P.synthetic_witness(n, 1000 + n), 1, 2000 + n))
    cs, z = random_circuit(5, 6, 2, 77)
    cases.append(prove_case("random_5x9_pub2", cs, z, 2, 78))
    cs, z = random_circuit(3, 3, 0, 91)
    cases.append(prove_case("random_3x4_pub0", cs, z, 0, 92))
    # row 1 broken (validate) and row 2 broken (quotient) on synthetic_4
    z = P.synthetic_witness(4, 1004)
    z[6] = (z[6] + 1) % P.R
    cases.append(prove_case("synthetic_4_bad_row1", P.synthetic_r1cs(4), z, 1, 2004))
    z = P.synthetic_witness(4, 1004)
    z[9] = (z[9] + 1) % P.R
    cases.append(prove_case("synthetic_4_bad_row2", P.synthetic_r1cs(4), z, 1, 2004))

    # MSM vectors
    rng = P.SplitMix64(0xA11CE)
    msm = []
    for nm, bits in (("g1_full", 255), ("g1_64", 64)):
        pts = [P.G1.mul(P.G1.gen, rng.next()) for _ in range(10)] + [P.INF]
        sc = [rng.fr() if bits == 255 else rng.next() for _ in range(11)]
        sc[3] = 0
        msm.append({"name": nm, "group": 1, "bases": [g1(p) for p in pts], "scalars": [hx(s) for s in sc],
                    "out": g1(P.G1.msm(list(zip(sc, pts))))})
    pts = [P.G2.mul(P.G2.gen, rng.next()) for _ in range(6)] + [P.INF]
    sc = [rng.fr() for _ in range(7)]
    msm.append({"name": "g2_full", "group": 2, "bases": [g2(p) for p in pts], "scalars": [hx(s) for s in sc],
                "out": g2(P.G2.msm(list(zip(sc, pts))))})
    # NTT vectors
    ntt = []
    for n in (1, 2, 8, 16):
        v = [rng.fr() for _ in range(n)]
        ntt.append({"n": n, "in": [hx(a) for a in v], "fft": [hx(a) for a in P.dft(v, n)],
                    "ifft": [hx(a) for a in P.dft(v, n, inverse=True)],
                    "coset_fft_g7": [hx(a) for a in P.dft([c * pow(7, i, P.R) % P.R for i, c in enumerate(v)], n)]})
    consts = {"r": hx(P.R), "p": hx(P.P), "root_of_unity_2_32": hx(P.root_of_unity(1 << 32)),
              "g1_generator_compressed": P.g1_compress(P.G1.gen).hex(),
              "g2_generator_compressed": P.g2_compress(P.G2.gen).hex()}
    out = {"generator": "tests/golden/gen_golden.py (oracle/pyref.py, literal dense restatement)",
           "consts": consts, "prove": cases, "msm": msm, "ntt": ntt}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", len(cases), "prove cases,", len(msm), "msm,", len(ntt), "ntt")


if __name__ == "__main__":
    main()
