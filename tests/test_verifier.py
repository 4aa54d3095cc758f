"""Verifier / BatchVerifier / pairing / compressed decoding (host code in
libzkp_amd.so, no GPU): crates/groth16-core/src/lib.rs:303-432, core:28.

The reference pins no pairing value.  What pins this code:
  * bilinearity and non-degeneracy KATs of the pairing (e(aP, bQ) =
    e(abP, Q), e(P, Q) != 1) -- properties a wrong Miller loop or final
    exponentiation does not have;
  * proofs built to satisfy the Groth16 equation by construction (verify ->
    True; any tampering -> False);
  * the reference's own test circuit x*y=z (core:445-511) through the oracle
    prover: with setup parameters whose derived scalars stay below 2^64 the
    lo64 truncation changes nothing and the proof verifies; with random
    full-width parameters it does not (SURVEY.md 4.3 -- the reference's
    test_simple_proof fails the same way);
  * compressed round trips of oracle proofs and the zcash flag rules.
"""
import numpy as np
import pytest

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def g1w(pyref, p):
    return np.array(pyref.g1_words(p), dtype=np.uint64)


def g2w(pyref, p):
    return np.array(pyref.g2_words(p), dtype=np.uint64)


def test_pairing_bilinear(zkp, pyref):
    G1, G2, g1, g2 = pyref.G1, pyref.G2, pyref.G1.gen, pyref.G2.gen
    a, b = 0xDEADBEEF12345, 0xC0FFEE99
    P, Q = G1.mul(g1, a), G2.mul(g2, b)
    ab = G1.neg(G1.mul(g1, a * b % R))
    assert zkp.pairing_product_is_one([g1w(pyref, P), g1w(pyref, ab)], [g2w(pyref, Q), g2w(pyref, g2)])
    off = G1.neg(G1.mul(g1, (a * b + 1) % R))
    assert not zkp.pairing_product_is_one([g1w(pyref, P), g1w(pyref, off)], [g2w(pyref, Q), g2w(pyref, g2)])
    assert not zkp.pairing_product_is_one([g1w(pyref, g1)], [g2w(pyref, g2)])          # non-degenerate
    # e(2P, Q) = e(P, 2Q); infinity on either side contributes 1
    assert zkp.pairing_product_is_one([g1w(pyref, G1.mul(g1, 2)), g1w(pyref, G1.neg(g1))],
                                      [g2w(pyref, g2), g2w(pyref, G2.mul(g2, 2))])
    assert zkp.pairing_product_is_one([g1w(pyref, None), g1w(pyref, g1)], [g2w(pyref, g2), g2w(pyref, None)])
    # full-width scalars: e(sP, Q) e(P, -sQ) = 1
    s = 0x5A5A_1234_5678_9ABC_DEF0_1111_2222_3333_4444_5555_6666_7777_8888_9999 % R
    assert zkp.pairing_product_is_one([g1w(pyref, G1.mul(g1, s)), g1w(pyref, g1)],
                                      [g2w(pyref, g2), g2w(pyref, G2.neg(G2.mul(g2, s)))])


def test_pairing_rejects_bad_points(zkp, pyref):
    p = g1w(pyref, pyref.G1.gen)
    p[6] ^= 1                                    # off the curve
    with pytest.raises(ValueError):
        zkp.pairing_product_is_one([p], [g2w(pyref, pyref.G2.gen)])


def _constructed(zkp, pyref, npub, seed):
    """vk and a proof satisfying e(A,B) = e(alpha,beta) e(IC,gamma) e(C,delta)
    by construction: A = a G, B = b H, C = (ab - alpha beta - ic gamma)/delta G."""
    G1, G2, g1, g2 = pyref.G1, pyref.G2, pyref.G1.gen, pyref.G2.gen
    rng = pyref.SplitMix64(seed)
    al, be, ga, de, a, b = (rng.fr() for _ in range(6))
    ks = [rng.fr() for _ in range(npub + 1)]
    x = [rng.next() for _ in range(npub)]        # public inputs (u64, so lo64 is exact)
    ic = (ks[0] + sum(xi * k for xi, k in zip(x, ks[1:]))) % R
    c = (a * b - al * be - ic * ga) * pow(de, R - 2, R) % R
    vk = zkp.VerificationKey.from_points(g1w(pyref, G1.mul(g1, al)), g2w(pyref, G2.mul(g2, be)),
                                         g2w(pyref, G2.mul(g2, ga)), g2w(pyref, G2.mul(g2, de)),
                                         [g1w(pyref, G1.mul(g1, k)) for k in ks])
    proof = zkp.Proof(np.concatenate([g1w(pyref, G1.mul(g1, a)), g2w(pyref, G2.mul(g2, b)),
                                      g1w(pyref, G1.mul(g1, c))]))
    return vk, proof, x


@pytest.mark.parametrize("npub", [0, 1, 3])
def test_verify_constructed(zkp, pyref, npub):
    vk, proof, x = _constructed(zkp, pyref, npub, 40 + npub)
    assert zkp.Verifier.verify(vk, proof, x)
    bad = zkp.Proof(proof.words.copy())
    bad.words[:13] = g1w(pyref, pyref.G1.gen)     # another A
    assert not zkp.Verifier.verify(vk, bad, x)
    if npub:
        y = list(x)
        y[0] = (y[0] + 1) % (1 << 64)
        assert not zkp.Verifier.verify(vk, proof, y)   # core:484-511 (wrong public input)
        # Fr::from(lo64(x)) (core:323-328): the high limbs are ignored
        assert zkp.Verifier.verify(vk, proof, [xi + (5 << 64) for xi in x])
    with pytest.raises(zkp.InvalidWitness):            # core:315-320
        zkp.Verifier.verify(vk, proof, list(x) + [1])


def _toy(oracle, params, z, r, s):
    """The reference's own test circuit x*y=z (core:445-481), x public."""
    csr = oracle.CSR.from_constraints([({1: 1}, {2: 1}, {3: 1})], 4)
    rc, pk, vk = oracle.setup(csr, params, 1)
    assert rc == 0
    rc, proof = oracle.prove(pk, csr, oracle.fr_array(z), 1, r, s)
    assert rc == 0
    return vk, proof


def _vk_of(zkp, ovk):
    return zkp.VerificationKey.from_points(ovk.field("alpha_g1"), ovk.field("beta_g2"), ovk.field("gamma_g2"),
                                           ovk.field("delta_g2"), ovk.ic_g1)


def test_verify_reference_toy_circuit(zkp, oracle, pyref):
    rng = pyref.SplitMix64(777)
    r, s = rng.fr(), rng.fr()
    # derived scalars (beta A_i + alpha B_i + C_i) / delta etc. all < 2^64:
    # truncation is the identity and the reference's construction verifies
    vk, proof = _toy(oracle, [2, 3, 1, 1, 5], [1, 3, 4, 12], r, s)
    vk = _vk_of(zkp, vk)
    proof = zkp.Proof(proof)
    assert zkp.Verifier.verify(vk, proof, [3])
    assert not zkp.Verifier.verify(vk, proof, [5])       # test_invalid_proof (core:484-511)
    # single-proof batch with coefficient 1 is the plain check; a random
    # coefficient c scales e(A, B) by c^2 but the rest by c (the reference's
    # batching rule, mirrored as written)
    assert zkp.BatchVerifier.verify_batch(vk, [(proof, [3])], coeffs=[1])
    assert not zkp.BatchVerifier.verify_batch(vk, [(proof, [3])], coeffs=[rng.fr()])
    assert zkp.BatchVerifier.verify_batch(vk, [], coeffs=[])
    with pytest.raises(zkp.InvalidWitness):
        zkp.BatchVerifier.verify_batch(vk, [(proof, [3, 4])], coeffs=[1])
    # random full-width setup parameters: lo64 truncation breaks the equation
    # (SURVEY.md 4.3), exactly as in the reference's test_simple_proof
    vk2, proof2 = _toy(oracle, [rng.fr() for _ in range(5)], [1, 3, 4, 12], r, s)
    assert not zkp.Verifier.verify(_vk_of(zkp, vk2), zkp.Proof(proof2), [3])


def test_deserialize_round_trip(zkp, oracle, pyref):
    rng = pyref.SplitMix64(99)
    vk, proof = _toy(oracle, [rng.fr() for _ in range(5)], [1, 3, 4, 12], rng.fr(), rng.fr())
    data = oracle.proof_compress(proof)
    back = zkp.Proof.deserialize_compressed(data)
    assert np.array_equal(back.words, proof)
    assert back.serialize_compressed() == data
    # identity points round-trip too
    inf = zkp.Proof(np.concatenate([g1w(pyref, None), g2w(pyref, None), g1w(pyref, None)]))
    assert np.array_equal(zkp.Proof.deserialize_compressed(inf.serialize_compressed()).words, inf.words)


def test_deserialize_rejects(zkp, oracle, pyref):
    rng = pyref.SplitMix64(5)
    _, proof = _toy(oracle, [rng.fr() for _ in range(5)], [1, 3, 4, 12], rng.fr(), rng.fr())
    good = bytearray(oracle.proof_compress(proof))
    cases = []
    b = bytearray(good); b[0] &= 0x7F; cases.append(b)                  # not compressed
    b = bytearray(good); b[0] |= 0x60; cases.append(b)                  # infinity + sort flag
    b = bytearray(good); b[0] = 0x80 | 0x1F; b[1:48] = b"\xff" * 47; cases.append(b)   # x >= p
    # an x whose x^3 + 4 is a square but whose point is outside the r-order
    # subgroup (cofactor ~2^126: a random curve point almost surely is)
    P = pyref.P
    x = 5
    while pow((x ** 3 + 4) % P, (P - 1) // 2, P) != 1:
        x += 1
    b = bytearray(good); b[:48] = x.to_bytes(48, "big"); b[0] |= 0x80; cases.append(b)
    # an x with no point on the curve
    x = 5
    while pow((x ** 3 + 4) % P, (P - 1) // 2, P) == 1:
        x += 1
    b = bytearray(good); b[:48] = x.to_bytes(48, "big"); b[0] |= 0x80; cases.append(b)
    # infinity flag with a non-zero x (G1 a, and G2 b in either half): the
    # zcash encoding has one identity; anything else would be malleable
    b = bytearray(good); b[0:48] = b"\xc0" + b"\0" * 47; b[17] = 1; cases.append(b)
    b = bytearray(good); b[0] = 0xC1; b[1:48] = b"\0" * 47; cases.append(b)
    b = bytearray(good); b[48:144] = b"\xc0" + b"\0" * 95; b[48 + 70] = 2; cases.append(b)
    for c in cases:
        with pytest.raises(ValueError):
            zkp.Proof.deserialize_compressed(bytes(c))
    # the canonical identity encoding still decodes
    b = bytearray(good); b[0:48] = b"\xc0" + b"\0" * 47
    assert zkp.Proof.deserialize_compressed(bytes(b)).a[12] == 1
