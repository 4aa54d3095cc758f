"""Key / proof files and the reference CLI's JSON shapes (host side, no GPU):
binary proving / verification key round trips (the reference's CLI only
writes JSON placeholders, crates/groth16-cli/src/lib.rs:157-219), and
CircuitDescription / WitnessData / PublicInputs (cli lib.rs:16-51)."""
import numpy as np

from helpers import constraints_of, g1_words, g2_words, golden

G = golden()


def _pk_vk_from_golden(zkp, case):
    import gpu_util as U
    qap = U.qap_from_case(zkp, case)
    pk = U.pk_from_golden(zkp, case, qap)
    vkd = case["vk"]
    vk = zkp.VerificationKey.from_points(g1_words(case["pk"]["alpha_g1"]), g2_words(case["pk"]["beta_g2"]),
                                         g2_words(vkd["gamma_g2"]), g2_words(case["pk"]["delta_g2"]),
                                         [g1_words(p) for p in vkd["ic_g1"]])
    return pk, vk


def test_key_files_round_trip(zkp, tmp_path):
    for case in G["prove"]:
        pk, vk = _pk_vk_from_golden(zkp, case)
        zkp.save_proving_key(pk, tmp_path / "k_pk.bin")
        back = zkp.load_proving_key(tmp_path / "k_pk.bin")
        for nm in ("a_g1", "b_g1", "b_g2", "ic_g1", "h_g1"):
            assert np.array_equal(getattr(back, nm), getattr(pk, nm)), (case["name"], nm)
        for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
            assert np.array_equal(back.point(nm), pk.point(nm))
        assert back.num_public == pk.num_public and back.qap.degree() == pk.qap.degree()
        for (rp, col, val), (rp2, col2, val2) in zip(pk.qap.csr.mats, back.qap.csr.mats):
            assert np.array_equal(rp, rp2) and np.array_equal(col, col2)
            assert (val is None and val2 is None) or np.array_equal(val, val2)
        zkp.save_verification_key(vk, tmp_path / "k_vk.bin")
        vb = zkp.load_verification_key(tmp_path / "k_vk.bin")
        assert np.array_equal(vb.ic_g1, vk.ic_g1) and vb.num_public == vk.num_public
        for nm in ("alpha_g1", "beta_g2", "gamma_g2", "delta_g2"):
            assert np.array_equal(vb.point(nm), vk.point(nm))


def test_loaded_vk_verifies_like_the_original(zkp, tmp_path):
    case = next(c for c in G["prove"] if c["error"] is None and c["num_public"] >= 1)
    _, vk = _pk_vk_from_golden(zkp, case)
    zkp.save_verification_key(vk, tmp_path / "v.bin")
    vb = zkp.load_verification_key(tmp_path / "v.bin")
    proof = zkp.Proof(np.array(g1_words(case["proof"]["a"]) + g2_words(case["proof"]["b"]) +
                               g1_words(case["proof"]["c"]), dtype=np.uint64))
    pub = [int(h, 16) for h in case["z"][1:case["num_public"] + 1]]
    assert zkp.Verifier.verify(vb, proof, pub) == zkp.Verifier.verify(vk, proof, pub)


def test_synthetic_key_file_unit_coefficients(zkp, tmp_path):
    qap = zkp.QAP(zkp.CSRMatrices.synthetic(8))
    pk = zkp.ProvingKey(qap.num_variables, qap.domain_size, 1, qap)
    pk.a_g1[:] = np.arange(pk.a_g1.size, dtype=np.uint64).reshape(pk.a_g1.shape)
    zkp.save_proving_key(pk, tmp_path / "s.bin")
    back = zkp.load_proving_key(tmp_path / "s.bin")
    assert np.array_equal(back.a_g1, pk.a_g1) and all(m[2] is None for m in back.qap.csr.mats)


def test_reference_json_shapes(zkp):
    # x*y=z with x public (the reference's test circuit, core:445-481)
    doc = {"num_variables": 3, "num_public": 1,
           "constraints": [{"a": [[1, "1"]], "b": [[2, "0x1"]], "c": [[3, "01"]]}]}
    cs = zkp.r1cs_from_circuit_json(doc)
    assert cs.num_variables == 4 and cs.num_constraints() == 1
    w = zkp.witness_from_json({"assignment": ["1", "3", "4", "c"], "num_public": 1})
    assert [int(r[0]) for r in w.assignment] == [1, 3, 4, 12]
    assert cs.is_satisfied([1, 3, 4, 12]) and not cs.is_satisfied([1, 3, 4, 13])
    assert zkp.public_inputs_from_json({"inputs": ["3"]}) == [3]
    # golden circuits with non-unit coefficients survive the JSON shape
    for case in G["prove"][:4]:
        cons = constraints_of(case)
        doc = {"num_variables": case["num_variables"] - 1, "num_public": case["num_public"],
               "constraints": [{m: [[v, "%x" % c] for v, c in sorted(lc.items())] for m, lc in zip("abc", con)}
                               for con in cons]}
        cs = zkp.r1cs_from_circuit_json(doc)
        assert cs.num_variables == case["num_variables"]
        import gpu_util as U
        want = U.qap_from_case(zkp, case).csr.mats
        for (rp, col, val), (rp2, col2, val2) in zip(zkp.CSRMatrices.from_r1cs(cs).mats, want):
            assert np.array_equal(rp, rp2) and np.array_equal(col, col2) and np.array_equal(val, val2)
        z = [int(h, 16) for h in case["z"]]
        assert cs.is_satisfied(z) == (case["error"] is None)
