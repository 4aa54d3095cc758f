"""CPU tests of the Python mirror of the reference interface (no GPU calls)."""
import numpy as np
import pytest

from helpers import constraints_of, golden


def test_r1cs_builder_matches_reference_layout(zkp):
    """crates/groth16-r1cs/src/lib.rs:240-293 + qap:334-353."""
    cs = zkp.R1CS(0)
    x, y, z = cs.allocate_variable(), cs.allocate_variable(), cs.allocate_variable()
    assert (x, y, z) == (1, 2, 3)
    cs.enforce_multiplication(zkp.LinearCombination.from_variable(x), zkp.LinearCombination.from_variable(y),
                              zkp.LinearCombination.from_variable(z))
    qap = zkp.QAP.from_r1cs(cs)
    assert qap.num_variables == 4 and qap.num_constraints == 1 and qap.domain_size >= 1
    assert qap.degree() == 1
    assert cs.is_satisfied([1, 3, 4, 12]) and not cs.is_satisfied([1, 3, 4, 13])
    rp, col, val = qap.csr.mats[0]
    assert list(rp) == [0, 1] and list(col) == [1] and list(val[0]) == [1, 0, 0, 0]


def test_linear_combination_merges_and_drops_zero(zkp):
    lc = zkp.LinearCombination()
    lc.add_term(5, 3)
    lc.add_term(5, zkp.R - 3)
    assert lc.terms == {}
    lc.add_term(2, 0)
    assert lc.terms == {}


def test_enforce_equal(zkp):
    cs = zkp.R1CS(1)
    a = cs.allocate_variable()
    cs.enforce_equal(zkp.LinearCombination.from_variable(1), zkp.LinearCombination.from_variable(a))
    assert cs.is_satisfied([1, 7, 7]) and not cs.is_satisfied([1, 7, 8])


def test_witness_errors(zkp):
    """Witness::new (crates/groth16-core/src/lib.rs:81-99)."""
    with pytest.raises(zkp.InvalidWitness):
        zkp.Witness([1, 3, 4, 12], 4)
    with pytest.raises(zkp.InvalidWitness):
        zkp.Witness([2, 3, 4, 12], 1)
    w = zkp.Witness([1, 3, 4, 12], 1)
    assert w.public_inputs()[0, 0] == 3


def test_setup_params_validate(zkp):
    with pytest.raises(zkp.SetupError):
        zkp.SetupParams(0, 1, 1, 1, 1).validate()
    zkp.SetupParams(1, 1, 1, 1, 0).validate()   # tau may be zero (setup:128-136)


def test_synthetic_csr(zkp, oracle):
    n = 16
    a = zkp.CSRMatrices.synthetic(n)
    b = oracle.CSR.synthetic(n)
    for (rp, col, val), (rp2, col2, val2) in zip(a.mats, b.mats):
        assert np.array_equal(rp, rp2) and np.array_equal(col, col2[:n]) and val is None and val2 is None


def test_from_r1cs_matches_golden_constraints(zkp):
    case = [c for c in golden()["prove"] if c["name"] == "random_5x9_pub2"][0]
    cs = zkp.R1CS(case["num_public"])
    while cs.num_variables < case["num_variables"]:
        cs.allocate_variable()
    for a, b, c in constraints_of(case):
        cs.enforce_multiplication(zkp.LinearCombination(a), zkp.LinearCombination(b), zkp.LinearCombination(c))
    z = [int(x, 16) for x in case["z"]]
    assert cs.is_satisfied(z)
