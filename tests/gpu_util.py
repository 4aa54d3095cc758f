"""Helpers for GPU parity tests: build product-side keys from golden / oracle data."""
import numpy as np

from helpers import g1_words, g2_words


def set_point(zkp, field, words):
    for i, w in enumerate(words):
        field.w[i] = int(w)


def pk_from_golden(zkp, case, qap):
    gp = case["pk"]
    V, n = case["num_variables"], case["domain"]
    pk = zkp.ProvingKey(V, n, case["num_public"], qap)
    pk.a_g1[:] = [g1_words(p) for p in gp["a_g1"]]
    pk.b_g1[:] = [g1_words(p) for p in gp["b_g1"]]
    pk.b_g2[:] = [g2_words(p) for p in gp["b_g2"]]
    if len(gp["ic_g1"]):
        pk.ic_g1[:] = [g1_words(p) for p in gp["ic_g1"]]
    pk.h_g1[:] = [g1_words(p) for p in gp["h_g1"]]
    for nm in ("alpha_g1", "beta_g1", "delta_g1"):
        set_point(zkp, getattr(pk.s, nm), g1_words(gp[nm]))
    for nm in ("beta_g2", "delta_g2"):
        set_point(zkp, getattr(pk.s, nm), g2_words(gp[nm]))
    return pk


def pk_from_oracle(zkp, opk, qap, num_public):
    V, n = qap.num_variables, qap.domain_size
    pk = zkp.ProvingKey(V, n, num_public, qap)
    pk.a_g1[:] = opk.a_g1
    pk.b_g1[:] = opk.b_g1
    pk.b_g2[:] = opk.b_g2
    pk.ic_g1[:] = opk.ic_g1[:len(pk.ic_g1)]
    pk.h_g1[:] = opk.h_g1
    for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
        set_point(zkp, getattr(pk.s, nm), opk.field(nm))
    return pk


def qap_from_case(zkp, case):
    from helpers import constraints_of
    cs = zkp.R1CS(case["num_public"])
    while cs.num_variables < case["num_variables"]:
        cs.allocate_variable()
    for a, b, c in constraints_of(case):
        cs.enforce_multiplication(zkp.LinearCombination(a), zkp.LinearCombination(b), zkp.LinearCombination(c))
    return zkp.QAP.from_r1cs(cs)


def oracle_pk_from(oracle, pk):
    """The oracle's PK struct holding the same bases as a product ProvingKey
    (host arrays, canonical words) -- the checker proves from the same key."""
    V, n = pk.qap.num_variables, pk.qap.domain_size
    opk = oracle.PK(V, n, pk.num_public)
    for nm in ("a_g1", "b_g1", "b_g2", "h_g1"):
        getattr(opk, nm)[:] = getattr(pk, nm)
    opk.ic_g1[:len(pk.ic_g1)] = pk.ic_g1
    for nm in ("alpha_g1", "beta_g1", "delta_g1", "beta_g2", "delta_g2"):
        arr = getattr(opk.s, nm)
        for i, x in enumerate(pk.point(nm)):
            arr[i] = int(x)
    opk.s.a_len, opk.s.b_len, opk.s.b2_len = len(pk.a_g1), len(pk.b_g1), len(pk.b_g2)
    opk.s.ic_len, opk.s.h_len, opk.s.num_public = len(pk.ic_g1), len(pk.h_g1), pk.num_public
    return opk
