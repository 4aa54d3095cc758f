"""Fixture loading and layout conversions shared by the tests."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
MASK = (1 << 64) - 1


def golden():
    with open(os.path.join(HERE, "golden", "golden.json")) as f:
        return json.load(f)


def limbs(v, k):
    return [(v >> (64 * i)) & MASK for i in range(k)]


def g1_words(p):
    """golden G1 ([x, y] hex or None) -> 13 uint64 words (zk_g1_affine)."""
    if p is None:
        return [0] * 12 + [1]
    return limbs(int(p[0], 16), 6) + limbs(int(p[1], 16), 6) + [0]


def g2_words(p):
    if p is None:
        return [0] * 24 + [1]
    return sum((limbs(int(c, 16), 6) for c in p), []) + [0]


def fr_rows(hexes):
    return np.array([limbs(int(h, 16), 4) for h in hexes], dtype=np.uint64).reshape(-1, 4)


def constraints_of(case):
    """golden constraints -> list of (a, b, c) dicts var -> int"""
    return [tuple({int(k): int(v, 16) for k, v in lc.items()} for lc in con) for con in case["constraints"]]


def proof_words(case):
    p = case["proof"]
    return g1_words(p["a"]) + g2_words(p["b"]) + g1_words(p["c"])
