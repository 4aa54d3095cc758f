"""Shared fixtures.  `-m gpu` tests need an MI355X and libzkp_amd.so; the rest
run on CPU (oracle, host mirror, C-ABI symbol table, gloo collectives)."""
import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def zkp():
    return importlib.import_module("zero-knowledge-proofs_amd")


@pytest.fixture(scope="session")
def oracle():
    import binding
    binding.lib()
    return binding


@pytest.fixture(scope="session")
def pyref():
    import pyref as P
    return P


@pytest.fixture(scope="session")
def ctx(zkp):
    c = zkp.Context(0)
    yield c
    c.close()
