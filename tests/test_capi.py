"""CPU checks of the drop-in boundary: libzkp_amd.so loads and exports every
function include/zkp.h declares; no compute calls (no GPU here)."""
import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(HERE, "..", "include", "zkp.h")
TEST_HEADER = os.path.join(HERE, "..", "include", "zkp_test.h")


def declared(header=HEADER):
    src = open(header).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(zk_[a-z0-9_]+)\s*\(", src)))


def test_header_parses():
    names = declared()
    assert "zk_groth16_prove" in names and "zk_msm_g1" in names and len(names) >= 20


def test_library_exports_every_symbol(zkp):
    lib = ctypes.CDLL(zkp.LIB_PATH)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(zkp.EXPORTS) == declared()


def test_test_hooks_live_in_their_own_library(zkp):
    """zk_test_* (virtual ranks, bare exchange, fault injection) are declared
    in include/zkp_test.h and exported by libzkp_amd_test.so only: the
    shipped library has no way to inject a failure."""
    lib = ctypes.CDLL(zkp.LIB_PATH)
    for n in declared(TEST_HEADER):
        assert not hasattr(lib, n), n
    assert sorted(zkp.TEST_EXPORTS) == declared(TEST_HEADER)
    t = zkp.test_lib()
    for n in zkp.TEST_EXPORTS:
        assert hasattr(t, n)


def test_struct_sizes(zkp):
    assert ctypes.sizeof(zkp._G1) == 104 and ctypes.sizeof(zkp._G2) == 200
    assert ctypes.sizeof(zkp._Proof) == 408 and ctypes.sizeof(zkp._SetupParams) == 160
    assert ctypes.sizeof(zkp._CSR) == 16 + 9 * 8


def test_ctx_create_fails_cleanly_without_gpu(zkp):
    import torch
    if torch.cuda.is_available():
        return
    assert zkp.lib().zk_ctx_create(0) is None
    try:
        zkp.Context(0)
    except zkp.DeviceError:
        pass
    else:
        raise AssertionError("Context(0) must fail loudly without a GPU")


def test_combine_rejects_bad_args(zkp):
    assert zkp.lib().zk_groth16_prove_combine(None, 0, None, None, None) == zkp.ZK_ERR_ARG


def test_build_id_matches_sources(zkp):
    """libzkp_amd.so embeds the hash of the sources it was compiled from
    (Makefile -> zk_build_id); it must be this tree's."""
    bid = zkp.build_id()
    assert " src:" in bid
    assert bid.endswith("src:" + zkp.source_hash()), (bid, zkp.source_hash())
