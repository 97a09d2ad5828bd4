"""CPU tests of the C-ABI boundary: the library builds, loads and exports exactly what
include/plk.h declares; calls that need no GPU behave (no compute without a GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    hdr = (ROOT / "include" / "plk.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(plk_\w+)\s*\(", hdr, re.M)))


def test_header_and_binding_agree(plk):
    assert sorted(plk.ABI_SYMBOLS) == declared_symbols()


def test_library_exports_every_declared_symbol(plk):
    lib = ctypes.CDLL(str(ROOT / "dusk-plonk_amd" / "libplk.so"))
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_status_strings(plk):
    lib = plk.plonk._lib()
    assert lib.plk_abi_version() == 2  # 2: plk_prover lanes, sharded commits, SCALE codec
    assert b"degree" in lib.plk_status_str(plk.PLK_E_DEGREE)
    assert lib.plk_status_str(99) == b"unknown status"


def test_null_arguments_are_rejected_without_gpu(plk):
    lib = plk.plonk._lib()
    assert lib.plk_ctx_create(0, None) == plk.PLK_E_ARG
    assert lib.plk_domain_get(None, 3, None) == plk.PLK_E_ARG
    assert lib.plk_ntt(None, None, 0, 1, 0) == plk.PLK_E_ARG
    assert lib.plk_commit(None, None, 0, None) == plk.PLK_E_ARG
    assert lib.plk_srs_len(None, None) == plk.PLK_E_ARG
    assert lib.plk_msm_sharded(None, 0, None, 0, None) == plk.PLK_E_ARG
    assert lib.plk_ntt_stream(None, None, 0, 1, 0, None) == plk.PLK_E_ARG
    assert lib.plk_aggregate_witness(None, None, None, 0, None, None, None, None) == plk.PLK_E_ARG
    assert lib.plk_aggregate_witness_dev(None, None, None, 0, None, None, None, None,
                                         None) == plk.PLK_E_ARG
    from dusk_plonk_amd.prover import _bind
    b = _bind()
    assert b.plk_prover_create(None, None) == plk.PLK_E_ARG
    assert b.plk_prover_prove(None, None, 0, None, None, 0, None) == plk.PLK_E_ARG
    assert b.plk_prover_shard(None, None, 0, 0, 2, None, None) == plk.PLK_E_ARG
    assert b.plk_proof_decode(None, 0, None) == plk.PLK_E_ARG


def test_device_count_never_fails(plk):
    assert plk.device_count() >= 0


def test_no_gpu_means_loud_failure(plk):
    if plk.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(plk.PlonkError) as e:
        plk.Context(0)
    assert e.value.status == plk.PLK_E_NODEV
