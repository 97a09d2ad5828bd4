import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C ABI on the GPU)")
    config.addinivalue_line("markers", "slow: large-size GPU property test")


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib.load()


@pytest.fixture(scope="session")
def plk():
    """The product package; on a GPU session the HIP library must load (no fallback)."""
    lib = ROOT / "dusk-plonk_amd" / "libplk.so"
    if not lib.exists():
        subprocess.run([sys.executable, str(ROOT / "dusk-plonk_amd" / "build_ext.py")], check=True)
    import dusk_plonk_amd
    # the library must have been built from this tree's sources and flags (plk_build_info)
    dusk_plonk_amd.check_build()
    return dusk_plonk_amd


@pytest.fixture(scope="session")
def gpu_ctx(plk):
    if plk.device_count() == 0:
        pytest.fail("GPU test selected but no GPU is visible")
    return plk.Context.default(0)


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    g = ROOT / "tests" / "golden"
    return {
        "ntt": dict(np.load(g / "ntt_golden.npz", allow_pickle=False)),
        "msm": dict(np.load(g / "msm_golden.npz", allow_pickle=False)),
    }
