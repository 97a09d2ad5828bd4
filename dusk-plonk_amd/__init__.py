"""dusk_plonk_amd — MI355X-native backend for dusk-plonk's hot path.

BLS12-381 Fr NTT family (poly_commit::Fft) and the G1 MSM behind KZG commit
(zksnarks PlonkParams::commit), as hand-written HIP kernels for gfx950 behind the C ABI
in include/plk.h. See DESIGN.md.
"""
from .plonk import (  # noqa: F401
    ABI_SYMBOLS, Coefficients, Commitment, Context, Fft, PLK_E_ARG, PLK_E_DEGREE, PLK_E_DEVICE,
    PLK_E_NODEV, PLK_E_OOM, PLK_OK, PlonkError, PlonkParams, PointsValue, build_info, check_build,
    device_count, g1_sum, msm_sharded,
)

__all__ = [
    "ABI_SYMBOLS", "Coefficients", "Commitment", "Context", "Fft", "PlonkError", "PlonkParams",
    "PointsValue", "build_info", "check_build", "device_count", "g1_sum", "msm_sharded",
]
