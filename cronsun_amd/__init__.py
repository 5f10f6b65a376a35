"""cronsun_amd -- MI355X-native batch fire-time expansion for cronsun's
scheduling path (node/cron Schedule.Next + Job/JobRule node resolution).

The compute path is libcronsun_gpu.so (HIP kernels for gfx950 behind the C-ABI
in include/cronsun_gpu.h).  This package is the Python mirror of the
reference's API surface on top of it; there is no CPU fallback.
"""
from . import _lib
from ._lib import (EXCLUDE_CUMULATIVE, EXCLUDE_NONE, EXCLUDE_RULE, MAX_HORIZON, ZERO_TIME,
                   CgError)

__version__ = "0.1.0"


def load():
    """Load the native library (raises if it is not built)."""
    return _lib.lib()


__all__ = ["load", "ZERO_TIME", "MAX_HORIZON", "EXCLUDE_NONE", "EXCLUDE_RULE",
           "EXCLUDE_CUMULATIVE", "CgError"]
