"""topfusion_amd -- MI355X-native (gfx950) dense RGB-D reconstruction hot path.

The product is libtfusion_hip.so (hand-written HIP kernels + C-ABI, include/tfusion_hip.h)
built from topfusion_amd/csrc.  This package holds the Python host mirror of the reference
tfusion API (TopFu, TopFuParams) over that C-ABI and the synthetic workload generators.
"""
from ._lib import TfError, TfParams, TfStats, default_params, load  # noqa: F401
from .topfu import TopFu, TopFuParams  # noqa: F401

__all__ = ["TopFu", "TopFuParams", "TfParams", "TfStats", "TfError", "default_params", "load"]
