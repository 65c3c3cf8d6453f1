"""ocean_model_arch_amd -- MI355X-native shallow-water barotropic step (HIP/gfx950).

Drop-in for the SW hot path of Andrcraft9/ocean_model_arch: kernels + PSy layer in
libocn_sw.so (C ABI: include/ocn_sw.h), hosts in Python (this package) and Fortran
(host/fortran, ISO_C_BINDING).
"""
from ._lib import OcnError, OcnLibraryError, build, build_id, lib  # noqa: F401
from .config import BasinConfig, ParallelConfig, SWConfig, box_config, read_mask  # noqa: F401
from .model import OceanModel, make_unique_id, run_ranks  # noqa: F401

__all__ = ["OceanModel", "BasinConfig", "SWConfig", "ParallelConfig", "box_config", "read_mask",
           "make_unique_id", "run_ranks", "build", "lib", "OcnError", "OcnLibraryError"]
