"""PSy dispatcher -- mirror of core/kernel_interface.f90.

``envoke(sub_kernel, sub_sync, kernel_parameters)`` runs ``sub_kernel(k, params)`` for every
local block k and then ``sub_sync(-1, sync_parameters_all)`` (kernel_interface.f90:48-119, the
_MPP_NO_PARALLEL_MODE_ / _MPP_BLOCK_MODE_ path).  Kernels launch asynchronously on the model's
HIP stream, so the block loop never waits on the device.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class KernelParameters:
    """kernel_parameters_type (kernel_interface.f90:15-21)."""
    tau: float = 0.0
    time_smooth: float = 0.0
    data_id: int = 0

    def clear(self):
        self.tau, self.time_smooth, self.data_id = 0.0, 0.0, 0


@dataclass
class SyncParameters:
    """sync_parameters_type (shared/mpp/sync.f90:27-32); sync_mode 3 = all."""
    sync_mode: int = 3
    sync_device_host: int = 0
    data_id: int = 0


def envoke_empty_kernel(k, kernel_parameters):   # kernel_interface.f90:38-41
    pass


def envoke_empty_sync(k, sync_parameters):        # kernel_interface.f90:43-46
    pass


def envoke(model, sub_kernel, sub_sync, kernel_parameters: KernelParameters):
    """kernel_interface.f90:48-119."""
    for k in range(len(model.blocks)):
        sub_kernel(k, kernel_parameters)
    sub_sync(-1, SyncParameters(sync_mode=3, data_id=kernel_parameters.data_id))
