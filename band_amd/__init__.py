"""band_amd — MI355X-native (gfx950) per-subgraph execution backend for Band.

The product is `libband_hip.so` (hand-written HIP kernels + the C++ HIP
backend implementing Band's IModel / IModelExecutor / ITensorView /
IBackendUtil, behind the C ABIs in include/).  This package is the Python
mirror of that interface (ctypes), used by tests and bench.py.
"""
from .backend import (DataType, DeviceFlag, GetAvailableDevices, HipModel, HipModelExecutor,  # noqa: F401
                      HipTensorView, ModelSpec, RunMixedJobs, SetWorkerDevice, Status, SubgraphKey, WorkerDevice)

__all__ = ["DataType", "DeviceFlag", "GetAvailableDevices", "HipModel", "HipModelExecutor",
           "HipTensorView", "ModelSpec", "RunMixedJobs", "SetWorkerDevice", "Status", "SubgraphKey", "WorkerDevice"]
