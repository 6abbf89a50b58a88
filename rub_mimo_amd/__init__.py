"""rub_mimo_amd -- MI355X (gfx950) OFDM-MIMO receive pipeline.

The drop-in boundary is the C-ABI of librub_mimo_amd.so (include/mimo_rx.h) and the C++
facade include/framing.h that mirrors /root/reference/mimo/framing.h. This package is the
Python host side: `framing` mirrors the reference classes, `receiver` drives the batched
device-resident path the benchmark times. All compute runs in the library's HIP kernels.
"""
from ._lib import (DET_MMSE, DET_SISO, DET_ZF, DET_ZF2, FRAME_INCOMPLETE, FRAME_NO_SYNC,
                   FRAME_OK, DeviceBuffer, MimoError, device_count, lib)

__all__ = ["lib", "DeviceBuffer", "MimoError", "device_count", "DET_ZF2", "DET_ZF", "DET_MMSE",
           "DET_SISO", "FRAME_OK", "FRAME_NO_SYNC", "FRAME_INCOMPLETE"]
__version__ = "0.1.0"
