"""blazingmq_amd -- MI355X-native replacement for BlazingMQ's per-message
CRC32C integrity-checksum path (bmqp::Crc32c and its batch callers).

The product is the C-ABI library ``lib/libbmqcrc.so`` (HIP kernels for gfx950
+ host dispatcher); this package is its Python host-side mirror.
"""
from .crc32c import (Blob, BmqCrcError, Crc32c, HostRegistration,  # noqa: F401
                     calculate_batch_multi, calculate_batch_ptr, device_count, fill_synthetic,
                     forget_shape, kernel_timing, last_launch, plan_wait, reserve)

__all__ = ["Blob", "BmqCrcError", "Crc32c", "HostRegistration", "calculate_batch_multi",
           "calculate_batch_ptr", "device_count", "fill_synthetic", "forget_shape", "plan_wait",
           "kernel_timing", "last_launch", "reserve"]
