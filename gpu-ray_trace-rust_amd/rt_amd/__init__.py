"""rt_amd — host side of the MI355X path-tracing hot path (drop-in for the reference's
`use_gpu` branch, src/renderer.rs:51-60).  The compute is in lib/librt_amd.so (HIP, gfx950),
reached through the C ABI of include/rt_abi.h; this package only loads scenes and calls it."""
import os

# Overlapped queue launches run on up to 8 pipeline streams (runtime.hip, launch pipeline); HIP
# maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default, and often exported as 4),
# and streams sharing a queue run one after another.  HIP reads it when it starts, so it is
# raised to at least 12 here, before the first HIP call of the process (a380 at its batch of
# 1 spp: 4 queues 183, 12 queues 313 Msamples/s).  Higher values are kept.
_HW_QUEUES = 12
try:
    _q = int(os.environ.get("GPU_MAX_HW_QUEUES", "0"))
except ValueError:
    _q = 0
if _q < _HW_QUEUES:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_HW_QUEUES)
from . import abi  # noqa: F401
from .abi import load_library, RtError  # noqa: F401
