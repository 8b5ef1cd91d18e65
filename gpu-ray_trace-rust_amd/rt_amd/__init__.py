"""rt_amd — host side of the MI355X path-tracing hot path (drop-in for the reference's
`use_gpu` branch, src/renderer.rs:51-60).  The compute is in lib/librt_amd.so (HIP, gfx950),
reached through the C ABI of include/rt_abi.h; this package only loads scenes and calls it."""
import os

# Overlapped queue launches run on up to 12 pipeline streams (runtime.hip, launch pipeline); HIP
# maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), and streams sharing a queue
# run one after another (a380 at its batch of 1 spp: 4 queues 183, 12 queues 356, 16 queues with
# 12 slots 400 Msamples/s).  HIP reads the variable when it starts, so when it is unset it is set
# to 16 here, before the first HIP call of the process; an explicit value is the caller's choice
# and is kept (the library then sizes its pipeline to it; bench.py and lib/rt_render choose 16
# themselves).  hw_queues() reports the value HIP started with, as far as this process can tell.
RECOMMENDED_HW_QUEUES = 16


def _hip_started() -> bool | None:
    import sys

    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return None


# Written only while HIP has not started: once it has, the queues are fixed, and a value written
# now would make the library size its pipeline for queues HIP never created (it reads the variable
# at rt_create as "what HIP started with").  Unset, the library assumes HIP's default of 4.
_HIP_STARTED_BEFORE = _hip_started()
_SET_BY_RT_AMD = "GPU_MAX_HW_QUEUES" not in os.environ and _HIP_STARTED_BEFORE is False
if _SET_BY_RT_AMD:
    os.environ["GPU_MAX_HW_QUEUES"] = str(RECOMMENDED_HW_QUEUES)
if _HIP_STARTED_BEFORE and "GPU_MAX_HW_QUEUES" not in os.environ:
    import warnings

    warnings.warn("rt_amd imported after HIP started: HIP runs with its default of 4 hardware queues, so "
                  "small batches overlap less (import rt_amd, or set GPU_MAX_HW_QUEUES, before using the GPU)")


def hw_queues() -> dict:
    """{"value": GPU_MAX_HW_QUEUES as set (None: HIP's default of 4), "source": "rt_amd" | "caller" |
    None, "hip_started_before_import": bool | None}."""
    v = os.environ.get("GPU_MAX_HW_QUEUES")
    return {"value": v, "source": "rt_amd" if _SET_BY_RT_AMD else ("caller" if v is not None else None),
            "hip_started_before_import": _HIP_STARTED_BEFORE}


from . import abi  # noqa: E402,F401
from .abi import load_library, RtError  # noqa: E402,F401
