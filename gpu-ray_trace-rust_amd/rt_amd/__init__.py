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
_SET_BY_RT_AMD = "GPU_MAX_HW_QUEUES" not in os.environ
if _SET_BY_RT_AMD:
    os.environ["GPU_MAX_HW_QUEUES"] = str(RECOMMENDED_HW_QUEUES)


def hw_queues() -> dict:
    """{"value": GPU_MAX_HW_QUEUES as set, "source": "rt_amd" | "caller",
    "hip_started_before_import": bool | None} — with HIP already started when rt_amd was first
    imported the variable had no effect (HIP's default of 4 queues then applies)."""
    return {"value": os.environ.get("GPU_MAX_HW_QUEUES"), "source": "rt_amd" if _SET_BY_RT_AMD else "caller",
            "hip_started_before_import": _HIP_STARTED_BEFORE}


def _hip_started() -> bool | None:
    import sys

    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return None


_HIP_STARTED_BEFORE = _hip_started()
if _HIP_STARTED_BEFORE:
    import warnings

    warnings.warn("rt_amd imported after HIP started: GPU_MAX_HW_QUEUES has no effect, the launch "
                  "pipeline may share hardware queues (import rt_amd before using the GPU)")

from . import abi  # noqa: E402,F401
from .abi import load_library, RtError  # noqa: E402,F401
