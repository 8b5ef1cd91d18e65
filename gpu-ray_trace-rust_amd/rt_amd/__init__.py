"""rt_amd — host side of the MI355X path-tracing hot path (drop-in for the reference's
`use_gpu` branch, src/renderer.rs:51-60).  The compute is in lib/librt_amd.so (HIP, gfx950),
reached through the C ABI of include/rt_abi.h; this package only loads scenes and calls it."""
from . import abi  # noqa: F401
from .abi import load_library, RtError  # noqa: F401
