"""viso_amd — MI355X-native (gfx950) hot path of the Seasandwpy/viso
visual-odometry engine, behind the C ABI of include/viso/viso_c.h.

Everything that touches pixels or points runs in hand-written HIP kernels in
``viso_amd/libviso_amd.so``; this package is the thin host mirror of the
reference interface.  There is no CPU fallback.
"""
from . import _lib  # noqa: F401
from .api import Context, default_context, default_params, pyramid_dims  # noqa: F401
from .frontend import FrameHandler, FrameSequence, Keyframe, Viso  # noqa: F401

# viso_params.precision (include/viso/viso_c.h)
PRECISION_FAITHFUL = 0
PRECISION_FAST = 1

__all__ = ["PRECISION_FAITHFUL", "PRECISION_FAST", "Context", "default_context", "default_params", "pyramid_dims", "Viso", "Keyframe",
           "FrameSequence", "FrameHandler"]
