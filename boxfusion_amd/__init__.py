"""boxfusion_amd — MI355X-native hot path of BoxFusion (per-frame detect + multi-view 3-D box
fusion).  Host code mirrors the reference's `boxfusion.*` API; compute runs in hand-written gfx950
HIP kernels behind the C-ABI in include/boxfusion_hip.h (libboxfusion_hip.so)."""

__version__ = "0.1.0"
