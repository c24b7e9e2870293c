"""The C-ABI library builds for gfx950, loads without a GPU, and exports every entry point that
include/boxfusion_hip.h declares (no compute calls here)."""
import ctypes
import os
import re

from boxfusion_amd import build as B

HEADER = os.path.join(os.path.dirname(B.HERE), "include", "boxfusion_hip.h")


def declared():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\*|int|size_t)\s+(bf_\w+)\s*\(", src, re.M)))


def test_header_declares_entry_points():
    names = declared()
    for must in ["bf_obb_iou_matrix", "bf_nms_scan", "bf_corr_assoc", "bf_fusion_fit",
                 "bf_depth_standardize", "bf_backproject", "bf_box_corners"]:
        assert must in names


def test_library_exports_all_symbols():
    path = B.build()
    lib = ctypes.CDLL(path)
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    lib.bf_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.bf_version()
