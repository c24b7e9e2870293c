"""GEMM shapes of the path (shared by the GEMM scripts): (name, M, N, K, act, out_bf16, resid)."""
SHAPES = [
    ("clip_fc1", 32896, 5120, 1280, "gelu", True, False),
    ("clip_fc1_noact", 32896, 5120, 1280, None, True, False),
    ("clip_fc2", 32896, 1280, 5120, None, False, True),
    ("clip_fc2_nores", 32896, 1280, 5120, None, False, False),
    ("clip_fc2_bf16", 32896, 1280, 5120, None, True, False),
    ("fc2_m256x", 32768, 1280, 5120, None, True, False),
    ("clip_qkv", 32896, 3840, 1280, None, True, False),
    ("clip_proj", 32896, 1280, 1280, None, False, True),
    ("clip_proj_nores", 32896, 1280, 1280, None, False, False),
    ("cutr_qkv_win", 36864, 2304, 768, None, True, False),
    ("cutr_fc1", 25600, 3072, 768, "gelu", True, False),
    ("cutr_fc2", 25600, 768, 3072, None, False, True),
    ("sq4096", 4096, 4096, 4096, None, True, False),
    ("sq8192", 8192, 8192, 8192, None, True, False),
]
