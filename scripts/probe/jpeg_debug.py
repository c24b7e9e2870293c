"""Debug probe: decode one JPEG fixture on the GPU and compare its workspace coefficients and
output with the oracle's stages.  usage: python scripts/probe/jpeg_debug.py NAME"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    from oracle import jpeg as J
    from tests.test_jpeg_oracle import fixtures
    name = sys.argv[1]
    jpg, img = next((j, i) for n, j, i in fixtures() if n == name)
    H, W = img.shape[:2]
    files, offs, _ = upload_files([jpg], "cuda")
    wb = _lib.jpeg_workspace_bytes(1, H, W)
    work = torch.zeros(wb, dtype=torch.uint8, device="cuda")
    out, st = _lib.jpeg_decode_rgb(files, offs, H, W, work=work, check=False)
    torch.cuda.synchronize()
    print("status", st.tolist())
    got = out[0].cpu().numpy()
    bad = np.argwhere((got != img).any(-1))
    print("mismatched pixels", len(bad), "first", bad[:5].tolist(), "rows", sorted(set(bad[:, 0].tolist()))[:40])
    P = J.parse(jpg)
    co = J.coefficients(P)
    w = work.cpu().numpy()
    coef = w[3072:].view(np.int16)
    off = 0
    for ci, c in enumerate(co):
        n = c.shape[0] * c.shape[1]
        g = coef[off * 64:(off + n) * 64].reshape(c.shape)
        d = np.argwhere((g != c).any(-1))
        print("comp", ci, c.shape, "bad blocks", len(d), d[:5].tolist())
        off += n


if __name__ == "__main__":
    main()
