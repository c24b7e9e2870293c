"""Where the colour-JPEG entropy decode's time goes: the JPG_STATS diagnostic build's per-file stamps
(shader clock, 100-MHz real time) and counters (rounds of the speculative walk, tokens, slow-path
tokens, ring refills and their cycles, blocks).
usage: BF_LIB_PATH=boxfusion_amd/_build/var_jpg_stats/libboxfusion_hip.so python scripts/probe/jpeg_stats_probe.py [F] [quality]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    q = int(sys.argv[2]) if len(sys.argv) > 2 else 90
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    from scripts.jpeg_bench import H, W, make_jpegs
    L = _lib.lib()
    pool = make_jpegs(quality=q)
    blobs = [pool[i % len(pool)] for i in range(F)]
    files, offs, _ = upload_files(blobs, "cuda")
    for _ in range(2):
        _lib.jpeg_decode_rgb(files, offs, H, W)
        torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (12 * F))()
    assert L.bf_jpeg_read_stats(buf, F) == 0
    a = np.frombuffer(buf, np.uint64).reshape(F, 12).astype(np.float64)
    cyc, rt = a[:, 0], a[:, 1] * 10.0
    rounds, tok, slow, nprod, cprod, blk = a[:, 2], a[:, 3], a[:, 4], a[:, 5], a[:, 6], a[:, 7]
    print(f"{F} files q{q}, {np.mean([len(b) for b in blobs]) / 1e3:.0f} KB")
    print(f"entropy: {rt.mean() / 1e6:.2f} ms/file (max {rt.max() / 1e6:.2f}), clock {np.mean(cyc / rt) * 1e3:.0f} MHz, "
          f"{rounds.mean():.0f} rounds, {tok.mean():.0f} tokens ({tok.mean() / rounds.mean():.2f}/round), "
          f"{slow.mean():.0f} slow, {blk.mean():.0f} blocks; {cyc.mean() / rounds.mean():.0f} cycles/round, "
          f"{cyc.mean() / tok.mean():.0f} cycles/token; refills {nprod.mean():.0f} taking {cprod.mean() / cyc.mean() * 100:.1f}%; "
          f"lane tokens {a[:, 8].mean() / rounds.mean():.0f} cycles/round (incl. refills), walk {a[:, 9].mean() / rounds.mean():.0f}; "
          f"{a[:, 10].mean() / rounds.mean():.2f} chain segments/round, placement {a[:, 11].mean() / a[:, 10].mean():.0f} cycles/segment")


if __name__ == "__main__":
    main()
