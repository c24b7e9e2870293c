"""Where the depth-PNG decode's time goes: the PNG_STATS diagnostic build's per-file stamps
(shader clock and 100-MHz real time around k_png_inflate and k_png_unfilter) and counters
(rounds of the speculative token walk, tokens, bit-serial tokens, matches).
usage: BF_LIB_PATH=boxfusion_amd/_build/var_png_stats/libboxfusion_hip.so python scripts/probe/png_stats_probe.py [F]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def main():
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    from boxfusion_amd import _lib
    from boxfusion_amd.capture_stream import upload_files
    from scripts.png_bench import make_pngs
    L = _lib.lib()
    pool = make_pngs()
    pool_s = make_pngs(smooth=True)
    for name, blobs in (("pil_level6_noisy", [pool[i % len(pool)] for i in range(F)]),
                        ("pil_level6_smoothed", [pool_s[i % len(pool_s)] for i in range(F)])):
        files, offs, offs_h = upload_files(blobs, "cuda")
        for rep in range(2):
            out, st = _lib.png_decode_u16(files, offs, 480, 640, offsets_host=offs_h, depth_scale=1000.0)
            torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * (10 * F))()
        assert L.bf_png_read_stats(buf, F) == 0
        a = np.frombuffer(buf, np.uint64).reshape(F, 10).astype(np.float64)
        cyc, rt, rounds, tok, slow, match = a[:, 0], a[:, 1] * 10.0, a[:, 2], a[:, 3], a[:, 4], a[:, 5]
        ucyc, urt = a[:, 6], a[:, 7] * 10.0
        print(f"{name}: {F} files, {np.mean([len(b) for b in blobs]) / 1e3:.0f} KB")
        print(f"  inflate: {rt.mean() / 1e6:.2f} ms/file (max {rt.max() / 1e6:.2f}), clock {np.mean(cyc / rt) * 1e3:.0f} MHz, "
              f"{rounds.mean():.0f} rounds, {tok.mean():.0f} tokens ({tok.mean() / rounds.mean():.2f}/round), "
              f"{slow.mean():.0f} bit-serial, {match.mean():.0f} matches; "
              f"{cyc.mean() / rounds.mean():.0f} cycles/round, {cyc.mean() / tok.mean():.0f} cycles/token")
        print(f"  unfilter: {urt.mean() / 1e6:.2f} ms/file, clock {np.mean(ucyc / urt) * 1e3:.0f} MHz, "
              f"{ucyc.mean() / (480 / 64 * (640 + 63)):.0f} cycles/step")


if __name__ == "__main__":
    main()
