"""TEST INFRASTRUCTURE ONLY — the CPU oracle of the depth PNG decode (`bf_png_decode_u16`).

Restates what cv2.imread(depth_path, cv2.IMREAD_UNCHANGED) returns for the reference's depth
files (/root/reference/boxfusion/capture_stream.py:197 ScanNet, :405 CA-1M): a 16-bit greyscale
PNG as uint16 [H, W].  cv2 decodes through libpng + zlib; this file uses the same zlib (Python's
`zlib` module, the library the reference's decoder links) for the inflate and restates PNG 1.2 §6
(row filters None / Sub / Up / Average / Paeth, bytes per pixel 2) and the chunk layout by hand.
Pinned against PIL's decoder (libpng-equivalent) in tests/test_png_oracle.py on the fixtures of
tests/golden/png_fixtures.npz (made by tests/golden/make_png_fixtures.py).  Only tests/, smoke()
and bench.py's cpu_baseline may import it.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIG = b"\x89PNG\r\n\x1a\n"


def chunks(data: bytes):
    """(type, payload) of every chunk, in file order (PNG 1.2 §5.3)"""
    if data[:8] != SIG:
        raise ValueError("not a PNG")
    pos = 8
    while pos + 12 <= len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        t = data[pos + 4:pos + 8]
        if pos + 12 + n > len(data):
            raise ValueError("truncated chunk")
        yield t, data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if t == b"IEND":
            return


def paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    if pa <= pb and pa <= pc:
        return a
    return b if pb <= pc else c


def unfilter(raw: bytes, H: int, W: int, bpp: int = 2) -> np.ndarray:
    """filtered scanlines (1 type byte + W*bpp bytes per row) -> unfiltered bytes [H, W*bpp]"""
    S = W * bpp + 1
    out = np.zeros((H, W * bpp), np.int64)
    prev = np.zeros(W * bpp, np.int64)
    for r in range(H):
        ft = raw[r * S]
        f = np.frombuffer(raw, np.uint8, W * bpp, r * S + 1).astype(np.int64)
        cur = np.zeros(W * bpp, np.int64)
        if ft == 0:
            cur = f.copy()
        elif ft == 2:
            cur = (f + prev) & 255
        elif ft in (1, 3, 4):
            for i in range(W * bpp):
                a = int(cur[i - bpp]) if i >= bpp else 0
                b = int(prev[i])
                c = int(prev[i - bpp]) if i >= bpp else 0
                p = a if ft == 1 else (a + b) >> 1 if ft == 3 else paeth(a, b, c)
                cur[i] = (int(f[i]) + p) & 255
        else:
            raise ValueError(f"bad filter type {ft}")
        out[r] = cur
        prev = cur
    return out.astype(np.uint8)


def decode_u16(data: bytes) -> np.ndarray:
    """16-bit greyscale non-interlaced PNG -> uint16 [H, W] (big-endian samples, PNG 1.2 §7.1)"""
    ihdr = None
    idat = b""
    for t, d in chunks(data):
        if t == b"IHDR":
            ihdr = struct.unpack(">IIBBBBB", d)
        elif t == b"IDAT":
            idat += d
    if ihdr is None:
        raise ValueError("no IHDR")
    W, H, depth, ctype, _, _, interlace = ihdr
    if depth != 16 or ctype != 0 or interlace != 0:
        raise ValueError("not 16-bit greyscale")
    raw = zlib.decompress(idat)
    if len(raw) != H * (2 * W + 1):
        raise ValueError("inflated size")
    b = unfilter(raw, H, W, 2).reshape(H, W, 2).astype(np.uint16)
    return (b[..., 0] << 8) | b[..., 1]


def encode_u16(img: np.ndarray, filters=None, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, idat_size=8192,
               extra_chunks=()) -> bytes:
    """a 16-bit greyscale PNG of img with the given row filter types (a list, one per row, or an
    int; None = 0) and zlib settings — test input with every filter and block kind forced"""
    H, W = img.shape
    be = img.astype(">u2").tobytes()
    S = 2 * W
    rows = [np.frombuffer(be, np.uint8, S, r * S).astype(np.int64) for r in range(H)]
    fl = [filters if isinstance(filters, int) else (filters[r] if filters is not None else 0) for r in range(H)]
    out = bytearray()
    prev = np.zeros(S, np.int64)
    for r in range(H):
        x, ft = rows[r], fl[r]
        a = np.concatenate([[0, 0], x[:-2]])
        c = np.concatenate([[0, 0], prev[:-2]])
        if ft == 0:
            f = x
        elif ft == 1:
            f = x - a
        elif ft == 2:
            f = x - prev
        elif ft == 3:
            f = x - ((a + prev) >> 1)
        else:
            f = x - np.array([paeth(int(a[i]), int(prev[i]), int(c[i])) for i in range(S)])
        out.append(ft)
        out += (f & 255).astype(np.uint8).tobytes()
        prev = x
    co = zlib.compressobj(level, zlib.DEFLATED, 15, 9, strategy)
    z = co.compress(bytes(out)) + co.flush()

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)

    png = SIG + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 16, 0, 0, 0, 0))
    for t, d in extra_chunks:
        png += chunk(t, d)
    step = max(1, idat_size)
    for i in range(0, len(z), step):
        png += chunk(b"IDAT", z[i:i + step])
    return png + chunk(b"IEND", b"")
