"""TEST INFRASTRUCTURE ONLY — the CPU oracle of the colour JPEG decode (`bf_jpeg_decode_rgb`).

Restates what cv2.imread(color_path) (/root/reference/boxfusion/capture_stream.py:194, :402)
returns for a baseline JPEG before its BGR->RGB swap: libjpeg(-turbo)'s default decompression --
sequential Huffman decode (ITU T.81 F.2), dequantisation, the accurate integer inverse DCT
(libjpeg's `jidctint.c` "islow": CONST_BITS 13, PASS1_BITS 2, the post-IDCT range-limit table of
`jdmaster.c`), "fancy" triangle upsampling of subsampled chroma (`jdsample.c` h2v1 / h2v2, context
rows replicated at the image edges) and the fixed-point YCbCr->RGB tables of `jdcolor.c`
(SCALEBITS 16).  cv2 is absent here, so the restatement is pinned against PIL's decoder (the same
libjpeg-turbo library with the same default parameters) on the fixtures of
tests/golden/jpeg_fixtures.npz (tests/golden/make_jpeg_fixtures.py; tests/test_jpeg_oracle.py).
Pure Python: small images only.  Only tests/, smoke() and bench.py's cpu_baseline may import it.
"""
from __future__ import annotations

import numpy as np

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27,
                   20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58,
                   59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], np.int64)   # zigzag k -> natural


class JpegError(ValueError):
    pass


def parse(data: bytes):
    """markers -> dict(q={id: [64] natural order}, frame=(H, W, comps[(id, h, v, tq)]), dc/ac
    huffman tables {id: (counts[16], values)}, dri, scans=[(comp idx list, td, ta, entropy bytes)])"""
    if data[:2] != b"\xff\xd8":
        raise JpegError("no SOI")
    pos = 2
    q, dc, ac, scans = {}, {}, {}, []
    frame, dri = None, 0
    while pos + 4 <= len(data):
        if data[pos] != 0xFF:
            raise JpegError("marker expected")
        m = data[pos + 1]
        if m == 0xFF:
            pos += 1
            continue
        if m == 0xD9:
            break
        ln = int.from_bytes(data[pos + 2:pos + 4], "big")
        seg = data[pos + 4:pos + 2 + ln]
        if m == 0xDB:
            i = 0
            while i < len(seg):
                pq, tq = seg[i] >> 4, seg[i] & 15
                i += 1
                if pq:
                    vals = np.frombuffer(seg[i:i + 128], ">u2").astype(np.int64)
                    i += 128
                else:
                    vals = np.frombuffer(seg[i:i + 64], np.uint8).astype(np.int64)
                    i += 64
                nat = np.zeros(64, np.int64)
                nat[ZIGZAG] = vals
                q[tq] = nat
        elif m in (0xC0, 0xC1):
            if seg[0] != 8:
                raise JpegError("not 8-bit")
            H, W, nf = int.from_bytes(seg[1:3], "big"), int.from_bytes(seg[3:5], "big"), seg[5]
            comps = [(seg[6 + 3 * c], seg[7 + 3 * c] >> 4, seg[7 + 3 * c] & 15, seg[8 + 3 * c]) for c in range(nf)]
            frame = (H, W, comps)
        elif m in (0xC2, 0xC3, 0xC5, 0xC6, 0xC7, 0xC9, 0xCA, 0xCB, 0xCD, 0xCE, 0xCF):
            raise JpegError("not baseline / extended sequential Huffman")
        elif m == 0xC4:
            i = 0
            while i < len(seg):
                tc, th = seg[i] >> 4, seg[i] & 15
                counts = list(seg[i + 1:i + 17])
                n = sum(counts)
                vals = list(seg[i + 17:i + 17 + n])
                (ac if tc else dc)[th] = (counts, vals)
                i += 17 + n
        elif m == 0xDD:
            dri = int.from_bytes(seg[0:2], "big")
        elif m == 0xDA:
            ns = seg[0]
            ids = [seg[1 + 2 * k] for k in range(ns)]
            tabs = [(seg[2 + 2 * k] >> 4, seg[2 + 2 * k] & 15) for k in range(ns)]
            cidx = [[c[0] for c in frame[2]].index(i) for i in ids]
            # entropy-coded data up to the next marker that is not RSTn / stuffing
            e = pos + 2 + ln
            j = e
            while j + 1 < len(data):
                if data[j] == 0xFF and data[j + 1] not in (0, 0xFF) and not (0xD0 <= data[j + 1] <= 0xD7):
                    break
                j += 1
            scans.append((cidx, tabs, data[e:j]))
            pos = j
            continue
        pos += 2 + ln
    if frame is None or not scans:
        raise JpegError("no frame / scan")
    return dict(q=q, frame=frame, dc=dc, ac=ac, dri=dri, scans=scans)


def _huff(counts, vals):
    """canonical code -> {(length, code): value}"""
    out, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(counts[ln - 1]):
            out[(ln, code)] = vals[k]
            code += 1
            k += 1
        code <<= 1
    return out


class _Bits:
    """MSB-first reader over entropy data: FF 00 -> FF, RSTn markers seen between intervals"""

    def __init__(self, b: bytes):
        self.b, self.p, self.acc, self.n = b, 0, 0, 0

    def bit(self):
        if self.n == 0:
            if self.p >= len(self.b):
                v = 0                          # past the end: zeros (libjpeg inserts zeros too)
            else:
                v = self.b[self.p]
                if v == 0xFF:                  # jdhuff.c: skip a run of FF (fill bytes), read what follows
                    q = self.p + 1
                    while q < len(self.b) and self.b[q] == 0xFF:
                        q += 1
                    nx = self.b[q] if q < len(self.b) else 0
                    if nx == 0:
                        self.p = q             # FF (FF ...) 00 -> one FF data byte
                    else:                      # a marker: do not consume; feed zeros
                        v = 0
                        self.p -= 1
                self.p += 1
            self.acc, self.n = v, 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, s):
        v = 0
        for _ in range(s):
            v = (v << 1) | self.bit()
        return v

    def restart(self):
        """byte-align and skip an RSTn marker"""
        self.n = 0
        q = self.p
        while q < len(self.b) and self.b[q] == 0xFF:   # fill bytes before the marker
            q += 1
        if q > self.p and q < len(self.b) and 0xD0 <= self.b[q] <= 0xD7:
            self.p = q + 1


def _decode(bs, table):
    code = 0
    for ln in range(1, 17):
        code = (code << 1) | bs.bit()
        v = table.get((ln, code))
        if v is not None:
            return v
    raise JpegError("bad Huffman code")


def _extend(v, s):
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def coefficients(j):
    """quantised coefficients per component: list of int64 [by, bx, 64] (natural order)"""
    H, W, comps = j["frame"]
    hmax, vmax = max(c[1] for c in comps), max(c[2] for c in comps)
    mcux, mcuy = -(-W // (8 * hmax)), -(-H // (8 * vmax))
    out = [np.zeros((mcuy * c[2], mcux * c[1], 64), np.int64) for c in comps]
    for cidx, tabs, ent in j["scans"]:
        bs = _Bits(ent)
        dct = [_huff(*j["dc"][t[0]]) for t in tabs]
        act = [_huff(*j["ac"][t[1]]) for t in tabs]
        pred = [0] * len(cidx)
        if len(cidx) == 1:               # non-interleaved: the component's own block grid
            c = comps[cidx[0]]
            bw = -(-(-(-W * c[1] // hmax)) // 8)
            bh = -(-(-(-H * c[2] // vmax)) // 8)
            units = [[(cidx[0], by, bx)] for by in range(bh) for bx in range(bw)]
        else:
            units = []
            for my in range(mcuy):
                for mx in range(mcux):
                    u = []
                    for ci in cidx:
                        c = comps[ci]
                        for v in range(c[2]):
                            for h in range(c[1]):
                                u.append((ci, my * c[2] + v, mx * c[1] + h))
                    units.append(u)
        for n, unit in enumerate(units):
            if j["dri"] and n and n % j["dri"] == 0:
                bs.restart()
                pred = [0] * len(cidx)
            for ci, by, bx in unit:
                k = cidx.index(ci)
                blk = np.zeros(64, np.int64)
                s = _decode(bs, dct[k])
                pred[k] += _extend(bs.bits(s), s)
                blk[0] = pred[k]
                i = 1
                while i < 64:
                    rs = _decode(bs, act[k])
                    r, s = rs >> 4, rs & 15
                    if s:
                        i += r
                        if i > 63:
                            raise JpegError("AC index past 63")
                        blk[ZIGZAG[i]] = _extend(bs.bits(s), s)
                        i += 1
                    elif r == 15:
                        i += 16
                    else:
                        break
                out[ci][by, bx] = blk
    return out


def _range_limit(v):
    """jdmaster.c post-IDCT range-limit table indexed by v & 1023 (v centred at 0)"""
    idx = v & 1023
    return np.where(idx < 128, idx + 128, np.where(idx < 512, 255, np.where(idx < 896, 0, idx - 896)))


def idct_islow(coef, qt):
    """jidctint.c jpeg_idct_islow on [..., 64] quantised coefficients (natural order) -> u8 [..., 8, 8]"""
    CB, P1 = 13, 2

    def fix(x):
        return int(x * (1 << CB) + 0.5)
    F = {k: fix(v) for k, v in dict(f0298=0.298631336, f0390=0.390180644, f0541=0.541196100,
                                    f0765=0.765366865, f0899=0.899976223, f1175=1.175875602,
                                    f1501=1.501321110, f1847=1.847759065, f1961=1.961570560,
                                    f2053=2.053119869, f2562=2.562915447, f3072=3.072711026).items()}

    def descale(x, n):
        return (x + (1 << (n - 1))) >> n

    def pass_(z0, z1, z2, z3, z4, z5, z6, z7):
        # even part
        a = z2
        b = z6
        z1e = (a + b) * F["f0541"]
        t2 = z1e + b * (-F["f1847"])
        t3 = z1e + a * F["f0765"]
        t0 = (z0 + z4) << CB
        t1 = (z0 - z4) << CB
        t10, t13, t11, t12 = t0 + t3, t0 - t3, t1 + t2, t1 - t2
        # odd part
        o0, o1, o2, o3 = z7, z5, z3, z1
        zz1, zz2, zz3, zz4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
        zz5 = (zz3 + zz4) * F["f1175"]
        o0 = o0 * F["f0298"]
        o1 = o1 * F["f2053"]
        o2 = o2 * F["f3072"]
        o3 = o3 * F["f1501"]
        zz1 = zz1 * (-F["f0899"])
        zz2 = zz2 * (-F["f2562"])
        zz3 = zz3 * (-F["f1961"]) + zz5
        zz4 = zz4 * (-F["f0390"]) + zz5
        o0 += zz1 + zz3
        o1 += zz2 + zz4
        o2 += zz2 + zz3
        o3 += zz1 + zz4
        return (t10 + o3, t11 + o2, t12 + o1, t13 + o0, t13 - o0, t12 - o1, t11 - o2, t10 - o3)

    c = (coef * qt).reshape(coef.shape[:-1] + (8, 8)).astype(np.int64)   # [.., row(v), col(u)]
    # pass 1: columns (over rows v) -> workspace, scaled by 2^PASS1_BITS
    cols = pass_(*[c[..., v, :] for v in range(8)])
    ws = np.stack([descale(x, CB - P1) for x in cols], axis=-2)           # [.., 8 rows, 8 cols]
    # pass 2: rows (over columns u)
    rows = pass_(*[ws[..., :, u] for u in range(8)])
    out = np.stack([descale(x, CB + P1 + 3) for x in rows], axis=-1)
    return _range_limit(out).astype(np.uint8)


def planes(j, coefs):
    """component sample planes u8 at their (padded) block-grid size"""
    out = []
    for ci, c in enumerate(j["frame"][2]):
        blocks = idct_islow(coefs[ci], j["q"][c[3]])           # [by, bx, 8, 8]
        by, bx = blocks.shape[:2]
        out.append(blocks.transpose(0, 2, 1, 3).reshape(by * 8, bx * 8))
    return out


def upsample(plane, h, v, hmax, vmax, cw, ch):
    """jdsample.c fancy upsampling of a downsampled plane (real size cw x ch) -> full resolution
    (2cw x 2ch for h2v2, 2cw x ch for h2v1; fullsize copy otherwise)"""
    p = plane[:ch, :cw].astype(np.int64)
    if (hmax // h, vmax // v) == (1, 1):
        return p
    if (hmax // h, vmax // v) == (2, 1):          # h2v1_fancy_upsample
        out = np.zeros((ch, 2 * cw), np.int64)
        if cw == 1:
            out[:, 0] = out[:, 1] = p[:, 0]
            return out
        out[:, 0] = p[:, 0]
        out[:, 1] = (p[:, 0] * 3 + p[:, 1] + 2) >> 2
        m = p[:, 1:-1] * 3
        out[:, 2:-2:2] = (m + p[:, :-2] + 1) >> 2
        out[:, 3:-2:2] = (m + p[:, 2:] + 2) >> 2
        out[:, -2] = (p[:, -1] * 3 + p[:, -2] + 1) >> 2
        out[:, -1] = p[:, -1]
        return out
    if (hmax // h, vmax // v) == (2, 2):          # h2v2_fancy_upsample, edge rows replicated
        up = np.concatenate([p[:1], p[:-1]], 0)
        dn = np.concatenate([p[1:], p[-1:]], 0)
        out = np.zeros((2 * ch, 2 * cw), np.int64)
        for r, nb in ((0, up), (1, dn)):
            s = p * 3 + nb                       # column sums
            o = np.zeros((ch, 2 * cw), np.int64)
            if cw == 1:
                o[:, 0] = (s[:, 0] * 4 + 8) >> 4
                o[:, 1] = (s[:, 0] * 4 + 7) >> 4
            else:
                o[:, 0] = (s[:, 0] * 4 + 8) >> 4
                o[:, 1] = (s[:, 0] * 3 + s[:, 1] + 7) >> 4
                o[:, 2:-2:2] = (s[:, 1:-1] * 3 + s[:, :-2] + 8) >> 4
                o[:, 3:-2:2] = (s[:, 1:-1] * 3 + s[:, 2:] + 7) >> 4
                o[:, -2] = (s[:, -1] * 3 + s[:, -2] + 8) >> 4
                o[:, -1] = (s[:, -1] * 4 + 7) >> 4
            out[r::2] = o
        return out
    raise JpegError(f"unsupported sampling {(hmax // h, vmax // v)}")


def ycc_rgb(y, cb, cr):
    """jdcolor.c ycc_rgb_convert (SCALEBITS 16), clamped with the simple range-limit table"""
    SB = 16
    half = 1 << (SB - 1)

    def fix(x):
        return int(x * (1 << SB) + 0.5)
    x = np.arange(256, dtype=np.int64) - 128
    cr_r = (fix(1.40200) * x + half) >> SB
    cb_b = (fix(1.77200) * x + half) >> SB
    cr_g = -fix(0.71414) * x
    cb_g = -fix(0.34414) * x + half
    r = np.clip(y + cr_r[cr], 0, 255)
    g = np.clip(y + ((cb_g[cb] + cr_g[cr]) >> SB), 0, 255)
    b = np.clip(y + cb_b[cb], 0, 255)
    return np.stack([r, g, b], -1).astype(np.uint8)


def decode_rgb(data: bytes) -> np.ndarray:
    """baseline JPEG -> u8 [H, W, 3] RGB (greyscale: the sample replicated, as PIL's convert("RGB"))"""
    j = parse(data)
    H, W, comps = j["frame"]
    pl = planes(j, coefficients(j))
    hmax, vmax = max(c[1] for c in comps), max(c[2] for c in comps)
    full = []
    for p, c in zip(pl, comps):
        cw, ch = -(-W * c[1] // hmax), -(-H * c[2] // vmax)
        full.append(upsample(p, c[1], c[2], hmax, vmax, cw, ch)[:H, :W])
    if len(comps) == 1:
        g = full[0].astype(np.uint8)
        return np.stack([g, g, g], -1)
    if len(comps) != 3:
        raise JpegError("1 or 3 components")
    return ycc_rgb(full[0], full[1], full[2])
