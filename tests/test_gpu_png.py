"""GPU depth-PNG decode (bf_png.hip) bit-exact against PIL (the libpng-equivalent decoder standing
in for the reference's cv2.imread(..., IMREAD_UNCHANGED), capture_stream.py:197/:405) and the
oracle restatement (oracle/png.py): the committed fixtures (every row filter, stored / fixed /
dynamic blocks, split IDATs, ancillary chunks, 1-pixel and 1-row images), full-size 640 x 480
depth maps from PIL's encoder at every compress level and from the forced-filter encoder, mixed
batches with corrupt files (each flagged with its own status bit, the good files still exact), and
DecodedFrameStream reading PNG files from disk."""
import io
import os
import zlib

import numpy as np
import pytest
import torch
from PIL import Image

from oracle import png as P

pytestmark = pytest.mark.gpu

FIX = os.path.join(os.path.dirname(__file__), "golden", "png_fixtures.npz")


@pytest.fixture(scope="module")
def L():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from boxfusion_amd import _lib
    _lib.lib()
    return _lib


def fixtures():
    z = np.load(FIX)
    n = sum(1 for k in z.files if k.startswith("png_"))
    return [(str(z[f"name_{i}"]), z[f"png_{i}"].tobytes(), z[f"img_{i}"]) for i in range(n)]


def decode(L, blobs, H, W, check=True):
    from boxfusion_amd.capture_stream import upload_files
    files, offs, offs_h = upload_files(blobs, "cuda")
    out, st = L.png_decode_u16(files, offs, H, W, offsets_host=offs_h, check=check)
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy()


def pil(png):
    return np.asarray(Image.open(io.BytesIO(png)))


@pytest.mark.parametrize("name,png,img", fixtures(), ids=lambda v: v if isinstance(v, str) else "")
def test_fixture_bit_exact(L, name, png, img):
    H, W = img.shape
    got, st = decode(L, [png], H, W)
    assert st.tolist() == [0]
    np.testing.assert_array_equal(got[0], img, err_msg=name)


def test_fixture_batch_same_size(L):
    """every 48 x 64 fixture in one launch (one wave per file)"""
    fx = [(n, p, i) for n, p, i in fixtures() if i.shape == (48, 64)]
    assert len(fx) >= 15
    got, st = decode(L, [p for _, p, _ in fx], 48, 64)
    assert not st.any()
    for k, (n, _, img) in enumerate(fx):
        np.testing.assert_array_equal(got[k], img, err_msg=n)


def _depth_frames(n, H=480, W=640):
    from boxfusion_amd.synthetic import frame_rgbd
    out = []
    for f in range(n):
        d = frame_rgbd(f * 7, H, W)[1]
        out.append(np.clip(d * 1000.0, 0, 65535).astype(np.uint16))
    return out


def test_full_size_depth_pil_levels(L):
    """640 x 480 depth maps as PIL writes them (adaptive filters) at compress levels 0-9"""
    imgs = _depth_frames(10)
    blobs = []
    for k, img in enumerate(imgs):
        b = io.BytesIO()
        Image.fromarray(img).save(b, format="PNG", compress_level=k)
        blobs.append(b.getvalue())
    got, st = decode(L, blobs, 480, 640)
    assert not st.any()
    for k, (png, img) in enumerate(zip(blobs, imgs)):
        np.testing.assert_array_equal(got[k], img, err_msg=f"level {k}")
        np.testing.assert_array_equal(got[k], pil(png))
    # fused depth scaling (bf_png_decode_depth): astype(float32) / depth_scale, IEEE f32
    from boxfusion_amd.capture_stream import upload_files
    files, offs, offs_h = upload_files(blobs, "cuda")
    for scale in (1000.0, 6553.5):
        dep, st = L.png_decode_u16(files, offs, 480, 640, offsets_host=offs_h, depth_scale=scale)
        want = np.stack(imgs).astype(np.float32) / np.float32(scale)
        np.testing.assert_array_equal(dep.cpu().numpy(), want)


def test_full_size_forced_filters(L):
    """Average and Paeth on every row (PIL's encoder rarely picks Average), Huffman-only / RLE /
    fixed blocks, 1 KiB IDAT chunks; one frame with a quantised depth (long zero and repeat runs)"""
    imgs = _depth_frames(6)
    imgs[5] = (imgs[5] // 50) * 50
    rng = np.random.default_rng(0)
    specs = [dict(filters=3), dict(filters=4), dict(filters=list(rng.integers(0, 5, 480)), strategy=zlib.Z_HUFFMAN_ONLY),
             dict(filters=1, strategy=zlib.Z_RLE, idat_size=1024), dict(filters=4, strategy=zlib.Z_FIXED, level=9),
             dict(filters=2, level=9)]
    blobs = [P.encode_u16(img, **sp) for img, sp in zip(imgs, specs)]
    got, st = decode(L, blobs, 480, 640)
    assert not st.any()
    for k, (png, img) in enumerate(zip(blobs, imgs)):
        np.testing.assert_array_equal(got[k], img, err_msg=str(specs[k]))
        np.testing.assert_array_equal(got[k], pil(png))


def test_oracle_agrees_full_size(L):
    img = _depth_frames(1)[0][:96]
    png = P.encode_u16(img, filters=list(np.random.default_rng(1).integers(0, 5, 96)))
    got, _ = decode(L, [png], 96, 640)
    np.testing.assert_array_equal(got[0], P.decode_u16(png))


def _with_payload(png, mutate):
    """rebuild a PNG with its concatenated IDAT payload mutated (one IDAT chunk)"""
    import struct
    ch = list(P.chunks(png))
    z = bytearray(b"".join(d for t, d in ch if t == b"IDAT"))
    z = mutate(z)

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    out = P.SIG
    done = False
    for t, d in ch:
        if t == b"IDAT":
            if not done:
                out += chunk(t, bytes(z))
                done = True
        else:
            out += chunk(t, d)
    return out


def test_corrupt_files_flagged_good_files_exact(L):
    img = _depth_frames(1, 48, 64)[0]
    good = P.encode_u16(img, filters=4)

    def bad_filter(z):
        raw = bytearray(zlib.decompress(bytes(z)))
        raw[5 * 129] = 7
        return bytearray(zlib.compress(bytes(raw)))

    def bad_adler(z):
        z[-1] ^= 0x5a
        return z

    def bad_block(z):
        raw = zlib.compress(zlib.decompress(bytes(z)), 0)     # stored blocks: break LEN / NLEN
        raw = bytearray(raw)
        raw[5] ^= 0xff
        return raw

    def short(z):
        return bytearray(zlib.compress(zlib.decompress(bytes(z))[:-10]))

    b8 = io.BytesIO()
    Image.fromarray((img >> 8).astype(np.uint8)).save(b8, format="PNG")
    cases = [("good", good, 0),
             ("signature", b"\x00" + good[1:], 1),
             ("filter", _with_payload(good, bad_filter), 64),
             ("adler", _with_payload(good, bad_adler), 32),
             ("block", _with_payload(good, bad_block), 16),
             ("short", _with_payload(good, short), 128),
             ("size", P.encode_u16(img[:40], filters=1), 128),
             ("eight_bit", b8.getvalue(), 4),
             ("truncated", good[:len(good) // 2], 8),
             ("good2", P.encode_u16(img, filters=3, strategy=zlib.Z_FIXED), 0)]
    got, st = decode(L, [c[1] for c in cases], 48, 64, check=False)
    for k, (name, _, bit) in enumerate(cases):
        if bit == 0:
            assert st[k] == 0, name
            np.testing.assert_array_equal(got[k], img, err_msg=name)
        else:
            assert st[k] & bit, (name, st[k])
    with pytest.raises(L.HipError, match="did not decode"):
        decode(L, [good, cases[1][1]], 48, 64, check=True)


def test_decoded_frame_stream_reads_png_files(L, tmp_path):
    """DecodedFrameStream: depth PNG files decoded on the GPU in batches, then bf_ingest_rgbd:
    the sample depth equals the PIL-decoded file / depth_scale"""
    from boxfusion_amd.capture_stream import DecodedFrameStream
    from boxfusion_amd.synthetic import SCANNET_K, frame_rgbd
    cps, dps, deps = [], [], []
    for f in range(5):
        rgb, d = frame_rgbd(f, 480, 640)
        d16 = np.clip(d * 1000.0, 0, 65535).astype(np.uint16)
        cp, dp = tmp_path / f"{f}.jpg", tmp_path / f"{f}.png"
        Image.fromarray(rgb).save(cp, quality=95)
        Image.fromarray(d16).save(dp)
        cps.append(str(cp)); dps.append(str(dp)); deps.append(d16)
    up = np.eye(4, dtype=np.float32)
    up[1:3, :3] = [[0, 0, 1], [0, -1, 0]]           # camera y down the world z: the upright roll
    poses = [up] * 5
    for mode in ("gpu", "host"):
        stream = DecodedFrameStream(cps, dps, poses, SCANNET_K, 1000.0, device="cuda", batch=2, depth_decode=mode)
        n = 0
        for i, s in enumerate(stream):
            dep = s["wide"]["depth"]
            want = torch.from_numpy(deps[i].astype(np.float32) / np.float32(1000.0))
            torch.testing.assert_close(dep.reshape(480, 640).cpu(), want, rtol=0, atol=0)
            n += 1
        assert n == 5, mode
