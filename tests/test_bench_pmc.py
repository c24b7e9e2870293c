"""The bench line's PMC traffic records (bench.PMC_KEYS) resolve against the committed profiles
(CPU only: reads profiles/r*_pmc.json)."""
import glob
import os
import re

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _newest_round_pmc():
    fs = [f for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))
          if re.fullmatch(r"r\d+_pmc\.json", os.path.basename(f))]
    return max(fs, key=lambda f: int(re.match(r"r(\d+)", os.path.basename(f)).group(1)))


@pytest.mark.parametrize("name", sorted(k for k in bench.PMC_KEYS if k != "fp8_gemm"))
def test_pmc_key_resolves_in_newest_round(name):
    """every key of the default workload's roofline objects matches >= 1 kernel of the newest
    round's PMC record (a renamed kernel would silently drop out of a sum)"""
    newest = _newest_round_pmc()
    d = bench.load_pmc_traffic(bench.PMC_KEYS[name])
    assert d, name
    assert d["source"].startswith(os.path.relpath(newest, ROOT)), (name, d["source"])
    if bench.PMC_KEYS[name].startswith("sum:"):
        assert d["kernels"] >= 1


def test_pmc_fp8_key_resolves():
    """the fp8 line's traffic comes from the fp8 workload's own record of the newest round
    (profiles/r<N>_fp8_pmc.json), not from an older round's"""
    d = bench.load_pmc_traffic(bench.PMC_KEYS["fp8_gemm"])
    assert d
    n = int(re.match(r"r(\d+)", os.path.basename(_newest_round_pmc())).group(1))
    assert re.match(rf"profiles/r0*{n}_", d["source"]), d["source"]


def test_depth_pmc_sum_covers_every_pass_and_the_writes():
    """the 8-frame bf_depth_preprocess call: three histogram passes + the normalise pass, and at
    least the bytes the normalise pass must write (standardised depth f32, xyz f32 x 3, valid u8)"""
    d = bench.load_pmc_traffic(bench.PMC_KEYS["depth_small"])
    assert d["kernels"] == 4
    written = 8 * 480 * 640 * (4 + 12 + 1)
    assert d["bytes_per_launch"] >= written
