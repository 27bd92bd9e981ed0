"""The drop-in host geometry (include/xrt/geometry.h: Matrix44::inverse / operator* /
transposed, orthonormalBasis, worldToLocal / localToWorld — Src/geometry.h:314-590,671-701,
Src/geometry.cpp:23-49) bit for bit against the reference's own code compiled in place
(oracle/ref_kats.cpp -> tests/golden/ref_kats.json).  CPU only: g++ builds a small driver
against the header with the reference build's float settings (-O2 -ffp-contract=off)."""
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def golden():
    return json.load(open(os.path.join(ROOT, "tests", "golden", "ref_kats.json")))


@pytest.fixture(scope="module")
def kat(tmp_path_factory):
    d = tmp_path_factory.mktemp("hostgeo")
    exe = str(d / "host_geometry_kat")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.join(ROOT, "include"),
                           "-o", exe, os.path.join(ROOT, "tests", "cpp", "host_geometry_kat.cpp")])

    def run(mode, words):
        i, o = d / f"{mode}.in", d / f"{mode}.out"
        np.asarray(words, np.uint32).tofile(i)
        subprocess.check_call([exe, mode, str(i), str(o)])
        return np.fromfile(o, np.uint32)
    return run


def test_matrix44_inverse_product_transpose(golden, kat):
    got = kat("m44", golden["m44_in"]).reshape(-1, 3, 16)
    assert np.array_equal(got[:, 0], np.asarray(golden["m44_inverse"], np.uint32).reshape(-1, 16))
    assert np.array_equal(got[:, 1], np.asarray(golden["m44_mul_next"], np.uint32).reshape(-1, 16))
    assert np.array_equal(got[:, 2], np.asarray(golden["m44_transposed"], np.uint32).reshape(-1, 16))
    # the singular matrix (second entry) inverts to the identity, as the reference returns
    eye = np.eye(4, dtype=np.float32).reshape(-1).view(np.uint32)
    assert np.array_equal(got[1, 0], eye)


def test_world_local_frames(golden, kat):
    got = kat("frame", golden["frame_in"]).reshape(-1, 2, 3)
    assert np.array_equal(got[:, 0], np.asarray(golden["frame_w2l"], np.uint32).reshape(-1, 3))
    assert np.array_equal(got[:, 1], np.asarray(golden["frame_l2w"], np.uint32).reshape(-1, 3))


def test_orthonormal_basis(golden, kat):
    got = kat("onb", golden["onb_in"]).reshape(-1, 3, 3)
    assert np.array_equal(got[:, 0], np.asarray(golden["onb_normalized"], np.uint32).reshape(-1, 3))
    assert np.array_equal(got[:, 1], np.asarray(golden["onb_t"], np.uint32).reshape(-1, 3))
    assert np.array_equal(got[:, 2], np.asarray(golden["onb_b"], np.uint32).reshape(-1, 3))
