"""Oracle pinning: the C restatement (oracle/oracle.c) against known answers produced by
the REFERENCE's own code (tests/golden/ref_kats.json, made by oracle/gen_ref_goldens.py
from /root/reference/Src compiled in place).  Bit-exact comparisons on float bit patterns.
"""
import ctypes as C

import numpy as np
import pytest

import pyoracle


def f32(words):
    return np.asarray(words, dtype=np.uint32).view(np.float32)


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


def test_mt19937_uniform_streams(golden):
    seeds = golden["rng_seeds"]
    ref = np.asarray(golden["rng_draws_2000"], dtype=np.uint32).reshape(len(seeds), 2000)
    for i, s in enumerate(seeds):
        got = bits(pyoracle.draws(s, 2000))
        assert np.array_equal(got, ref[i]), f"seed {s}: first mismatch at {np.argmax(got != ref[i])}"


def test_mt19937_deep_stream(golden):
    got = bits(pyoracle.draws(7, 100, skip=100000))
    assert np.array_equal(got, np.asarray(golden["rng_seed7_skip100000"], dtype=np.uint32))


def test_getnext2d_order(golden):
    # Vec2f(dis(gen), dis(gen)) under GCC = (second draw, first draw) (Src/sampler.h:49)
    ref = np.asarray(golden["rng_seed12345_next2d"], dtype=np.uint32).reshape(-1, 2)
    d = bits(pyoracle.draws(12345, 128)).reshape(-1, 2)
    assert np.array_equal(ref[:, 0], d[:, 1]) and np.array_equal(ref[:, 1], d[:, 0])


def test_normalize_and_onb(golden):
    lib = pyoracle.lib()
    vin = f32(golden["onb_in"]).reshape(-1, 3)
    n_ref = np.asarray(golden["onb_normalized"], np.uint32).reshape(-1, 3)
    t_ref = np.asarray(golden["onb_t"], np.uint32).reshape(-1, 3)
    b_ref = np.asarray(golden["onb_b"], np.uint32).reshape(-1, 3)
    for k in range(len(vin)):
        v = np.ascontiguousarray(vin[k])
        n = np.zeros(3, np.float32)
        lib.orc_kat_normalize(pyoracle.fp(v), pyoracle.fp(n))
        assert np.array_equal(bits(n), n_ref[k]), k
        t = np.zeros(3, np.float32)
        b = np.zeros(3, np.float32)
        lib.orc_kat_onb(pyoracle.fp(n), pyoracle.fp(t), pyoracle.fp(b))
        assert np.array_equal(bits(t), t_ref[k]) and np.array_equal(bits(b), b_ref[k]), k


def test_lambert_sample_dir(golden):
    lib = pyoracle.lib()
    m = pyoracle.mt(golden["lambert_seed"][0])
    inp = f32(golden["lambert_in"]).reshape(-1, 3, 3)
    wi_ref = np.asarray(golden["lambert_wi"], np.uint32).reshape(-1, 3)
    pdf_ref = np.asarray(golden["lambert_pdf"], np.uint32)
    for k in range(len(inp)):
        ng, dpdu, dpdv = (np.ascontiguousarray(inp[k, q]) for q in range(3))
        wi = np.zeros(3, np.float32)
        pdf = np.zeros(1, np.float32)
        lib.orc_kat_lambert(C.byref(m), pyoracle.fp(ng), pyoracle.fp(dpdu), pyoracle.fp(dpdv), pyoracle.fp(wi),
                            pyoracle.fp(pdf))
        assert np.array_equal(bits(wi), wi_ref[k]), k
        assert bits(pdf)[0] == pdf_ref[k]


def test_sphere_intersect_and_occluded(golden):
    lib = pyoracle.lib()
    inp = f32(golden["sphere_in"]).reshape(-1, 11)
    hit = golden["sphere_hit"]
    out = np.asarray(golden["sphere_out"], np.uint32).reshape(-1, 7)
    occ = golden["sphere_occluded"]
    for k in range(len(inp)):
        o, d, c = (np.ascontiguousarray(inp[k, 3 * q:3 * q + 3]) for q in range(3))
        r, tmax = float(inp[k, 9]), float(inp[k, 10])
        res = np.zeros(7, np.float32)
        h = lib.orc_kat_sphere(pyoracle.fp(o), pyoracle.fp(d), pyoracle.fp(c), C.c_float(r), pyoracle.fp(res))
        assert h == hit[k], k
        assert np.array_equal(bits(res), out[k]), (k, res, f32(out[k]))
        assert lib.orc_kat_sphere_occluded(pyoracle.fp(o), pyoracle.fp(d), pyoracle.fp(c), C.c_float(r),
                                           C.c_float(tmax)) == occ[k], k


def test_box_intersect(golden):
    lib = pyoracle.lib()
    inp = f32(golden["box_in"]).reshape(-1, 12)
    hit = golden["box_hit"]
    out = np.asarray(golden["box_out"], np.uint32).reshape(-1, 2)
    for k in range(len(inp)):
        o, d, lo, hi = (np.ascontiguousarray(inp[k, 3 * q:3 * q + 3]) for q in range(4))
        res = np.zeros(2, np.float32)
        assert lib.orc_kat_box(pyoracle.fp(o), pyoracle.fp(d), pyoracle.fp(lo), pyoracle.fp(hi),
                               pyoracle.fp(res)) == hit[k], k
        assert np.array_equal(bits(res), out[k]), k


def test_henyey_greenstein(golden):
    lib = pyoracle.lib()
    gs = f32(golden["hg_g"])
    wo = f32(golden["hg_wo"]).reshape(len(gs), -1, 3)
    wi_ref = np.asarray(golden["hg_wi"], np.uint32).reshape(len(gs), -1, 3)
    ev_ref = np.asarray(golden["hg_eval"], np.uint32).reshape(len(gs), -1)
    for gi, g in enumerate(gs):
        m = pyoracle.mt(golden["hg_seed"][0])
        for k in range(wo.shape[1]):
            w = np.ascontiguousarray(wo[gi, k])
            wi = np.zeros(3, np.float32)
            ev = lib.orc_kat_hg(C.byref(m), C.c_float(g), pyoracle.fp(w), pyoracle.fp(wi))
            assert np.array_equal(bits(wi), wi_ref[gi, k]), (g, k)
            assert bits(np.float32(ev)) == ev_ref[gi, k], (g, k)


def test_sample_wavelength(golden):
    lib = pyoracle.lib()
    m = pyoracle.mt(golden["wl_seed"][0])
    inp = f32(golden["wl_in"]).reshape(-1, 2, 3)
    ch = golden["wl_channel"]
    pmf_ref = np.asarray(golden["wl_pmf"], np.uint32).reshape(-1, 3)
    for k in range(len(inp)):
        thr, alb = np.ascontiguousarray(inp[k, 0]), np.ascontiguousarray(inp[k, 1])
        pmf = np.zeros(3, np.float32)
        c = lib.orc_kat_wavelength(C.byref(m), pyoracle.fp(thr), pyoracle.fp(alb), pyoracle.fp(pmf))
        assert c == ch[k], k
        assert np.array_equal(bits(pmf), pmf_ref[k]), k


def test_path_counters_match_reference_probe():
    """SURVEY.md §6 / BASELINE.md: the reference, compiled and run by the survey on Cornell
    800x600x16 GI(3), made 1.776 Scene::intersect and 0.752 Scene::occluded calls per
    sample, and 84.5 ray-triangle tests per sample at 200x150.  The oracle's integrator
    must reproduce those path statistics (they depend on every draw and every hit)."""
    from xraytracer_amd import scenes
    s = scenes.cornell(200, 150)
    _, st = pyoracle.render(s, 200, 150, 16)
    n = 200 * 150 * 16
    assert round(st["segments"] / n, 3) == 1.776
    assert round(st["shadow_rays"] / n, 3) in (0.751, 0.752)
    assert round(st["tri_tests"] / n, 1) == 84.5
    assert st["rejected"] == 0


def test_indirect_and_normal_integrators_oracle():
    """CPU restatements of IndirectIntegrator / NormalIntegrator (parity unpinned beyond the
    building-block KATs; the GPU parity tests compare against these): NormalIntegrator draws
    only the two jitter words per sample and returns 0.5 * (ns + 1) (or 0 on a miss);
    IndirectIntegrator never samples lights."""
    import numpy as np
    from xraytracer_amd import scenes

    s = scenes.cornell(32, 24)
    img, st = pyoracle.render(s, 32, 24, 4, integrator="normal")
    assert st["draws"] == 2 * st["samples"] and st["shadow_rays"] == 0
    assert np.all(img >= 0.0) and np.all(img <= 1.0)
    assert np.any(img == 0.0) and np.any(img > 0.4)
    img, st = pyoracle.render(s, 32, 24, 4, integrator="indirect", max_depth=3)
    assert st["shadow_rays"] == 0 and np.all(np.isfinite(img)) and img.max() > 0
    gi, stg = pyoracle.render(s, 32, 24, 4, integrator="gi", max_depth=3)
    assert stg["shadow_rays"] > 0 and not np.array_equal(img, gi)


def test_vpt_nee_oracle():
    """CPU restatement of VolumePathTracingNEE (parity unpinned beyond the building-block
    KATs — HenyeyGreenstein, sampleWavelength, BoxMesh — and the glibc logf/expf it calls):
    light samples happen only at scattering events, so there are fewer shadow rays than
    segments, and the image is finite and non-negative."""
    import numpy as np
    from xraytracer_amd import scenes

    s = scenes.smoke(24, 18, n=24)
    img, st = pyoracle.render(s, 24, 18, 4, integrator="vpt_nee")
    assert 0 < st["shadow_rays"] < st["segments"] and st["stalled"] == 0
    assert np.all(np.isfinite(img)) and np.all(img >= 0) and img.max() > 0
    vpt, stv = pyoracle.render(s, 24, 18, 4, integrator="vpt")
    assert stv["shadow_rays"] == 0 and not np.array_equal(img, vpt)


def test_camera_ray_direction(golden):
    """PinholeCamera::sampleRay's direction (Src/camera.h:52-55) — multDirMatrix
    (geometry.h:653-669) + normalize evaluated by the reference's own code — for the
    Cornell, C3 and C5 cameras and random matrices; the origin is c2w row 3."""
    lib = pyoracle.lib()
    mats = f32(golden["cam_c2w"]).reshape(-1, 16)
    inp = f32(golden["cam_in"]).reshape(len(mats), -1, 4)
    ref = np.asarray(golden["cam_dir"], np.uint32).reshape(len(mats), -1, 3)
    for mi, m in enumerate(mats):
        cam = pyoracle.OrcCamera()
        for i in range(16):
            cam.c2w[i] = float(m[i])
        for k in range(inp.shape[1]):
            u, v, cam.scale, cam.aspect = (float(x) for x in inp[mi, k])
            o = np.zeros(3, np.float32)
            d = np.zeros(3, np.float32)
            lib.orc_kat_camera(C.byref(cam), C.c_float(u), C.c_float(v), pyoracle.fp(o), pyoracle.fp(d))
            assert np.array_equal(bits(d), ref[mi, k]), (mi, k)
            assert np.array_equal(o, m[12:15])


def test_lambert_bxdf_through_material_interface(golden):
    """Lambert::sampleBxDF + evaluateBxDF (Src/material.h:39-53): f = albedo / PI per
    channel, the sampled direction and pdf 1 / (2 PI)."""
    lib = pyoracle.lib()
    m = pyoracle.mt(golden["bxdf_seed"][0])
    inp = f32(golden["bxdf_in"]).reshape(-1, 5, 3)
    f_ref = np.asarray(golden["bxdf_f"], np.uint32).reshape(-1, 3)
    wi_ref = np.asarray(golden["bxdf_wi"], np.uint32).reshape(-1, 3)
    pdf_ref = np.asarray(golden["bxdf_pdf"], np.uint32)
    ev_ref = np.asarray(golden["bxdf_eval"], np.uint32).reshape(-1, 3)
    assert np.array_equal(f_ref, ev_ref)
    for k in range(len(inp)):
        alb, ng, dpdu, dpdv, _ = (np.ascontiguousarray(inp[k, q]) for q in range(5))
        f = np.zeros(3, np.float32)
        wi = np.zeros(3, np.float32)
        pdf = np.zeros(1, np.float32)
        lib.orc_kat_lambert_bxdf(C.byref(m), pyoracle.fp(alb), pyoracle.fp(ng), pyoracle.fp(dpdu), pyoracle.fp(dpdv),
                                 pyoracle.fp(f), pyoracle.fp(wi), pyoracle.fp(pdf))
        assert np.array_equal(bits(f), f_ref[k]), k
        assert np.array_equal(bits(wi), wi_ref[k]), k
        assert bits(pdf)[0] == pdf_ref[k]


def test_sphere_light_area_sampling(golden):
    """SphereLight::sample built with AREA_SAMPLING (Src/light.h:131-135,185-191) and
    UniformSampleSphere (Src/light.cpp:99-105), evaluated by the reference's own Vec3f /
    UniformSampler code with the call's shape kept (GCC: the first draw is r2): wi, pdf,
    tmax and whether the sample faces the point, for 512 lights and points on one stream."""
    from xraytracer_amd import abi
    lib = pyoracle.lib()
    m = pyoracle.mt(golden["sphere_area_seed"][0])
    inp = f32(golden["sphere_area_in"]).reshape(-1, 7)
    ref = np.asarray(golden["sphere_area_out"], np.uint32).reshape(-1, 6)
    front = 0
    for k in range(len(inp)):
        lt = abi.XrtLight()
        lt.kind = abi.XRT_LIGHT_SPHERE_AREA
        for q in range(3):
            lt.center[q] = float(inp[k, q])
            lt.Le[q] = 1.0
        lt.radius = float(inp[k, 3])
        pos = np.ascontiguousarray(inp[k, 4:7])
        out = np.zeros(8, np.float32)
        lib.orc_kat_light(C.byref(m), C.byref(lt), pyoracle.fp(pos), pyoracle.fp(out))
        faces = int(ref[k, 5])
        front += faces
        assert int(out[5] != 0.0) == faces, k
        assert bits(out[4:5])[0] == ref[k, 4], k          # tmax is written either way
        if faces:
            assert np.array_equal(bits(out[0:3]), ref[k, 0:3]), k
            assert bits(out[3:4])[0] == ref[k, 3], k
    assert 100 < front < 412   # both outcomes are covered
