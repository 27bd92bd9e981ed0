"""Host Scene layer (C++ include/xrt/scene.h via the xrt_hscene facade): no GPU needed."""
import os

import numpy as np
import pytest

from xraytracer_amd import abi, scenes


def test_cornell_object_order_matches_reference_unordered_map():
    # SURVEY.md §7 hard part 2 [probe of the reference]: Cornell iterates
    # tall_block, short_block, QuadLight, green_wall, red_wall, back_wall, ceiling, floor
    s = scenes.cornell(256, 256)
    assert s.object_names() == ["tall_block", "short_block", "QuadLight", "green_wall", "red_wall",
                                "back_wall", "ceiling", "floor"]


def test_cornell_geometry():
    s = scenes.cornell(256, 256)
    d = s.desc
    assert d.n_tris == 36 and d.n_objects == 8 and d.n_lights == 1   # 34 OBJ triangles + 2 light
    counts = [d.objects[i].count for i in range(d.n_objects)]
    assert counts == [10, 10, 2, 2, 2, 2, 2, 6]
    light_obj = d.objects[2]
    assert light_obj.light == 0 and light_obj.material == abi.XRT_MAT_NONE
    red = d.objects[4]
    assert list(red.albedo) == [1.0, 0.0, 0.0] and red.material == abi.XRT_MAT_LAMBERT
    L = d.lights[0]
    assert L.kind == abi.XRT_LIGHT_QUAD and list(L.Le) == [25.0, 25.0, 25.0]
    assert list(L.v0) == [343.0, 548.0, 227.0]


def test_tinyobj_quad_split_shorter_diagonal():
    # floor face "f 1 2 3 4": |v2-v0|^2 = 618292.5 > |v3-v1|^2 = 614764.8 -> (0,1,3),(1,2,3)
    s = scenes.cornell(8, 8)
    tris = s.triangles()
    floor_first = s.desc.objects[7].first
    v = np.array([[552.8, 0, 0], [0, 0, 0], [0, 0, 559.2], [549.6, 0, 559.2]], np.float32)
    assert np.array_equal(tris[floor_first], v[[0, 1, 3]])
    assert np.array_equal(tris[floor_first + 1], v[[1, 2, 3]])


def test_face_normals_when_obj_has_no_vn():
    s = scenes.cornell(8, 8)
    d = s.desc
    tn = np.ctypeslib.as_array(d.tri_n, shape=(d.n_tris * 9,)).reshape(-1, 3, 3)
    tv = s.triangles()
    for t in range(d.n_tris):
        e1, e2 = tv[t, 1] - tv[t, 0], tv[t, 2] - tv[t, 0]
        n = np.cross(e1.astype(np.float64), e2.astype(np.float64))
        n /= np.linalg.norm(n)
        assert np.allclose(tn[t, 0], n, atol=1e-6) and np.array_equal(tn[t, 0], tn[t, 2])


def test_sphere_mesh_triangulation_count():
    s = scenes.cornell_spheremesh(8, 8, n_theta=160, n_phi=160)
    names = s.object_names()
    k = names.index("sphere_mesh")
    assert s.desc.objects[k].count == 2 * 160 * 160 == 51200
    assert s.desc.n_tris == 36 + 51200


def test_sphere_scene_c3():
    s = scenes.spheres(64, 36)
    d = s.desc
    assert d.n_spheres == 1001 and d.n_lights == 1 and d.n_tris == 0
    kinds = {d.objects[i].kind for i in range(d.n_objects)}
    assert kinds == {abi.XRT_OBJ_SPHERE}
    light_objs = [i for i in range(d.n_objects) if d.objects[i].light >= 0]
    assert len(light_objs) == 1


def test_pinhole_scale_is_the_gcc_folded_value():
    """tan(0.5*deg2rad(FOV)) (Src/camera.h:45): the reference examples pass a constant FOV
    and GCC -O2 folds the tan correctly rounded (FOV 60 -> 0x1.279a74p-1; glibc's run-time
    tanf would give 0x1.279a76p-1).  The host layer reproduces the folded value."""
    import math
    pi = np.float32(3.14159265359)
    for fov in (60.0, 45.0, 90.0, 37.5):
        arg = np.float32(0.5) * (np.float32(fov) / np.float32(180.0) * pi)
        sc = np.float32(abi.lib().xrt_pinhole_scale(fov))
        assert sc == np.float32(math.tan(float(arg))), fov
    assert np.float32(abi.lib().xrt_pinhole_scale(60.0)) == np.float32(float.fromhex("0x1.279a74p-1"))


def test_load_obj_missing_file_is_an_error():
    s = scenes.SceneBundle()
    with pytest.raises(abi.XrtError):
        s.load_obj("/nonexistent/file.obj")


def test_obj_parser_negative_indices_and_vn(tmp_path):
    obj = tmp_path / "t.obj"
    (tmp_path / "t.mtl").write_text("newmtl a\nKd 0.5 0.25 1\nnewmtl hidden\nKd 1 1 1\nno_surface 1\n")
    obj.write_text("mtllib t.mtl\no tri\nusemtl a\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\n"
                   "f -3//1 -2//1 -1//1\no tri2\nusemtl hidden\nv 0 0 1\nv 1 0 1\nv 0 1 1\nf 4 5 6\n")
    s = scenes.SceneBundle()
    s.load_obj(str(obj))
    d = s.flatten()
    names = s.object_names()
    a = d.objects[names.index("tri")]
    assert a.material == abi.XRT_MAT_LAMBERT and list(a.albedo) == [0.5, 0.25, 1.0]
    assert d.objects[names.index("tri2")].material == abi.XRT_MAT_NONE   # no_surface -> nullptr
    tn = np.ctypeslib.as_array(d.tri_n, shape=(d.n_tris * 9,)).reshape(-1, 3, 3)
    assert np.array_equal(tn[a.first, 0], [0, 0, 1])


def _polygon_obj(tmp_path, polys):
    """An OBJ with one shape per polygon (vertex lists in the z = 1 plane) and one material."""
    (tmp_path / "p.mtl").write_text("newmtl white\nKd 0.5 0.5 0.5\n")
    lines, base = ["mtllib p.mtl"], 1
    for name, pts in polys:
        lines.append(f"o {name}")
        lines += [f"v {x} {y} 1.0" for x, y in pts]
        lines.append("usemtl white")
        lines.append("f " + " ".join(str(base + k) for k in range(len(pts))))
        base += len(pts)
    path = tmp_path / "p.obj"
    path.write_text("\n".join(lines) + "\n")
    return str(path)


def _area2(t):
    (ax, ay), (bx, by), (cx, cy) = t[:, :2].astype(np.float64)
    return (bx - ax) * (cy - ay) - (by - ay) * (cx - ax)


@pytest.mark.parametrize("name,pts", [
    ("hexagon", [(2, 0), (1, 1.7), (-1, 1.7), (-2, 0), (-1, -1.7), (1, -1.7)]),
    ("arrow", [(0, 0), (4, 0), (4, 3), (2, 1), (0, 3)]),              # concave: reflex corner at (2, 1)
    ("comb", [(0, 0), (6, 0), (6, 4), (5, 4), (5, 1), (3, 1), (3, 4), (2, 4), (2, 1), (0, 1)]),
])
def test_tinyobj_ear_clipping_polygons(tmp_path, name, pts):
    """Faces of five or more vertices go through tinyobjloader's built-in ear clipping
    (Src/scene.cpp:54 ParseFromFile with triangulate = true).  tinyobjloader is absent, so the
    exact triangle list is parity-unpinned; what ear clipping guarantees is checked: n - 2
    triangles, none wound against the polygon (collinear vertices may give a zero-area one,
    as tinyobjloader's test `cross * area < 0` lets through), covering exactly the
    polygon's area, using only the polygon's vertices."""
    s = scenes.SceneBundle()
    s.load_obj(_polygon_obj(tmp_path, [(name, pts)]))
    s.flatten()
    tris = s.triangles()
    assert len(tris) == len(pts) - 2
    p = np.array(pts, np.float64)
    poly2 = np.sum(p[:, 0] * np.roll(p[:, 1], -1) - np.roll(p[:, 0], -1) * p[:, 1])
    areas = [_area2(t) for t in tris]
    assert all(a * poly2 >= 0 for a in areas)
    assert abs(sum(areas) - poly2) < 1e-3
    verts = {tuple(np.float32(v)) for v in np.array([(x, y, 1.0) for x, y in pts], np.float32)}
    assert all(tuple(v) in verts for t in tris for v in t)


def test_sphere_light_sampling_kind_in_flattened_scene():
    """SphereLight::Sampling::Area (the reference's AREA_SAMPLING build, Src/light.h:131-135)
    flattens to XRT_LIGHT_SPHERE_AREA, the default to the cone-sampled XRT_LIGHT_SPHERE."""
    from xraytracer_amd import abi, scenes
    for area, kind in ((True, abi.XRT_LIGHT_SPHERE_AREA), (False, abi.XRT_LIGHT_SPHERE)):
        s = scenes.SceneBundle()
        s.add_sphere("ball", (0.0, 0.0, -3.0), 0.5, (0.5, 0.5, 0.5))
        s.add_sphere_light("SphereLight", (0.0, 4.0, -3.0), 1.0, (10.0, 10.0, 10.0), area=area)
        s.flatten()
        assert s.desc.n_lights == 1 and s.desc.lights[0].kind == kind
        assert [s.desc.lights[0].center[q] for q in range(3)] == [0.0, 4.0, -3.0]
