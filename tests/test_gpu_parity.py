"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's own golden outputs.  Integer/index work must be bit-exact; pixel RGB
is compared with a 1e-4 tolerance (north_star) and is in fact expected to be
bit-identical because both sides use the same IEEE op sequence without FMA."""
import json
import os

import numpy as np
import pytest

import raytracebvh_amd as rt
from oracle import lib as orc
from tests.conftest import GOLDEN, load_scene_fixture

pytestmark = pytest.mark.gpu
RGB_TOL = 1e-4


def fnv_u32_values(vals):
    h = 1469598103934665603
    for v in vals:
        h ^= int(v) & 0xFFFFFFFF
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="module")
def ctx():
    c = rt.Context(device=0, flags=rt.FLAG_TIMING)
    yield c
    c.close()


def _oscene(s):
    return orc.Scene(s.vertices, s.indices, s.mat_indices, s.material_blob)


def _assert_nodes_equal(got, want, n):
    for f in ("parent", "child_l", "child_r"):
        np.testing.assert_array_equal(got[f], want[f], err_msg=f)
    np.testing.assert_array_equal(got["code"][:n], want["code"][:n])
    np.testing.assert_array_equal(got["index"][:n], want["index"][:n])
    np.testing.assert_array_equal(got["bb_min"], want["bb_min"])
    np.testing.assert_array_equal(got["bb_max"], want["bb_max"])


# ---------------------------------------------------------------- sort
@pytest.mark.parametrize("n", [1, 2, 3, 255, 4095, 4096, 4097, 12289, 100_003])
@pytest.mark.parametrize("key_bits", [32, 30])
def test_sort_pairs_stable(ctx, n, key_bits):
    rng = np.random.default_rng(n + key_bits)
    keys = rng.integers(0, 1 << key_bits, size=n, dtype=np.uint64).astype(np.uint32)
    keys[::7] = keys[0]   # duplicates
    vals = np.arange(n, dtype=np.uint32)
    ko, vo = ctx.sort_pairs(keys, vals, key_bits)
    perm = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(ko, keys[perm])
    np.testing.assert_array_equal(vo, perm.astype(np.uint32))


def test_sort_matches_reference_combo(ctx):
    z = np.load(os.path.join(GOLDEN, "combo.npz"))
    keys = z["input_codes"]
    ko, vo = ctx.sort_pairs(keys, np.arange(len(keys), dtype=np.uint32), 30)
    np.testing.assert_array_equal(ko, z["sorted_codes"])
    np.testing.assert_array_equal(vo, orc.split_sort(keys))


def test_sort_large_property(ctx):
    """10M keys (BASELINE C4 size): sortedness + permutation + stability."""
    n = 10_000_000
    rng = np.random.default_rng(4)
    keys = rng.integers(0, 1 << 30, size=n, dtype=np.uint32)
    keys[: n // 4] &= np.uint32(0x3FF00000)   # heavy duplicates
    ko, vo = ctx.sort_pairs(keys, np.arange(n, dtype=np.uint32), 30)
    assert (np.diff(ko.astype(np.int64)) >= 0).all()
    np.testing.assert_array_equal(keys[vo], ko)
    np.testing.assert_array_equal(np.sort(vo), np.arange(n, dtype=np.uint32))
    eq = ko[1:] == ko[:-1]
    assert (vo[1:][eq] > vo[:-1][eq]).all()   # stable


# ---------------------------------------------------------------- Karras + refit
@pytest.mark.parametrize("mode", [rt.DELTA_CPUTESTS, rt.DELTA_CLZ64])
def test_karras_refit_matches_reference_combo(mode):
    """RadixBVHCombo: every parent/child link and refit box of the reference's 11,775 nodes."""
    z = np.load(os.path.join(GOLDEN, "combo.npz"))
    n = len(z["sorted_codes"])
    boxes = np.concatenate([z["bb_min"][:n], z["bb_max"][:n]], axis=1)
    with rt.Context(device=0, delta_mode=mode) as c:
        nodes = c.build_from_codes(z["sorted_codes"], boxes)
    np.testing.assert_array_equal(nodes["parent"], z["parent"].astype(np.uint32))
    np.testing.assert_array_equal(nodes["child_l"], z["child_l"].astype(np.uint32))
    np.testing.assert_array_equal(nodes["child_r"], z["child_r"].astype(np.uint32))
    np.testing.assert_array_equal(nodes["bb_min"], z["bb_min"])
    np.testing.assert_array_equal(nodes["bb_max"], z["bb_max"])
    kat = json.load(open(os.path.join(GOLDEN, "shadersim_kats.json")))["combo_topology_fnv"]["value"]
    links = np.stack([nodes["parent"], nodes["child_l"], nodes["child_r"]], 1).ravel()
    assert "%016x" % fnv_u32_values(links) == kat


def test_karras_paper_example():
    z = np.load(os.path.join(GOLDEN, "bvhct.npz"))
    codes = z["code"][:8].astype(np.uint32)
    boxes = np.zeros((8, 6), np.float32)
    with rt.Context(device=0) as c:
        nodes = c.build_from_codes(codes, boxes)
    np.testing.assert_array_equal(nodes["child_l"][8:], z["child_l"][8:].astype(np.uint32))
    np.testing.assert_array_equal(nodes["child_r"][8:], z["child_r"][8:].astype(np.uint32))


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 65_537])
def test_from_codes_random_duplicates_vs_oracle(n):
    rng = np.random.default_rng(n)
    codes = np.sort(rng.integers(0, 1 << 12, size=n, dtype=np.uint32) << np.uint32(18))
    lo = rng.standard_normal((n, 3)).astype(np.float32)
    hi = lo + rng.random((n, 3), dtype=np.float32)
    with rt.Context(device=0) as c:
        nodes = c.build_from_codes(codes, np.concatenate([lo, hi], 1))
    if n == 1:
        assert nodes["parent"][0] == 0xFFFFFFFF
        return
    parent, cl, cr = orc.karras(codes, orc.DELTA_CLZ64)
    bmin = np.zeros((2 * n - 1, 3), np.float32)
    bmax = np.zeros((2 * n - 1, 3), np.float32)
    bmin[:n], bmax[:n] = lo, hi
    bmin, bmax, _ = orc.refit(n, parent, cl, cr, bmin, bmax)
    np.testing.assert_array_equal(nodes["parent"], parent)
    np.testing.assert_array_equal(nodes["child_l"], cl)
    np.testing.assert_array_equal(nodes["child_r"], cr)
    np.testing.assert_array_equal(nodes["bb_min"], bmin)
    np.testing.assert_array_equal(nodes["bb_max"], bmax)


# ---------------------------------------------------------------- full build on the reference scenes
@pytest.mark.parametrize("name", ["Rect", "Image_Test", "Test"])
@pytest.mark.parametrize("morton_mode", [rt.MORTON_CPUTESTS, rt.MORTON_HLSL])
def test_build_matches_oracle_on_obj(name, morton_mode):
    d = load_scene_fixture(name)
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    wvp, wv = rt.camera_reference(1920, 1080)
    with rt.Context(device=0, morton_mode=morton_mode) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.build()
        codes = c.read_morton()
        keys, ids = c.read_sorted()
        nodes = c.read_bvh()
    os_ = _oscene(s)
    ocodes = orc.morton_tris(os_, morton_mode, wvp, (-700,) * 3, (700,) * 3)
    np.testing.assert_array_equal(codes, ocodes)
    if morton_mode == rt.MORTON_CPUTESTS:
        kat = json.load(open(os.path.join(GOLDEN, "shadersim_kats.json")))[name]
        assert "%016x" % fnv_u32_values(codes) == kat["fnv"]
    perm = orc.split_sort(ocodes)
    np.testing.assert_array_equal(ids, perm)
    np.testing.assert_array_equal(keys, ocodes[perm])
    onodes = orc.build(os_, wvp, morton_mode=morton_mode, sort_mode=0)
    _assert_nodes_equal(nodes, onodes, s.num_tris)


@pytest.mark.parametrize("ntris", [1, 2, 5, 1000, 200_000])
def test_build_matches_oracle_synthetic(ntris):
    s = rt.synthetic(ntris, seed=0x5EED0004, half_extent=(50, 50, 50))
    wvp, wv = rt.camera_reference(1920, 1080)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.build()
        nodes = c.read_bvh()
    onodes = orc.build(_oscene(s), wvp)
    _assert_nodes_equal(nodes, onodes, ntris)


def test_build_10m_tree_properties():
    """C4 size: 10M triangles.  Valid tree (one parent per node), boxes nest, codes sorted."""
    n = 10_000_000
    s = rt.synthetic(n, seed=0x5EED0004, half_extent=(50, 50, 50))
    wvp, wv = rt.camera_reference(1920, 1080)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.build()
        nodes = c.read_bvh()
        keys, ids = c.read_sorted()
    assert (np.diff(keys.astype(np.int64)) >= 0).all()
    np.testing.assert_array_equal(np.sort(ids), np.arange(n, dtype=np.uint32))
    cl = nodes["child_l"][n:].astype(np.int64)
    cr = nodes["child_r"][n:].astype(np.int64)
    counts = np.bincount(np.concatenate([cl, cr]), minlength=2 * n - 1)
    assert counts[n] == 0 and (np.delete(counts, n) == 1).all()
    np.testing.assert_array_equal(nodes["parent"][cl], np.arange(n, 2 * n - 1))
    np.testing.assert_array_equal(nodes["parent"][cr], np.arange(n, 2 * n - 1))
    for side in (cl, cr):
        assert (nodes["bb_min"][side] >= nodes["bb_min"][n:]).all()
        assert (nodes["bb_max"][side] <= nodes["bb_max"][n:]).all()


# ---------------------------------------------------------------- trace
# the shipped walk combinations (include/rtbvh.h RTBVH_FLAG_*; "auto" picks one of them by size)
WALK_FLAGS = rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE | rt.FLAG_WIDE_BVH
TRACE_MODES = {"reference": 0, "reference+sort": rt.FLAG_SORT_BOUNCE, "nearest": rt.FLAG_NEAREST_FIRST,
               "packet": rt.FLAG_PACKET_PRIMARY,
               "nearest+packet": rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY,
               "refill+sort": rt.FLAG_REFILL_BOUNCE | rt.FLAG_SORT_BOUNCE,
               "nearest+packet+refill": rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_REFILL_BOUNCE,
               "nearest+packet+wide": rt.FLAG_NEAREST_FIRST | rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH,
               "packet+wide": rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH,
               "wide+sort": rt.FLAG_WIDE_BVH | rt.FLAG_SORT_BOUNCE,
               "binned": rt.FLAG_BINNED_PRIMARY,
               "binned+wide+refill": WALK_FLAGS | rt.FLAG_BINNED_PRIMARY,
               "auto": rt.FLAG_AUTO_WALK,
               "certified": rt.FLAG_CERTIFIED}


def _trace_both(s, W, H, bounces, rows=None, flags=0):
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=flags | rt.FLAG_COUNT_VISITS) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, bounces)
        fb = c.read_framebuffer()
        inten = c.read_intensity()
        nodes = c.read_bvh()
        st = c.stats()
    r0, r1, step = rows if rows else (0, H, 1)
    ofb, oint, ost = orc.trace(_oscene(s), nodes, wvp, wv, W, H, bounces, r0, r1, step, want_intensity=True)
    return fb[r0:r1:step], inten[r0:r1:step], st, ofb, oint, ost


@pytest.mark.parametrize("mode", list(TRACE_MODES))
@pytest.mark.parametrize("name,W,H,bounces", [("Rect", 320, 240, 1), ("Image_Test", 1920, 1080, 0),
                                               ("Test", 1920, 1080, 1), ("Test", 800, 800, 3)])
def test_trace_matches_oracle_on_obj(name, W, H, bounces, mode):
    d = load_scene_fixture(name)
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    fb, inten, st, ofb, oint, ost = _trace_both(s, W, H, bounces, flags=TRACE_MODES[mode])
    np.testing.assert_allclose(fb, ofb, atol=RGB_TOL, rtol=0)
    assert np.array_equal(fb, ofb), "expected bit-identical pixels"
    np.testing.assert_array_equal(inten, oint)
    assert sum(st["hits"]) == ost["hits"] and st["textured_hits"] == ost["textured_hits"]
    assert st["bounce_rays"] == ost["bounce"] and st["stack_overflows"] == 0
    if not any(k in mode for k in ("nearest", "wide", "binned", "auto", "certified")):   # reference order: the oracle's steps
        assert sum(st["internal_visits"]) == ost["internal_visits"]
        assert sum(st["leaf_visits"]) == ost["leaf_visits"]
    else:
        assert sum(st["internal_visits"]) <= ost["internal_visits"]
    assert ost["hits"] > 0


@pytest.mark.parametrize("name,W,H,bounces", [("Rect", 320, 240, 1), ("Test", 800, 800, 3), ("Test", 640, 360, 0)])
def test_ray_records_match_oracle(name, W, H, bounces):
    """reflectRay / refractRay RayPresent records (RTBVH_FLAG_REFRACT_RECORDS) vs the oracle,
    bit for bit (NaN where both have NaN: refract of a total internal reflection)."""
    d = load_scene_fixture(name)
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=rt.FLAG_REFRACT_RECORDS | rt.FLAG_PACKET_PRIMARY) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, bounces)
        refl, refr = c.read_rays()
        fb = c.read_framebuffer()
        nodes = c.read_bvh()
    ofb, _, _, orefl, orefr = orc.trace(_oscene(s), nodes, wvp, wv, W, H, bounces, want_records=True)
    assert np.array_equal(fb, ofb)
    np.testing.assert_array_equal(refl, orefl)
    np.testing.assert_array_equal(refr, orefr)
    assert np.array_equal(refl[..., 10:14], fb)   # the record's colour is the framebuffer
    assert (refl[..., 0] > 0).any() or bounces > 0


def _textures(seed=3):
    """Synthetic sRGB textures of odd sizes (the reference's image files are not on the GPU box;
    decoding is pinned on CPU against PIL, tests/test_host.py)."""
    rng = np.random.default_rng(seed)
    return [rng.integers(0, 256, (37, 53, 4), dtype=np.uint8), rng.integers(0, 256, (64, 29, 4), dtype=np.uint8)]


@pytest.mark.parametrize("name,W,H,bounces", [("Test", 1920, 1080, 1), ("Image_Test", 1920, 1080, 0),
                                               ("Test", 800, 800, 3), ("Rect", 320, 240, 1)])
def test_textured_frames_match_oracle(name, W, H, bounces):
    """renderPixel with diffuse textures (RayTraceRender.hlsl:22-26): GPU vs oracle, bit for bit,
    for every traversal mode family; the textures must change the frame."""
    d = load_scene_fixture(name)
    tex = _textures()
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"], textures=tex)
    os_ = orc.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"], textures=tex)
    wvp, wv = rt.camera_reference(W, H)
    for flags in (0, rt.FLAG_PACKET_PRIMARY | rt.FLAG_NEAREST_FIRST | rt.FLAG_WIDE_BVH):
        with rt.Context(device=0, flags=flags | rt.FLAG_COUNT_VISITS) as c:
            c.set_scene(s)
            c.set_camera(wvp, wv)
            c.compute_bvh(W, H, bounces)
            fb = c.read_framebuffer()
            st = c.stats()
            nodes = c.read_bvh()
        ofb, _, ost = orc.trace(os_, nodes, wvp, wv, W, H, bounces)
        np.testing.assert_allclose(fb, ofb, atol=RGB_TOL, rtol=0)
        assert np.array_equal(fb, ofb)
        assert st["textured_hits"] == ost["textured_hits"] > 0
    white, _, _ = orc.trace(_oscene(s), nodes, wvp, wv, W, H, bounces)
    assert not np.array_equal(white, ofb)


def _reference_textures():
    """Test.obj's own textures (Test.mtl: Balls.jpg, Map__1_Composite.bmp), decoded by librtbvh
    (the files are the reference's CPUTests data, committed under tests/golden/textures)."""
    from raytracebvh_amd.scene import load_texture
    d = load_scene_fixture("Test")
    return [load_texture(os.path.join(GOLDEN, "textures", str(n))) for n in d["texture_names"]]


@pytest.mark.parametrize("mode", ["reference", "nearest+packet+wide", "auto", "certified"])
def test_reference_scene_with_its_own_textures(mode):
    """The reference's default scene as Graphics::onInit loads it (Graphics.cpp:364: Obj/Test.obj
    with Balls.jpg and Map__1_Composite.bmp), 1920x1080, primary + 1 bounce: GPU frame equals the
    oracle's with the same texels, bit for bit, and the textures change the frame."""
    d = load_scene_fixture("Test")
    tex = _reference_textures()
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"], textures=tex)
    os_ = orc.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"], textures=tex)
    W, H = 1920, 1080
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=TRACE_MODES[mode] | rt.FLAG_COUNT_VISITS) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        fb = c.read_framebuffer()
        st = c.stats()
        nodes = c.read_bvh()
    ofb, _, ost = orc.trace(os_, nodes, wvp, wv, W, H, 1)
    np.testing.assert_allclose(fb, ofb, atol=RGB_TOL, rtol=0)
    assert np.array_equal(fb, ofb)
    assert st["textured_hits"] == ost["textured_hits"] > 0
    white, _, _ = orc.trace(_oscene(s), nodes, wvp, wv, W, H, 1)
    assert not np.array_equal(white, ofb)


def test_present_is_flipped_unorm8_framebuffer():
    """RayTraceBVHPS.hlsl:13-16 into R8G8B8A8_UNORM: screen row y = framebuffer row H-1-y."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"], textures=_textures())
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(640, 360))
        c.compute_bvh(640, 360, 1)
        fb = c.read_framebuffer()
        img = c.present()
    want = np.floor(np.clip(fb, 0, 1) * np.float32(255) + np.float32(0.5)).astype(np.uint8)[::-1]
    np.testing.assert_array_equal(img, want)


def test_read_rays_needs_records_flag():
    d = load_scene_fixture("Rect")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(64, 64))
        c.compute_bvh(64, 64, 1)
        with pytest.raises(RuntimeError, match="REFRACT_RECORDS"):
            c.read_rays()


def _tiny_scene(ntris):
    """ntris big triangles facing the camera, one behind the other (z = 0, 5, 10)."""
    verts, idx = [], []
    for k in range(ntris):
        z = 5.0 * k
        for x, y in ((-20.0 - k, -15.0), (20.0, -15.0 - k), (0.0, 18.0 + k)):
            verts.append([x, y, z, 0.0, 0.0, -1.0, 0.5, 0.5])
        idx += [3 * k, 3 * k + 1, 3 * k + 2]
    mat = np.zeros(1, dtype=rt.MATERIAL_DTYPE)
    mat["diffuse"] = [0.6, 0.5, 0.4, 1.0]
    mat["specular"] = [1.0, 1.0, 1.0, 1.0]
    mat["shininess"] = 400.0
    mat["alpha"] = 1.0
    mat["tex_num"] = -1
    return rt.Scene(np.array(verts, np.float32), np.array(idx, np.uint32), np.zeros(ntris, np.uint32), mat)


@pytest.mark.parametrize("ntris", [1, 2, 3])
@pytest.mark.parametrize("mode", list(TRACE_MODES))
def test_trace_tiny_scenes(ntris, mode):
    """One-, two- and three-triangle trees (a leaf root, a root with two leaves, ...) in every mode."""
    s = _tiny_scene(ntris)
    fb, inten, st, ofb, oint, ost = _trace_both(s, 160, 90, 2, flags=TRACE_MODES[mode])
    assert np.array_equal(fb, ofb)
    np.testing.assert_array_equal(inten, oint)
    assert ost["hits"] > 0 and st["stack_overflows"] == 0


@pytest.mark.parametrize("mode", list(TRACE_MODES))
def test_trace_synthetic_sampled_rows(mode):
    """C5 scene at reduced size: 500k triangles, 1920x1080, every 37th row vs oracle."""
    s = rt.synthetic(500_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    fb, inten, st, ofb, oint, ost = _trace_both(s, 1920, 1080, 1, rows=(3, 1080, 37), flags=TRACE_MODES[mode])
    np.testing.assert_allclose(fb, ofb, atol=RGB_TOL, rtol=0)
    assert np.array_equal(fb, ofb)
    np.testing.assert_array_equal(inten, oint)


C5_SCENE = dict(ntris=10_000_000, seed=0x5EED0005, half=(100, 100, 50))
C4_SCENE = dict(ntris=10_000_000, seed=0x5EED0004, half=(50, 50, 50))


def _oracle_threads():
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS") or 0) or (os.cpu_count() or 1)))


@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_10m_tree_matches_oracle(cfg):
    """BASELINE C4 / C5 at full size (10M triangles): the GPU tree equals the oracle's own build
    of the same scene in every field of every one of the 2n-1 nodes (Morton codes, sorted
    order, Karras links, refit boxes)."""
    p = C4_SCENE if cfg == "C4" else C5_SCENE
    s = rt.synthetic(p["ntris"], seed=p["seed"], half_extent=p["half"])
    wvp, wv = rt.camera_reference(1920, 1080) if cfg == "C4" else rt.camera_reference(3840, 2160)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.build()
        nodes = c.read_bvh()
    onodes = orc.build(_oscene(s), wvp)
    for f in ("parent", "child_l", "child_r", "code", "index", "bb_min", "bb_max"):
        assert np.array_equal(nodes[f], onodes[f]), f


@pytest.mark.parametrize("mode", ["nearest+packet+wide", "binned+wide+refill", "auto"])
def test_c5_frame_matches_oracle_sampled_rows(mode):
    """The headline frame at full size (C5: 10M triangles, 3840x2160, primary + 1 bounce) in the
    bench's walk, against the oracle tracing 1 row in 4 on its OWN tree (OpenMP over rows):
    bit-identical pixels and intensities (tolerance 1e-4 stated)."""
    s = rt.synthetic(C5_SCENE["ntris"], seed=C5_SCENE["seed"], half_extent=C5_SCENE["half"])
    W, H = 3840, 2160
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=TRACE_MODES[mode]) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        fb = c.read_framebuffer()
        inten = c.read_intensity()
    os_ = _oscene(s)
    onodes = orc.build(os_, wvp)
    orc.set_threads(_oracle_threads())
    try:
        ofb, oint, ost = orc.trace(os_, onodes, wvp, wv, W, H, 1, 1, H, 4, want_intensity=True)
    finally:
        orc.set_threads(1)
    np.testing.assert_allclose(fb[1::4], ofb, atol=RGB_TOL, rtol=0)
    assert np.array_equal(fb[1::4], ofb)
    np.testing.assert_array_equal(inten[1::4], oint)
    assert ost["hits"] > 100_000 and ost["bounce"] > 100_000


def test_trace_c5_full_frame_modes_agree():
    """C5 at full size (10M triangles, 3840x2160, primary + 1 bounce): every traversal
    mode renders the identical frame (the reference-order mode is bit-exact vs the
    oracle by the tests above; the oracle itself is too slow for 16M rays here)."""
    s = rt.synthetic(10_000_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    W, H = 3840, 2160
    with rt.Context(device=0, flags=rt.FLAG_WIDE_BVH) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.build()
        frames = {}
        for mode, flags in TRACE_MODES.items():
            c.set_flags(flags)
            c.trace(W, H, 1)
            frames[mode] = c.read_framebuffer()
    for mode, fb in frames.items():
        assert np.array_equal(fb, frames["reference"]), mode


def test_wide_trace_on_any_build():
    """One node layout serves both walks: a build made without the wide flag traces
    with FLAG_WIDE_BVH to the same frame as the binary walk."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(320, 240))
        c.build()
        c.trace(320, 240, 1)
        ref = c.read_framebuffer()
        c.set_flags(rt.FLAG_WIDE_BVH | rt.FLAG_PACKET_PRIMARY)
        c.trace(320, 240, 1)
        assert np.array_equal(c.read_framebuffer(), ref)


def test_wide_view_records_match_binary_tree():
    """Slot 2p + side holds the record of p's child on that side (its children's boxes
    and ids, and its own index; a pseudo record for a leaf child): checked against the
    exported binary tree."""
    s = rt.synthetic(20_000, seed=7, half_extent=(30, 30, 20))
    W, H = 320, 240
    with rt.Context(device=0, flags=rt.FLAG_WIDE_BVH) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.build()
        nodes = c.read_bvh()
        w4 = c.read_wide()
    T = s.num_tris
    assert w4.shape == (2 * (T - 1), 16)
    f = w4.view(np.float32)
    par = nodes["parent"]

    def box(rec, side):   # (min xyz, max xyz) of child `side` in the record word layout
        b, z = (4, 10) if side else (0, 8)
        return np.array([rec[b], rec[b + 1], rec[z]]), np.array([rec[b + 2], rec[b + 3], rec[z + 1]])

    for k in (x for x in range(2 * T - 1) if x != T):   # every node but the root (reference layout: root = T)
        e = par[k] - T                       # parent internal index
        side = 0 if nodes["child_l"][par[k]] == k else 1
        rec, fr = w4[2 * e + side], f[2 * e + side]
        if k < T:   # leaf: its box, then the absent child's (the same box, min.z a quiet NaN)
            assert rec[12] == (0x80000000 | k) and rec[13] == 0xFFFFFFFF and rec[14] == (0x80000000 | k)
            lo, hi = box(fr, 0)
            np.testing.assert_array_equal(lo, nodes["bb_min"][k])
            np.testing.assert_array_equal(hi, nodes["bb_max"][k])
            assert rec[15] == 3 * _general_box(lo, hi)
            assert list(rec[4:8]) == list(rec[0:4]) and rec[10] == 0x7FC00000 and rec[11] == rec[9]
        else:
            cl, cr = nodes["child_l"][k], nodes["child_r"][k]
            ids = [(0x80000000 | x) if x < T else x - T for x in (cl, cr)]
            assert list(rec[12:15]) == ids + [k - T]
            gen = 0
            for sd, ch in ((0, cl), (1, cr)):
                lo, hi = box(fr, sd)
                np.testing.assert_array_equal(lo, nodes["bb_min"][ch])
                np.testing.assert_array_equal(hi, nodes["bb_max"][ch])
                gen |= _general_box(lo, hi) << sd
            assert rec[15] == gen


def _tiny_scene(seed=5):
    """Triangles at every scale down to the denormals (for the identity camera: clip space = object space):
    groups of a synthetic scene scaled by 2^0, 2^-40, 2^-70, 2^-100, 2^-118, 2^-126, 2^-135 -- edge bounds whose
    squares underflow and whose margin constant c is denormal (margin.h mt_edge_bound / mt_tcap_down)."""
    base = rt.synthetic(7000, seed=seed, half_extent=(1.0, 1.0, 1.0))
    v = base.vertices.copy()
    T = base.num_tris
    scales = np.float32(2.0) ** np.array([0, -40, -70, -100, -118, -126, -135], np.float32)
    tri_scale = scales[np.arange(T) % len(scales)]
    idx = base.indices.reshape(-1, 3)
    for k in range(3):   # (each vertex belongs to one triangle in the synthetic scenes)
        v[idx[:, k], :3] = v[idx[:, k], :3] * tri_scale[:, None]
    return rt.Scene(v, base.indices, base.mat_indices, base.materials)


def _edge_bound_np(e1, e2):
    """margin.h mt_edge_bound in numpy float32 (the device's operation order)."""
    sq = lambda e: (e[:, 0] * e[:, 0] + e[:, 1] * e[:, 1]) + e[:, 2] * e[:, 2]
    with np.errstate(invalid="ignore", under="ignore"):
        m = np.sqrt(np.maximum(sq(e1), sq(e2))) * np.float32(1 + 2.0 ** -20)
        mx = np.max(np.abs(np.concatenate([e1, e2], 1)), axis=1)
        tiny = (mx * np.float32(1.7320510)) * np.float32(1 + 2.0 ** -20) + np.float32(2.0 ** -149)
    out = np.where(mx < np.float32(2.0 ** -50), tiny, m)
    return np.where(np.isnan(m), np.float32(np.inf), out).astype(np.float32)


@pytest.mark.parametrize("scene", ["synthetic", "general boxes", "Test", "tiny triangles"])
def test_qnodes_contain_the_exact_boxes(scene):
    """Quantized node of internal node k (rtbvh_device.h QNode) at k's slot: power-of-two grid
    steps, the entries of the largest-area greedy collapse (build.hip greedy_qnode: from k's
    two children, the internal entry with the largest box surface replaced by its children,
    twice; internal entries by their slots), and decoded corners (origin + q * step in fp32,
    the traversal's arithmetic) that contain every entry's exact box.  The low 16 bits of the
    steps scl[1] / scl[2] carry the certified walk's per-node margin codes (margin.h
    mt_node_codes): the largest edge bound of the node's leaves rounded up -- exactly, from the
    clip-space triangles -- and a margin range no larger than that bound's.  Checked on the QNodes the
    4-wide walk reads -- the root's and, recursively, those of its entries' internal nodes (k_refit
    writes no other: DESIGN.md 2)."""
    if scene == "synthetic":
        s = rt.synthetic(20_000, seed=7, half_extent=(30, 30, 20))
    elif scene == "general boxes":
        s = _general_box_scene()
    elif scene == "tiny triangles":
        s = _tiny_scene()
    else:
        d = load_scene_fixture("Test")
        s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    cam = (np.eye(4, dtype=np.float32), np.eye(4, dtype=np.float32)) if scene == "tiny triangles" \
        else rt.camera_reference(320, 240)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*cam)
        c.build()
        nodes = c.read_bvh()
        q = c.read_qnodes()
    T = s.num_tris
    assert q.shape == (2 * T - 1, 16)
    cl, cr, par = nodes["child_l"], nodes["child_r"], nodes["parent"]

    def slot(x):   # reference-layout internal node x (>= T): its record's slot
        if x == T:
            return 2 * T - 2
        return 2 * (par[x] - T) + (0 if cl[par[x]] == x else 1)

    q = q[[slot(T + k) for k in range(T - 1)]]   # node-indexed from here on
    codes_e, codes_t = q[:, 4] & 0xFFFF, q[:, 5] & 0xFFFF
    q = q.copy()
    q[:, 3:6] &= np.uint32(0xFF800000)   # the steps without the margin codes
    f = q.view(np.float32)
    org, scl = f[:, 0:3], f[:, 3:6]
    shifts = np.arange(4, dtype=np.uint32) * 8
    lo = ((q[:, 6:9, None] >> shifts) & 255).astype(np.float32)   # [k, axis, c]
    hi = ((q[:, 9:12, None] >> shifts) & 255).astype(np.float32)
    dlo = org[:, :, None] + lo * scl[:, :, None]   # q * step exact; one rounding in the add
    dhi = org[:, :, None] + hi * scl[:, :, None]
    top = np.full((T - 1, 3), -np.inf, dtype=np.float32)   # the exact max corner of the four boxes
    bmin, bmax = nodes["bb_min"], nodes["bb_max"]

    def area(g):   # fp32, the kernel's operation order
        d = (bmax[g] - bmin[g]).astype(np.float32)
        return (d[0] * d[1] + d[1] * d[2]) + d[2] * d[0]

    def greedy(x):
        ents = [cl[x], cr[x]]
        for _ in range(2):
            best, pick = np.float32(-1), -1
            for idx in range(min(len(ents), 3)):
                if ents[idx] >= T:
                    ar = area(ents[idx])
                    if ar > best:
                        best, pick = ar, idx
            if pick < 0:
                break
            g = ents[pick]
            ents[pick] = cl[g]
            ents.append(cr[g])
        if len(ents) == 2:
            return [ents[0], None, ents[1], None]
        return ents + [None] * (4 - len(ents))

    read, todo = [], [0]   # the QNodes the walk reads: the root, then the entries' internal nodes
    while todo:
        k = todo.pop()
        read.append(k)
        todo.extend(g - T for g in greedy(T + k) if g is not None and g >= T)
    read = np.array(sorted(read))
    assert len(read) < 0.5 * (T - 1) or T < 3000   # (the greedy collapse expands about two in three)
    assert (scl[read, 0] != 0).all()   # every node of these scenes has a finite grid
    m, e = np.frexp(scl[read])
    assert (m == 0.5).all(), "grid steps are powers of two"
    for k in read:
        gc = greedy(T + k)
        ids = [0xFFFFFFFF if g is None else ((0x80000000 | g) if g < T else slot(g)) for g in gc]
        assert list(q[k, 12:16]) == ids, k
        for cidx, g in enumerate(gc):
            if g is None:
                continue
            assert (dlo[k, :, cidx] <= nodes["bb_min"][g]).all(), (k, cidx)
            assert (dhi[k, :, cidx] >= nodes["bb_max"][g]).all(), (k, cidx)
            top[k] = np.maximum(top[k], nodes["bb_max"][g])
    # the step is the smallest power of two (>= 2^-120) whose grid reaches the boxes' max
    half = scl / np.float32(2)
    reach = org + np.float32(255) * half   # product exact, one rounding in the add
    assert ((reach < top) | (half < np.float32(2.0 ** -120)))[read].all(), "grid step not minimal"
    # the margin codes: E_k = max over node k's leaves of margin.h mt_edge_bound on the clip-space
    # triangle (rtbvh_device.h xform_point's operation order, no FMA: numpy float32), rounded up
    wvp = cam[0].reshape(4, 4)
    P = s.vertices[:, :3].astype(np.float32)
    with np.errstate(under="ignore"):
        clip = ((P[:, 0:1] * wvp[0] + P[:, 1:2] * wvp[1]) + P[:, 2:3] * wvp[2]) + wvp[3]
    tri = clip[s.indices.reshape(-1, 3), :3]
    e1, e2 = tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]
    eb = _edge_bound_np(e1, e2)
    if scene == "tiny triangles":   # the bound is >= the exact 2-norm at every scale
        n64 = lambda e: np.sqrt((e.astype(np.float64) ** 2).sum(1))
        assert (eb.astype(np.float64) >= np.maximum(n64(e1), n64(e2))).all()
        assert (eb < 2.0 ** -100).sum() > 500
    leaf_e = eb[nodes["index"][:T] // 3]
    node_e = np.zeros(T - 1, np.float32)
    order = []   # internal nodes, children before parents
    st = [T]
    while st:
        x = st.pop()
        order.append(x)
        st.extend(c for c in (cl[x], cr[x]) if c >= T)

    def ev(c):
        return leaf_e[c] if c < T else node_e[c - T]
    for x in reversed(order):
        node_e[x - T] = max(ev(cl[x]), ev(cr[x]))
    want_e = ((node_e.view(np.uint32).astype(np.uint64) + 0xFFFF) >> 16).astype(np.uint32)
    np.testing.assert_array_equal(codes_e[read], want_e[read])
    eq = (codes_e[read] << 16).view(np.float32).astype(np.float64)
    tcn = (codes_t[read] << 16).view(np.float32).astype(np.float64)
    # the device's range (margin.h mt_tcap_down: the hardware reciprocal) against condition (C) in exact
    # arithmetic (float64; no allowance on the unsafe side): c (A t + 2 E) <= 0.2 for every t <= tcn; a
    # negative range covers no t
    c = 28.3 * 100.01 * (1 + 2.0 ** -18) * 2.0 ** -24 * eq
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        tcap = np.where(np.isfinite(eq), (0.2 / c - 2 * eq) / (1 + 2.0 ** -18), -1.0)
    assert np.where(tcap >= 0, tcn <= tcap, tcn < 0).all()
    big = (tcap >= 1) & (tcap < 2.0 ** 127)   # (the 16-bit code truncates: within 2^-8; 0.999 of mt_margin)
    assert (tcn[big] >= 0.99 * 0.999 * tcap[big]).all()


def _general_box(lo, hi):
    """Record word 15's bit (rtbvh_device.h): the box needs the general primary slab test."""
    ok = lo[0] < hi[0] and lo[1] < hi[1] and lo[2] <= hi[2] and 0 <= hi[2] < np.inf
    return 0 if ok else 1


def _general_box_scene(seed=11):
    """A synthetic scene plus triangles whose boxes take the general primary slab test:
    triangles in planes x = const (clip x = x * M0 exactly for the reference camera, so
    their boxes are flat in x), single-point triangles (flat in x and y), and triangles
    behind the eye (max.z < 0 in clip space)."""
    base = rt.synthetic(3000, seed=seed, half_extent=(30, 30, 20))
    rng = np.random.default_rng(seed)
    extra = []
    for _ in range(300):   # x = const
        x = rng.uniform(-25, 25)
        p = np.stack([np.full(3, x), rng.uniform(-25, 25, 3), rng.uniform(-20, 20, 3)], 1)
        extra.append(p)
    for _ in range(150):   # points
        extra.append(np.repeat(rng.uniform(-25, 25, (1, 3)), 3, 0))
    for _ in range(300):   # behind the eye (z = -100)
        extra.append(np.stack([rng.uniform(-40, 40, 3), rng.uniform(-40, 40, 3), rng.uniform(-160, -101, 3)], 1))
    pos = np.concatenate(extra).astype(np.float32)
    v = np.zeros((len(pos), 8), np.float32)
    v[:, :3] = pos
    v[:, 5] = -1.0
    V0 = len(base.vertices)
    verts = np.concatenate([base.vertices, v])
    idx = np.concatenate([base.indices, V0 + np.arange(len(pos), dtype=np.uint32)])
    mats = np.concatenate([base.mat_indices, np.zeros(len(pos) // 3, np.uint32)])
    return rt.Scene(verts, idx, mats, base.materials)


@pytest.mark.parametrize("mode", ["packet+wide", "nearest+packet+wide", "packet", "binned", "binned+wide+refill"])
def test_primary_general_boxes(mode):
    """Flat and behind-the-eye boxes (record word 15 set) in the axis-parallel primary walk:
    frames identical to the oracle's, and the record bits as the tree's boxes say."""
    s = _general_box_scene()
    fb, inten, st, ofb, oint, ost = _trace_both(s, 320, 240, 1, flags=TRACE_MODES[mode])
    assert np.array_equal(fb, ofb)
    np.testing.assert_array_equal(inten, oint)
    assert ost["hits"] > 0
    with rt.Context(device=0, flags=rt.FLAG_WIDE_BVH) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(320, 240))
        c.build()
        w4 = c.read_wide()
    assert np.count_nonzero(w4[:, 15]) > 100   # the general path is taken


@pytest.mark.parametrize("W,H", [(64, 64), (97, 53)])
def test_binned_primary_boxes_on_the_pixel_grid(W, H):
    """The binned pass's rectangles at their edges: with the identity camera, clip space is object
    space and the primary rays sit at multiples of 1/4 (RayTraceLaunch.hlsl:23-24), so triangles
    with vertices ON that grid put box edges exactly on rays -- the strict min < o < max of the
    axis-parallel test excludes them, and the build's footprint (leaf_footprint) must agree pixel
    for pixel.  Plus thin triangles (boxes narrower than a pixel, between two rays or through one),
    and an odd frame (W/2 rounds down).  Frames vs the CPU oracle, bit for bit: the primary pass
    alone with the fast walks (their 4-wide bounce walk meets containment failures on this grid of
    coincident vertices -- DESIGN.md 3 -- in the packet walk's frames as in the binned pass's), and
    primary + bounce with the binned pass beside the reference-order bounce."""
    from tests.containment import identity_camera
    rng = np.random.default_rng(5)
    tris = []
    for _ in range(4000):   # vertices on the quarter grid, boxes of 0..12 rays
        c = rng.integers(-4 * W // 8, 4 * W // 8, 2)
        p = (c[None, :] + rng.integers(-6, 7, (3, 2))) / 4.0
        tris.append(np.concatenate([p, rng.uniform(1, 60, (3, 1))], 1))
    for _ in range(1000):   # thin in x: width 0, 1/8 or 1/4 around a ray or between two
        x = rng.integers(-W // 2, W // 2) / 4.0 + rng.choice([0.0, 0.125, -0.125])
        wd = rng.choice([0.0, 0.125, 0.25])
        p = np.stack([[x, x + wd, x + wd / 2], rng.uniform(-H / 8, H / 8, 3), rng.uniform(1, 60, 3)], 1)
        tris.append(p)
    pos = np.concatenate(tris).astype(np.float32)
    v = np.zeros((len(pos), 8), np.float32)
    v[:, :3] = pos
    v[:, 5] = -1.0
    d = load_scene_fixture("Test")
    n = len(pos) // 3
    s = rt.Scene(v, np.arange(len(pos), dtype=np.uint32), (np.arange(n) % 3).astype(np.uint32), d["material_blob"])
    wvp, wv = identity_camera()
    os_ = _oscene(s)
    for flags, bounces in ((BINNED_FAST, 0), (rt.FLAG_BINNED_PRIMARY, 1)):
        with rt.Context(device=0, flags=flags) as c:
            c.set_scene(s)
            c.set_camera(wvp, wv)
            c.compute_bvh(W, H, bounces)
            fb = c.read_framebuffer()
            nodes = c.read_bvh()
        ofb, _, ost = orc.trace(os_, nodes, wvp, wv, W, H, bounces)
        np.testing.assert_array_equal(fb, ofb)
        assert ost["hits"] > W * H // 4


@pytest.mark.parametrize("mode", ["nearest+packet+wide", "reference", "nearest+packet+refill"])
@pytest.mark.parametrize("nsplit", [2, 3, 4])
def test_trace_chains_match_one_chain(mode, nsplit):
    """A trace dealt over nsplit primary -> bounce chains on their own streams renders the
    same frame, intensities, ray records and ray counts as one chain: whole frames, and
    band shards of N = 3 and 8 ranks (ragged frame, ranks with fewer bands than chains)."""
    import torch
    s = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    W, H = 1000, 357
    base = TRACE_MODES[mode] | rt.FLAG_REFRACT_RECORDS
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.build()
        out = {}
        for k in (1, nsplit):
            c.set_flags(base | k << rt.FLAG_SPLIT_SHIFT)
            c.trace(W, H, 2)
            st = c.stats()
            out[k] = (c.read_framebuffer(), c.read_intensity(), c.read_rays(), st["bounce_rays"])
            for nranks in (3, 8):
                for r in range(nranks):
                    rows = rt.lib().rtbvh_band_rows(H, r, nranks)
                    buf = torch.full((rows, W, 4), -1.0, dtype=torch.float32, device="cuda:0")
                    torch.cuda.synchronize()   # the fill runs on torch's stream, not the context's
                    c.trace_band_async(W, H, 2, r, nranks, buf.data_ptr())
                    c.synchronize()
                    out[(k, nranks, r)] = (buf.cpu().numpy(), c.stats()["bounce_rays"])
    fb1, in1, (rf1, rr1), nb1 = out[1]
    fbk, ink, (rfk, rrk), nbk = out[nsplit]
    assert np.array_equal(fbk, fb1) and np.array_equal(ink, in1) and nb1 == nbk and nb1 > 0
    assert np.array_equal(rfk.view(np.uint8), rf1.view(np.uint8)) and np.array_equal(rrk.view(np.uint8), rr1.view(np.uint8))
    for key in [k for k in out if isinstance(k, tuple) and k[0] == 1]:
        band, nb = out[key]
        band_k, nb_k = out[(nsplit,) + key[1:]]
        assert np.array_equal(band_k, band) and nb_k == nb, key


@pytest.mark.parametrize("nranks", [1, 3, 8])
def test_frames_in_flight_match_one_at_a_time(nranks):
    """Frames in flight (bench.py): one context, frames dealt over three caller streams
    (each gets a trace-buffer slot of its own over the one BVH) and traced back to back
    without synchronisation -- every frame equals the one traced alone on the context
    stream, and the stats are the last frame's; rank 1's bands of N ranks (N = 1: the
    whole frame).  A rebuild waits for the frames in flight."""
    import torch
    s = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    W, H = 1000, 357
    r = min(1, nranks - 1)
    rows = rt.lib().rtbvh_band_rows(H, r, nranks)
    streams = [torch.cuda.Stream() for _ in range(3)]
    with rt.Context(device=0, flags=TRACE_MODES["nearest+packet+wide"]) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.build()
        alone = torch.full((rows, W, 4), -1.0, dtype=torch.float32, device="cuda:0")
        bufs = [torch.full((rows, W, 4), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(6)]
        torch.cuda.synchronize()
        c.trace_band_async(W, H, 1, r, nranks, alone.data_ptr())
        c.synchronize()
        st_alone = c.stats()
        for i, b in enumerate(bufs):
            c.trace_band_async(W, H, 1, r, nranks, b.data_ptr(), stream_ptr=streams[i % 3].cuda_stream)
        c.build()   # waits for the frames in flight before it rewrites the BVH
        c.synchronize()
        torch.cuda.synchronize()
        st = c.stats()
        for i, b in enumerate(bufs):
            assert torch.equal(b, alone), i
        assert (alone[:, :, 3] != -1.0).all()
        assert st["bounce_rays"] == st_alone["bounce_rays"] > 0 and st["hits"] == st_alone["hits"]
        with pytest.raises(rt.RtbvhError):   # a fourth caller stream has no slot
            c.trace_band_async(W, H, 1, r, nranks, bufs[0].data_ptr(), stream_ptr=torch.cuda.Stream().cuda_stream)


def test_packet_frames_in_flight_after_a_binned_build():
    """A binned context's build leaves out the leaf pseudo-records; switched to the packet walk,
    its first frames go straight to caller streams (frames in flight): the pseudo-records are
    written on the context stream first and every slot's trace waits for them -- each frame equals
    the packet walk's frame on a tree built with them, and the binned frame is unchanged."""
    import torch
    s = rt.synthetic(200_000, seed=0x5EED0014, half_extent=(100, 100, 50))
    W, H = 800, 400
    streams = [torch.cuda.Stream() for _ in range(3)]
    packet = TRACE_MODES["nearest+packet+wide"]
    with rt.Context(device=0, flags=packet) as ref:
        ref.set_scene(s)
        ref.set_camera(*rt.camera_reference(W, H))
        ref.compute_bvh(W, H, 1)
        want = torch.from_numpy(ref.read_framebuffer()).to("cuda:0")
    with rt.Context(device=0, flags=BINNED_FAST) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.compute_bvh(W, H, 1)
        binned = c.read_framebuffer()
        c.set_flags(packet)
        bufs = [torch.full((H, W, 4), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(3)]
        torch.cuda.synchronize()
        for i, b in enumerate(bufs):
            c.trace_band_async(W, H, 1, 0, 1, b.data_ptr(), stream_ptr=streams[i].cuda_stream)
        c.synchronize()
        torch.cuda.synchronize()
        for i, b in enumerate(bufs):
            assert torch.equal(b, want), i
        np.testing.assert_array_equal(binned, want.cpu().numpy())


def test_compute_bvh_graph_replays_the_frame():
    """RTBVH_FLAG_GRAPH: compute_bvh captures build + trace into a hipGraph and replays it; the
    frames and trees equal a plain context's, across replays, the re-capture that a new frame size
    and bounce count force, and a new camera (replayed: the kernels read the camera buffer)."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    with rt.Context(device=0) as plain, rt.Context(device=0, flags=rt.FLAG_GRAPH) as g:
        for c in (plain, g):
            c.set_scene(s)
        for W, H, b, cam in [(320, 240, 1, (320, 240)), (320, 240, 1, (320, 240)), (400, 200, 2, (400, 200)),
                             (400, 200, 2, (640, 480)), (400, 200, 2, (640, 480))]:
            wvp, wv = rt.camera_reference(*cam)
            for c in (plain, g):
                c.set_camera(wvp, wv)
                c.compute_bvh(W, H, b)
            np.testing.assert_array_equal(g.read_framebuffer(), plain.read_framebuffer())
            np.testing.assert_array_equal(g.read_bvh()["bb_min"], plain.read_bvh()["bb_min"])
        assert g.stats()["graph_captures"] == 2   # (320, 240, 1), (400, 200, 2); the new camera replays


def test_graph_replay_writes_the_frame():
    """A replayed graph (not a re-capture) renders the frame: the camera set every frame with
    the same matrices (Graphics::onUpdate) keeps the graph; between replays the framebuffer is
    overwritten by a different frame of the same size (0 bounces), and each replay must restore
    the 1-bounce frame of a plain context, with one capture in all."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0) as plain, rt.Context(device=0, flags=rt.FLAG_GRAPH) as g:
        for c in (plain, g):
            c.set_scene(s)
            c.set_camera(wvp, wv)
        plain.compute_bvh(W, H, 1)
        want = plain.read_framebuffer()
        plain.trace(W, H, 0)
        other = plain.read_framebuffer()
        assert not np.array_equal(other, want)
        for i in range(4):
            g.set_camera(wvp.copy(), wv.copy())   # every frame, unchanged
            g.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(g.read_framebuffer(), want, err_msg=f"replay {i}")
            g.trace(W, H, 0)                      # overwrite the framebuffer between replays
            np.testing.assert_array_equal(g.read_framebuffer(), other)
        assert g.stats()["graph_captures"] == 1


def test_graph_replay_after_band_traces_and_other_sizes():
    """A replay after a band trace on a caller stream (a frame in flight over the BVH the replay
    rebuilds) and after a trace of another size: the replay waits for the frame in flight, and
    read_framebuffer returns the replayed W x H frame."""
    import torch
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    stream = torch.cuda.Stream()
    with rt.Context(device=0) as plain, rt.Context(device=0, flags=rt.FLAG_GRAPH) as g:
        for c in (plain, g):
            c.set_scene(s)
            c.set_camera(wvp, wv)
        plain.compute_bvh(W, H, 1)
        want = plain.read_framebuffer()
        g.compute_bvh(W, H, 1)
        band = torch.full((H, W, 4), -1.0, dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        g.trace_band_async(W, H, 1, 0, 1, band.data_ptr(), stream_ptr=stream.cuda_stream)
        g.compute_bvh(W, H, 1)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(band.cpu().numpy(), want)
        np.testing.assert_array_equal(g.read_framebuffer(), want)
        g.trace(200, 100, 2)                       # another size in between
        g.compute_bvh(W, H, 1)
        assert g.read_framebuffer().shape == (H, W, 4)
        np.testing.assert_array_equal(g.read_framebuffer(), want)


def test_graph_replay_after_a_larger_trace_reallocates():
    """compute_bvh(320x240) -> trace(640x480) -> compute_bvh(320x240): the larger trace
    reallocates the trace buffers the captured graph points at, so the context drops the graph
    and captures again; the replayed frame is the plain context's and read_framebuffer returns
    it (a stale graph wrote to freed buffers)."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0) as plain, rt.Context(device=0, flags=rt.FLAG_GRAPH) as g:
        for c in (plain, g):
            c.set_scene(s)
            c.set_camera(wvp, wv)
        plain.compute_bvh(W, H, 1)
        want = plain.read_framebuffer()
        g.compute_bvh(W, H, 1)
        g.compute_bvh(W, H, 1)
        assert g.stats()["graph_captures"] == 1
        g.trace(640, 480, 1)        # grows every trace buffer
        plain.trace(640, 480, 1)
        np.testing.assert_array_equal(g.read_framebuffer(), plain.read_framebuffer())
        for _ in range(2):
            g.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(g.read_framebuffer(), want)
        assert g.stats()["graph_captures"] == 2


@pytest.mark.parametrize("mode", ["reference", "nearest", "packet", "nearest+packet", "nearest+packet+refill",
                                  "nearest+packet+wide", "refill+sort"])
def test_stack_limit_reports_overflow(mode):
    """rtbvh_config.stack_limit: a ray whose stack would exceed the limit ends early and the
    synchronising call returns RTBVH_ERR_STACK_OVERFLOW once (the frame is complete); with the
    compiled capacity, and with the reference's 32 entries on its own mesh, nothing overflows."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 320, 240
    frames = {}
    for limit in (0, 32, 2):
        with rt.Context(device=0, flags=TRACE_MODES[mode], stack_limit=limit) as c:
            c.set_scene(s)
            c.set_camera(*rt.camera_reference(W, H))
            c.build()
            if limit == 2:
                with pytest.raises(rt.RtbvhError) as e:
                    c.trace(W, H, 1)
                assert e.value.status == rt._lib.ERR_STACK_OVERFLOW
                assert "stack" in str(e.value)
                assert c.stats()["stack_overflows"] > 0
                c.synchronize()   # reported once
            else:
                c.trace(W, H, 1)
                assert c.stats()["stack_overflows"] == 0
            c.width, c.height = W, H
            frames[limit] = c.read_framebuffer()
    np.testing.assert_array_equal(frames[32], frames[0])
    assert not np.array_equal(frames[2], frames[0])


CERT_WALKS = rt.FLAG_NEAREST_FIRST | rt.FLAG_REFILL_BOUNCE | rt.FLAG_WIDE_BVH | rt.FLAG_BINNED_PRIMARY


def test_verify_walk_and_auto_walk():
    """rtbvh_verify_walk: the fast walks render the reference-order frame (0 differing pixels);
    RTBVH_FLAG_AUTO_WALK takes the reference-order kernels on small scenes (lanes or wave packets for the
    primary rays, whichever its first frame timed faster) and, on large ones, the
    certified fast walks (binned primary pass, 4-wide bounce walk, per-ray certificates)
    from the first frame on (walk_state 2), with the reference frame throughout."""
    d = load_scene_fixture("Test")
    small = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    big = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    W, H = 960, 540
    for s, walk in ((small, 0), (big, CERT_WALKS)):
        with rt.Context(device=0) as ref, rt.Context(device=0, flags=rt.FLAG_AUTO_WALK) as auto, \
                rt.Context(device=0, flags=TRACE_MODES["nearest+packet+wide"]) as fast:
            for c in (ref, auto, fast):
                c.set_scene(s)
                c.set_camera(*rt.camera_reference(W, H))
                c.compute_bvh(W, H, 1)
            want = ref.read_framebuffer()
            for k in range(2):
                st = auto.stats()
                # (small scenes: the lane or the wave-packet reference-order primary pass, timed on the first frame)
                assert st["walk_flags"] in ((walk,) if walk else (0, rt.FLAG_PACKET_PRIMARY))
                assert st["walk_state"] == (2 if walk else 0)
                assert st["cert_traces"] == (k + 1 if walk else 0)
                np.testing.assert_array_equal(auto.read_framebuffer(), want)
                np.testing.assert_array_equal(auto.read_intensity(), ref.read_intensity())
                auto.compute_bvh(W, H, 1)
            assert fast.verify_walk(W, H, 1) == 0
            np.testing.assert_array_equal(fast.read_framebuffer(), want)
            assert auto.verify_walk(W, H, 1) == 0


def test_containment_failure_auto_walk_returns_the_reference_frame():
    """On a scene where containment fails (tests/containment.py: two coplanar triangles whose
    Moller-Trumbore t rounds below their slab entry), the 4-wide packet walk's frame DIFFERS from
    findCollision's (RayTraceTraversal.hlsl:106-193) at PIXEL, and rtbvh_verify_walk reports it.
    RTBVH_FLAG_AUTO_WALK (the scene is above its 65536-triangle size) takes the certified walks: the
    pixel's hit (B, whose t lies below its own box's entry) fails its certificate and is re-traced in
    the reference order (redo_rays[0] >= 1), so the frame is the reference's -- equal to the CPU
    oracle's -- on every frame, also through the hipGraph path."""
    from tests.containment import PIXEL, H, W, containment_scene, identity_camera
    s = containment_scene()
    wvp, wv = identity_camera()
    os_ = orc.Scene(s.vertices, s.indices, s.mat_indices, s.material_blob)
    ofb, _, _ = orc.trace(os_, orc.build(os_, wvp), wvp, wv, W, H, 1)
    x, y = PIXEL
    with rt.Context(device=0) as ref, rt.Context(device=0, flags=TRACE_MODES["nearest+packet+wide"]) as fast, \
            rt.Context(device=0, flags=rt.FLAG_AUTO_WALK) as auto, \
            rt.Context(device=0, flags=rt.FLAG_AUTO_WALK | rt.FLAG_GRAPH) as gauto:
        for c in (ref, fast, auto, gauto):
            c.set_scene(s)
            c.set_camera(wvp, wv)
            c.compute_bvh(W, H, 1)
        want = ref.read_framebuffer()
        np.testing.assert_array_equal(want, ofb)
        got = fast.read_framebuffer()
        assert not np.array_equal(got[y, x], want[y, x])     # the fast walk took A, the reference B
        assert fast.verify_walk(W, H, 1) > 0
        for c in (auto, gauto):
            for _ in range(3):
                st = c.stats()
                assert st["walk_state"] == 2 and st["walk_flags"] == CERT_WALKS
                assert st["redo_rays"][0] >= 1 and st["redo_total"] >= 1
                np.testing.assert_array_equal(c.read_framebuffer(), want)
                c.set_camera(wvp.copy(), wv.copy())   # every frame, unchanged (Graphics::onUpdate)
                c.compute_bvh(W, H, 1)
        assert gauto.stats()["graph_captures"] == 1


def test_auto_walk_orbit_replays_one_graph():
    """the reference's only interaction orbits the eye (Graphics::onKeyDown,
    Graphics.cpp:937-960) and re-uploads WVP / WV every frame (Graphics.cpp:40-56).  Under
    RTBVH_FLAG_AUTO_WALK | RTBVH_FLAG_GRAPH at 200k triangles, five distinct cameras (four key presses)
    replay ONE captured graph (graph_captures == 1; the camera lives in a device buffer) with the
    certified walks, and every frame equals the reference-order frame of its camera (and the CPU
    oracle's on one of them)."""
    s = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    W, H, B = 960, 540, 1
    eye = np.array(rt.EYE_REFERENCE, np.float32)
    cams = []
    for key in (None, rt.KEY_LEFT, rt.KEY_LEFT, rt.KEY_UP, rt.KEY_RIGHT):
        if key is not None:
            eye = rt.camera_orbit(eye, key)
        cams.append(rt.camera_look(eye, W, H))
    with rt.Context(device=0, flags=rt.FLAG_AUTO_WALK | rt.FLAG_GRAPH) as g, rt.Context(device=0) as ref:
        g.set_scene(s)
        ref.set_scene(s)
        for i, (wvp, wv) in enumerate(cams):
            g.set_camera(wvp, wv)
            g.compute_bvh(W, H, B)
            ref.set_camera(wvp, wv)
            ref.compute_bvh(W, H, B)
            want = ref.read_framebuffer()
            np.testing.assert_array_equal(g.read_framebuffer(), want, err_msg=f"camera {i}")
            np.testing.assert_array_equal(g.read_intensity(), ref.read_intensity())
            st = g.stats()
            assert st["graph_captures"] == 1 and st["walk_state"] == 2 and st["walk_flags"] == CERT_WALKS
            if i == 2:   # the oracle on one camera (1 row in 8)
                nodes = ref.read_bvh()
                np.testing.assert_array_equal(g.read_bvh()["bb_min"], nodes["bb_min"])
                ofb, _, _ = orc.trace(_oscene(s), nodes, wvp, wv, W, H, B, 0, H, 8)
                np.testing.assert_array_equal(want[0:H:8], ofb)
        assert len({c[0].tobytes() for c in cams}) == 5


def _material(ns=300.0):
    m = np.zeros(1, rt._lib.MATERIAL_DTYPE)
    m[0]["diffuse"] = (0.64, 0.64, 0.64, 1.0)
    m[0]["specular"] = (0.5, 0.5, 0.5, 1.0)
    m[0]["shininess"] = ns
    m[0]["alpha"] = 1.0
    m[0]["tex_num"] = -1
    return m


def _mesh(tris, normals):
    """rt.Scene from (n, 3, 3) positions and (n, 3) per-triangle vertex normals, one material."""
    n = len(tris)
    v = np.zeros((3 * n, 8), np.float32)
    v[:, :3] = tris.reshape(-1, 3)
    v[:, 3:6] = np.repeat(normals, 3, axis=0)
    return rt.Scene(v, np.arange(3 * n, dtype=np.uint32), np.zeros(n, np.uint32), _material())


def _grid(n0, n1, lo0, lo1, step):
    """Two triangles per cell of an n0 x n1 grid (cell corners at lo + step * i): (2 n0 n1, 3, 2)."""
    i, j = np.meshgrid(np.arange(n0), np.arange(n1), indexing="ij")
    a0, a1 = (lo0 + step * i).ravel(), (lo1 + step * j).ravel()
    b0, b1 = a0 + step, a1 + step
    t1 = np.stack([np.stack([a0, a1], 1), np.stack([b0, a1], 1), np.stack([b0, b1], 1)], 1)
    t2 = np.stack([np.stack([a0, a1], 1), np.stack([b0, b1], 1), np.stack([a0, b1], 1)], 1)
    return np.concatenate([t1, t2])


def _far_wall_scene(big=True):
    """Identity camera (clip space = object space; tests/containment.py): a mirror of small triangles
    in the plane z = 10 over the frame, whose shading normal (~(0.70, 0.02, -0.714)) reflects the
    primary rays (d = +z) to ~(1, 0.03, -0.02), and a wall of small triangles at x = 450 facing them:
    almost every bounce ray's hit lies at t ~ 370..530.  With `big`, one huge triangle far outside every ray's path makes
    the scene's largest edge ~1000: the scene-wide margin's range (margin.h tcap) is then negative --
    round 4's certified walk could prune no bounce box by distance past t ~ 0 and walked exhaustively;
    per-node margins (the mirror's and the wall's QNodes carry edges ~1.4, tcap ~ 840) prune as
    usual."""
    g = _grid(161, 121, -80.1, -60.1, 1.0)   # x, y (no cell edge on the primary rays' quarter grid)
    mirror = np.concatenate([g, np.full(g.shape[:2] + (1,), 10.0)], 2)
    w = _grid(170, 40, -85.0, -20.0, 1.0)    # y, z
    wall = np.concatenate([np.full(w.shape[:2] + (1,), 450.0), w], 2)
    tris = [mirror, wall]
    nrm = [np.tile([0.70, 0.02, -0.714], (len(mirror), 1)), np.tile([-1.0, 0.0, 0.0], (len(wall), 1))]
    if big:
        tris.append(np.array([[[0.0, 3000.0, 0.0], [1000.0, 3000.0, 0.0], [0.0, 3000.0, 1000.0]]]))
        nrm.append(np.array([[0.0, -1.0, 0.0]]))
    return _mesh(np.concatenate(tris).astype(np.float32), np.concatenate(nrm).astype(np.float32))


def _counts(s, wvp, wv, W, H, flags):
    with rt.Context(device=0, flags=flags | rt.FLAG_COUNT_VISITS) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        return c.read_framebuffer(), c.stats()


@pytest.mark.parametrize("big", [False, True])
def test_certified_walk_prunes_past_the_scene_margin_range(big):
    """bounce hits past the scene-wide margin's range (margin.h tcap of the largest
    edge; with `big` every t is past it).  The certified walk grows each box by its OWN node's margin
    (the largest edge bound below it, carried by the QNode), so it still prunes by distance there: its
    frame equals the reference order's (and the oracle's), its bounce visits stay within 1.3x the
    unchecked 4-wide walk's (round 4's walk, which stopped pruning past the scene's range, visited every
    box the rays crossed), and (almost) no ray is re-traced."""
    from tests.containment import identity_camera
    s = _far_wall_scene(big)
    wvp, wv = identity_camera()
    W, H = 640, 480
    ref, _ = _counts(s, wvp, wv, W, H, 0)
    os_ = _oscene(s)
    ofb, _, _ = orc.trace(os_, orc.build(os_, wvp), wvp, wv, W, H, 1, 0, H, 4)
    np.testing.assert_array_equal(ref[0:H:4], ofb)
    cert, cst = _counts(s, wvp, wv, W, H, rt.FLAG_CERTIFIED)
    fast, fst = _counts(s, wvp, wv, W, H, TRACE_MODES["nearest+packet+wide"])
    np.testing.assert_array_equal(cert, ref)
    assert cst["bounce_rays"] > 200_000 and cst["hits"][1] > 0.9 * cst["bounce_rays"]
    assert cst["redo_rays"][1] <= 0.001 * cst["bounce_rays"]
    assert cst["internal_visits"][1] <= 1.3 * fst["internal_visits"][1], (cst["internal_visits"], fst["internal_visits"])


def test_certified_walks_with_a_few_huge_triangles():
    """one large triangle used to set the scene-wide edge bound, collapsing the margin's range
    for every ray (every bounce ray re-traced in the reference order).  A C5-like 200k-triangle scene plus
    three triangles of ~60-unit edges off to the side: the certified frame (RTBVH_FLAG_AUTO_WALK) equals
    the reference order's, (almost) no bounce ray is re-traced, and the walk stays within 1.3x the unchecked
    walk's visits -- only the few subtrees holding the huge triangles lose distance pruning."""
    base = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    huge = np.array([[[-190, -190, 40], [-120, -190, 40], [-190, -120, 45]],
                     [[190, 190, -40], [120, 190, -40], [190, 120, -45]],
                     [[-190, 190, 0], [-150, 150, 30], [-120, 190, -30]]], np.float32)
    v = np.zeros((9, 8), np.float32)
    v[:, :3] = huge.reshape(-1, 3)
    v[:, 5] = -1.0
    V0 = len(base.vertices)
    s = rt.Scene(np.concatenate([base.vertices, v]), np.concatenate([base.indices, V0 + np.arange(9, dtype=np.uint32)]),
                 np.concatenate([base.mat_indices, np.zeros(3, np.uint32)]), base.materials)
    W, H = 800, 450
    wvp, wv = rt.camera_reference(W, H)
    ref, _ = _counts(s, wvp, wv, W, H, 0)
    auto, ast = _counts(s, wvp, wv, W, H, rt.FLAG_AUTO_WALK)
    fast, fst = _counts(s, wvp, wv, W, H, TRACE_MODES["nearest+packet+wide"])
    np.testing.assert_array_equal(auto, ref)
    assert ast["walk_state"] == 2 and ast["bounce_rays"] > 0
    assert ast["redo_rays"][1] <= 0.001 * ast["bounce_rays"]
    assert ast["internal_visits"][1] <= 1.3 * fst["internal_visits"][1], (ast["internal_visits"], fst["internal_visits"])


@pytest.mark.parametrize("obj", ["Test", "Image_Test"])
def test_auto_walk_small_scene_primary_kind(obj):
    """RTBVH_FLAG_AUTO_WALK on a small scene times the reference order's lane and wave-packet primary passes
    on the first frame and keeps the faster (api.hip enqueue_trace): whichever it keeps, the frame -- traced
    directly and replayed as a hipGraph -- is the reference order's, and the stats name the kind."""
    s = load_scene_fixture(obj)
    sc = rt.Scene(s["vertices"], s["indices"], s["mat_indices"], s["material_blob"])
    W, H = 640, 360
    cam = rt.camera_reference(W, H)
    with rt.Context(device=0) as ref, rt.Context(device=0, flags=rt.FLAG_AUTO_WALK) as auto, \
            rt.Context(device=0, flags=rt.FLAG_AUTO_WALK | rt.FLAG_GRAPH) as graph:
        for c in (ref, auto, graph):
            c.set_scene(sc)
            c.set_camera(*cam)
        ref.compute_bvh(W, H, 1)
        want = ref.read_framebuffer()
        for _ in range(2):
            auto.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(auto.read_framebuffer(), want)
        assert auto.stats()["walk_flags"] in (0, rt.FLAG_PACKET_PRIMARY)
        for _ in range(3):
            graph.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(graph.read_framebuffer(), want)
        assert graph.stats()["walk_flags"] in (0, rt.FLAG_PACKET_PRIMARY)


def test_certified_walks_end_at_nodes_without_a_grid():
    """A QNode whose boxes reach past 2^100 keeps no 8-bit grid (build.hip quantize_axis): the certified
    walk ends a ray there, flagged, and the reference-order re-trace takes it.  A 20k-triangle scene plus
    two triangles at x ~ 1e31: every node above them has no grid, so the certified frame must come from
    re-traced rays wherever the walk meets one -- and equal the reference order's."""
    base = rt.synthetic(20_000, seed=77, half_extent=(60, 60, 30))
    far = np.array([[[1e31, 0, 10], [1.0001e31, 0, 10], [1e31, 5, 12]],
                    [[-1e31, 0, 10], [-1.0001e31, 0, 10], [-1e31, 5, 12]]], np.float32)
    v = np.zeros((6, 8), np.float32)
    v[:, :3] = far.reshape(-1, 3)
    v[:, 5] = -1.0
    V0 = len(base.vertices)
    s = rt.Scene(np.concatenate([base.vertices, v]), np.concatenate([base.indices, V0 + np.arange(6, dtype=np.uint32)]),
                 np.concatenate([base.mat_indices, np.zeros(2, np.uint32)]), base.materials)
    W, H = 320, 180
    wvp, wv = rt.camera_reference(W, H)
    ref, _ = _counts(s, wvp, wv, W, H, 0)
    cert, st = _counts(s, wvp, wv, W, H, rt.FLAG_CERTIFIED)
    np.testing.assert_array_equal(cert, ref)
    assert st["bounce_rays"] > 0 and st["redo_rays"][1] > 0, st["redo_rays"]


def test_certified_walks_flag_rays_they_cannot_take():
    """Rays the certified bounce walk cannot vouch for are re-traced in the reference order: here the
    bounce rays of triangles whose shading normal is (0, 0, -1) -- under the reference camera (WV's x
    axis is exactly (1, 0, 0)) they reflect the primary rays' d = (0, 0, 1) into a direction with an
    exact zero x component, |1/d.x| = inf, which the slack test (qnode_fast_ray) cannot take.  The frame
    equals the reference's, and the re-trace count is the number of such rays."""
    s = _flat_normal_scene()   # every 7th triangle's normals (0, 0, -1)
    W, H = 640, 360
    with rt.Context(device=0) as ref, rt.Context(device=0, flags=rt.FLAG_AUTO_WALK) as auto:
        for c in (ref, auto):
            c.set_scene(s)
            c.set_camera(*rt.camera_reference(W, H))
            c.compute_bvh(W, H, 1)
        np.testing.assert_array_equal(auto.read_framebuffer(), ref.read_framebuffer())
        np.testing.assert_array_equal(auto.read_intensity(), ref.read_intensity())
        st = auto.stats()
        assert st["walk_state"] == 2 and st["bounce_rays"] > 0
        assert 0.05 * st["bounce_rays"] < st["redo_rays"][1] < 0.3 * st["bounce_rays"]


def _flat_normal_scene():
    s = rt.synthetic(200_000, seed=0x5EED0005, half_extent=(100, 100, 50))
    v = s.vertices.copy()
    v[(np.arange(len(v)) // 3) % 7 == 0, 3:6] = (0.0, 0.0, -1.0)
    return rt.Scene(v, s.indices, s.mat_indices, s.materials)


@pytest.mark.parametrize("nranks,share", [(2, 16), (3, 11), (8, 13)])
def test_certified_band_traces_and_frames_in_flight(nranks, share):
    """the certified walks on band traces (nranks > 1, the weighted deal) and on
    caller-stream slots (frames in flight), with re-traced rays on every rank and slot: the per-slot
    re-trace lists and k_primary_redo / k_bounce_redo's compact-row pixel index.  Each rank's bands,
    traced alone and as three frames in flight, put back in their rows, give the reference-order frame;
    bounce rays are re-traced on every rank (the scene's flat-normal triangles), and the containment
    scene's primary pixel is re-traced on the rank that owns its row."""
    import torch

    from raytracebvh_amd.tiles import band_row_ids
    from tests.containment import PIXEL, containment_scene, identity_camera
    cases = [(_flat_normal_scene(), 640, 357, rt.camera_reference(640, 357), 1),
             (containment_scene(), 64, 64, identity_camera(), 0)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for s, W, H, (wvp, wv), kind in cases:
        with rt.Context(device=0) as ref, rt.Context(device=0, flags=rt.FLAG_CERTIFIED) as c:
            for x in (ref, c):
                x.set_scene(s)
                x.set_camera(wvp, wv)
                x.compute_bvh(W, H, 1)
            want = ref.read_framebuffer()
            np.testing.assert_array_equal(c.read_framebuffer(), want)
            c.set_band_deal(share)
            frame = np.zeros_like(want)
            redo = []
            for r in range(nranks):
                rows = rt.lib().rtbvh_deal_rows(H, r, nranks, share)
                alone = torch.full((rows, W, 4), -1.0, dtype=torch.float32, device="cuda:0")
                bufs = [torch.full((rows, W, 4), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(3)]
                torch.cuda.synchronize()
                c.trace_band_async(W, H, 1, r, nranks, alone.data_ptr())
                c.synchronize()
                redo.append(c.stats()["redo_rays"][kind])
                for i, b in enumerate(bufs):
                    c.trace_band_async(W, H, 1, r, nranks, b.data_ptr(), stream_ptr=streams[i].cuda_stream)
                c.synchronize()
                torch.cuda.synchronize()
                for i, b in enumerate(bufs):
                    assert torch.equal(b, alone), (r, i)
                assert c.stats()["redo_rays"][kind] == redo[-1]
                frame[band_row_ids(H, r, nranks, share)] = alone.cpu().numpy()
            np.testing.assert_array_equal(frame, want)
            if kind == 1:
                assert all(n > 0 for n in redo), redo
            else:
                owner = [r for r in range(nranks) if PIXEL[1] in band_row_ids(H, r, nranks, share)]
                assert redo[owner[0]] >= 1, redo


@pytest.mark.parametrize("nranks,share", [(2, 16), (3, 16), (8, 16), (3, 11), (8, 13)])
def test_band_split_reassembles_full_frame(nranks, share):
    """Every rank's bands under the deal (16: b % nranks; below: rank 0 takes share/16 of a
    share, tiles.band_row_ids) put back in their rows give the full frame."""
    import torch

    from raytracebvh_amd.tiles import band_row_ids
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 640, 357
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        full = c.read_framebuffer()
        c.set_band_deal(share)
        frame = np.zeros_like(full)
        for r in range(nranks):
            rows = rt.lib().rtbvh_deal_rows(H, r, nranks, share)
            buf = torch.zeros((rows, W, 4), dtype=torch.float32, device="cuda:0")
            torch.cuda.synchronize()   # the fill runs on torch's stream, not the context's
            c.trace_band_async(W, H, 1, r, nranks, buf.data_ptr())
            c.synchronize()
            got = buf.cpu().numpy()
            ys = band_row_ids(H, r, nranks, share)
            assert len(ys) == rows
            frame[ys] = got
    np.testing.assert_array_equal(frame, full)


BINNED_FAST = WALK_FLAGS | rt.FLAG_BINNED_PRIMARY


@pytest.mark.parametrize("nranks,share", [(1, 16), (2, 16), (3, 11), (8, 13)])
def test_binned_band_traces_match_oracle(nranks, share):
    """RTBVH_FLAG_BINNED_PRIMARY on a rank's bands (the footprints in the rank's compact rows, a
    ragged 357-row frame, the even and the weighted deal): every rank's bands put back in their
    rows give the oracle's frame (C4 at 1/16 size: a dense random scene, many leaves per tile)."""
    import torch

    from raytracebvh_amd.tiles import band_row_ids
    s = rt.synthetic(200_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))
    W, H = 640, 357
    wvp, wv = rt.camera_reference(W, H)
    os_ = _oscene(s)
    with rt.Context(device=0, flags=BINNED_FAST) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        nodes = c.read_bvh()
        ofb, _, _ = orc.trace(os_, nodes, wvp, wv, W, H, 1)
        np.testing.assert_array_equal(c.read_framebuffer(), ofb)
        c.set_band_deal(share)
        frame = np.zeros_like(ofb)
        for r in range(nranks):
            rows = rt.lib().rtbvh_deal_rows(H, r, nranks, share)
            buf = torch.zeros((rows, W, 4), dtype=torch.float32, device="cuda:0")
            torch.cuda.synchronize()
            c.trace_band_async(W, H, 1, r, nranks, buf.data_ptr())
            c.synchronize()
            frame[band_row_ids(H, r, nranks, share)] = buf.cpu().numpy()
    np.testing.assert_array_equal(frame, ofb)


def test_binned_band_traces_tall_frame():
    """A frame of more than 16,384 rows (2,048 bands): the bin passes read the deal from memory instead of
    their per-block LDS copy (pb_bin.h PB_LDS_BANDS); every rank's bands put back give the whole frame."""
    import torch

    from raytracebvh_amd.tiles import band_row_ids
    s = rt.synthetic(20_000, seed=0x5EED0004, half_extent=(50.0, 50.0, 50.0))
    W, H, nranks, share = 24, 16_411, 3, 11
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=BINNED_FAST) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        full = c.read_framebuffer()
        assert (full[..., :3] != 0).any()
        c.set_band_deal(share)
        frame = np.zeros_like(full)
        for r in range(nranks):
            rows = rt.lib().rtbvh_deal_rows(H, r, nranks, share)
            buf = torch.zeros((rows, W, 4), dtype=torch.float32, device="cuda:0")
            torch.cuda.synchronize()
            c.trace_band_async(W, H, 1, r, nranks, buf.data_ptr())
            c.synchronize()
            frame[band_row_ids(H, r, nranks, share)] = buf.cpu().numpy()
    np.testing.assert_array_equal(frame, full)


@pytest.mark.parametrize("overlap", ["0", "1"])
@pytest.mark.parametrize("tris", [3000, 300_000])
def test_rebuilt_frame_overlap_matches_build_then_trace(tris, overlap, monkeypatch):
    """rtbvh_compute_bvh with the binned primary pass, and with RTBVH_OVERLAP=1 the pass on a side
    stream from the moment the build's leaves are written (ev_leaf, after k_refit + k_zrange),
    beside the crossing nodes (k_refit_top, k_qnodes_cross); the walk of overflowed tiles and the
    bounce wait for it.  Frame, intensities, counts and tree equal build() then trace() on one
    stream -- plain, timed, and as a replayed hipGraph -- over frames and a scene change (3000
    triangles: also the oracle's frame)."""
    monkeypatch.setenv("RTBVH_OVERLAP", overlap)
    W, H = 640, 360
    wvp, wv = rt.camera_reference(W, H)
    f = BINNED_FAST | rt.FLAG_MULTI_KERNEL_BUILD | rt.FLAG_COUNT_VISITS
    scenes = [rt.synthetic(tris, seed=0x5EED0011), rt.synthetic(tris, seed=0x5EED0012, half_extent=(100, 100, 50))]
    with rt.Context(device=0, flags=f) as a, rt.Context(device=0, flags=f | rt.FLAG_TIMING) as b, \
            rt.Context(device=0, flags=f | rt.FLAG_GRAPH) as g:
        for k, sc in enumerate(scenes):
            for c in (a, b, g):
                c.set_scene(sc)
                c.set_camera(wvp, wv)
            a.build()
            a.trace(W, H, 1)
            want, want_i, want_st = a.read_framebuffer(), a.read_intensity(), a.stats()
            assert want_st["bounce_rays"] > 0 and sum(want_st["hits"]) > 0
            if tris == 3000 and k == 0:
                ofb, _, ost = orc.trace(_oscene(sc), a.read_bvh(), wvp, wv, W, H, 1)
                np.testing.assert_array_equal(want, ofb)
                assert sum(want_st["hits"]) == ost["hits"]
            for c in (b, g):
                for frame in range(3):
                    c.compute_bvh(W, H, 1)
                    np.testing.assert_array_equal(c.read_framebuffer(), want, err_msg=f"scene {k} frame {frame}")
                    np.testing.assert_array_equal(c.read_intensity(), want_i)
                    st = c.stats()
                    for key in ("hits", "bounce_rays"):
                        assert np.array_equal(np.asarray(st[key]), np.asarray(want_st[key])), key
                    # the entries binned (entries past the block test depend on the tiles' claim order)
                    assert st["bin_entries"][0] == want_st["bin_entries"][0]
                np.testing.assert_array_equal(c.read_bvh()["bb_min"], a.read_bvh()["bb_min"])
        assert g.stats()["graph_captures"] == 2


def _far_scene(seed=5):
    """A synthetic scene plus small triangles ~1e33 away: the nodes above them have corners past
    2^100, so their QNodes carry no grid and the 4-wide bounce walk reads their exact records
    (trace.hip qchildren), leaf children among them."""
    base = rt.synthetic(6000, seed=seed, half_extent=(30, 30, 20))
    rng = np.random.default_rng(seed)
    tris = []
    for k in range(64):
        c = np.array([(1 if k % 2 else -1) * 1e33 * rng.uniform(1, 2), rng.uniform(-25, 25), rng.uniform(-20, 20)])
        tris.append(c + rng.uniform(-0.5, 0.5, (3, 3)))
    pos = np.concatenate(tris).astype(np.float32)
    v = np.zeros((len(pos), 8), np.float32)
    v[:, :3] = pos
    v[:, 5] = -1.0
    V0 = len(base.vertices)
    verts = np.concatenate([base.vertices, v])
    idx = np.concatenate([base.indices, V0 + np.arange(len(pos), dtype=np.uint32)])
    mats = np.concatenate([base.mat_indices, np.zeros(len(pos) // 3, np.uint32)])
    return rt.Scene(verts, idx, mats, base.materials)


@pytest.mark.parametrize("mode", ["reference", "nearest+packet+wide", "binned+wide+refill"])
def test_nodes_without_a_grid_trace_their_exact_records(mode):
    """QNodes without a finite grid (corners past 2^100): the 4-wide bounce walk takes the node's
    exact records -- a leaf child from the node's own record, as a binned build writes no leaf
    pseudo-records -- and the frame equals the oracle's over two bounces."""
    s = _far_scene()
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=TRACE_MODES[mode] | rt.FLAG_MULTI_KERNEL_BUILD | rt.FLAG_COUNT_VISITS) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 2)
        fb, st = c.read_framebuffer(), c.stats()
        nodes, q = c.read_bvh(), c.read_qnodes()
    T = s.num_tris
    internal = np.zeros(2 * T - 1, bool)
    par, cl = nodes["parent"], nodes["child_l"]
    for x in range(T + 1, 2 * T - 1):   # internal nodes but the root: their slots
        p = par[x] - T
        internal[2 * p + (0 if cl[par[x]] == x else 1)] = True
    internal[2 * T - 2] = True
    assert (q[internal, 3].view(np.float32) == 0).sum() >= 8   # nodes without a grid
    ofb, _, ost = orc.trace(_oscene(s), nodes, wvp, wv, W, H, 2)
    np.testing.assert_array_equal(fb, ofb)
    assert st["bounce_rays"] == ost["bounce"] > 0 and sum(st["hits"]) == ost["hits"]


def _huge_scene(seed=9, T=8000):
    """A synthetic scene of T triangles, 400 of them huge (spanning about +-1e31 in x, centred among the
    others): the nodes above them sit deep in the tree and have corners past 2^100, so their QNodes carry no
    grid and the uncertified 4-wide bounce walk steps through their exact records to their grandchildren."""
    base = rt.synthetic(T, seed=seed, half_extent=(30, 30, 20))
    v = base.vertices.copy()
    rng = np.random.default_rng(seed)
    idx = base.indices.reshape(-1, 3)
    for t in rng.choice(T, 400, replace=False):
        y, z = rng.uniform(-25, 25), rng.uniform(-15, 15)
        v[idx[t, 0], :3] = (-1e31 * rng.uniform(0.5, 2), y, z)
        v[idx[t, 1], :3] = (1e31 * rng.uniform(0.5, 2), y + rng.uniform(0.1, 2), z)
        v[idx[t, 2], :3] = (rng.uniform(-5, 5), y, z + rng.uniform(0.1, 2))
    return rt.Scene(v, base.indices, base.mat_indices, base.materials)


@pytest.mark.parametrize("mode", ["nearest+packet+wide", "binned+wide+refill"])
def test_deep_nodes_without_a_grid_after_another_build(mode):
    """k_refit writes only the QNodes a 4-wide walk reads; under a QNode without a grid the walk
    reads its node's binary grandchildren's QNodes (not the greedy entries), so those must be written too --
    else the walk reads what an earlier build of the same context left there.  The context first builds and
    traces another scene of the same size, then the scene with deep grid-less nodes: its frame (two bounces)
    is the oracle's."""
    s0 = rt.synthetic(8000, seed=17, half_extent=(30, 30, 20))
    s = _huge_scene()
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=TRACE_MODES[mode] | rt.FLAG_MULTI_KERNEL_BUILD) as c:
        c.set_scene(s0)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 2)
        c.set_scene(s)
        c.compute_bvh(W, H, 2)
        fb = c.read_framebuffer()
        nodes, q = c.read_bvh(), c.read_qnodes()
    T = s.num_tris
    par, cl = nodes["parent"], nodes["child_l"]
    depth = np.zeros(2 * T - 1, np.int32)
    for x in range(T + 1, 2 * T - 1):   # each internal node's depth below the root
        d, y = 0, x
        while y != T:
            y, d = par[y], d + 1
        depth[x] = d
    slots = {}
    for x in range(T + 1, 2 * T - 1):
        p = par[x] - T
        slots[x] = 2 * p + (0 if cl[par[x]] == x else 1)
    nogrid_deep = [x for x in slots if depth[x] >= 6 and q[slots[x], 3].view(np.float32) == 0]
    assert len(nogrid_deep) >= 20   # grid-less nodes well below the top
    ofb, _, _ = orc.trace(_oscene(s), nodes, wvp, wv, W, H, 2)
    np.testing.assert_array_equal(fb, ofb)


def test_packet_walk_after_a_build_without_pseudo_records():
    """A binned (or AUTO) context's build writes no leaf pseudo-records; a packet primary walk on
    that tree (flags changed since) writes them first (rtbvh enqueue_walks), and its frame is the
    oracle's -- then a rebuild under the packet flags writes them in the build."""
    s = rt.synthetic(20_000, seed=0x5EED0013, half_extent=(30, 30, 20))
    W, H = 320, 240
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=BINNED_FAST | rt.FLAG_MULTI_KERNEL_BUILD) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        nodes = c.read_bvh()
        ofb, _, _ = orc.trace(_oscene(s), nodes, wvp, wv, W, H, 1)
        np.testing.assert_array_equal(c.read_framebuffer(), ofb)
        for f in (TRACE_MODES["nearest+packet+wide"], TRACE_MODES["packet"], TRACE_MODES["nearest+packet"]):
            c.set_flags(f | rt.FLAG_MULTI_KERNEL_BUILD)
            c.trace(W, H, 1)
            np.testing.assert_array_equal(c.read_framebuffer(), ofb)
            c.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(c.read_framebuffer(), ofb)
            c.set_flags(BINNED_FAST | rt.FLAG_MULTI_KERNEL_BUILD)
            c.compute_bvh(W, H, 1)
            np.testing.assert_array_equal(c.read_framebuffer(), ofb)


def test_binned_primary_bins_overflow_falls_back_to_a_walk():
    """Leaves whose boxes cover most of the frame overflow the bins (3 entries per leaf + 16 per
    tile): the overflowed tiles are traced by the per-lane nearest-first walk behind the binned
    kernel, the others by the bins, and the frame is the oracle's, pixel for pixel."""
    rng = np.random.default_rng(11)
    n = 3000
    c0 = rng.uniform(-40, 40, (n, 1, 3)).astype(np.float32)
    tri = (c0 + rng.uniform(-60, 60, (n, 3, 3)).astype(np.float32)).reshape(-1, 3)
    verts = np.zeros((3 * n, 8), np.float32)
    verts[:, :3] = tri
    verts[:, 5] = 1.0
    d = load_scene_fixture("Test")
    s = rt.Scene(verts, np.arange(3 * n, dtype=np.uint32), np.zeros(n, np.uint32), d["material_blob"])
    W, H = 800, 600
    wvp, wv = rt.camera_reference(W, H)
    with rt.Context(device=0, flags=BINNED_FAST | rt.FLAG_COUNT_VISITS) as c:
        c.set_scene(s)
        c.set_camera(wvp, wv)
        c.compute_bvh(W, H, 1)
        fb = c.read_framebuffer()
        st = c.stats()
        nodes = c.read_bvh()
    ofb, _, ost = orc.trace(_oscene(s), nodes, wvp, wv, W, H, 1)
    np.testing.assert_array_equal(fb, ofb)
    assert st["internal_visits"][0] > 0   # a walk traced the overflowed tiles (the binned pass visits no node)
    assert ost["hits"] > 100_000


@pytest.mark.parametrize("nranks,share", [(2, 16), (3, 16), (8, 16), (3, 11), (8, 13)])
def test_assemble_bands_matches_full_frame(nranks, share):
    """rtbvh_assemble_bands (rank 0's step of rtbvh_trace_tiles): the ranks' band buffers,
    stacked as RCCL delivers them, give the full frame, under the even and the uneven deal;
    after a band trace the context reports that its framebuffer is not a frame."""
    import torch
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 640, 357
    with rt.Context(device=0, flags=rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.compute_bvh(W, H, 1)
        full = c.read_framebuffer()
        c.set_band_deal(share)
        rows0 = max(rt.lib().rtbvh_deal_rows(H, r, nranks, share) for r in range(nranks))
        bands = torch.full((nranks, rows0, W, 4), -1.0, dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()   # the fill runs on torch's stream, not the context's
        for r in range(nranks):
            c.trace_band_async(W, H, 1, r, nranks, bands[r].data_ptr())
        frame = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
        c.assemble_bands(W, H, nranks, bands.data_ptr(), rows0, frame.data_ptr())
        c.synchronize()
        np.testing.assert_array_equal(frame.cpu().numpy(), full)
        with pytest.raises(rt.RtbvhError) as e:
            c.read_framebuffer()
        assert e.value.status == 4


def test_trace_tiles_one_rank_matches_trace():
    """rtbvh_comm_* + rtbvh_trace_tiles through RCCL with one rank (a box has one GPU, and
    RCCL takes one rank per device): the frame on rank 0 equals rtbvh_trace's.  More ranks
    reuse the same calls; their assembly is test_assemble_bands_matches_full_frame."""
    d = load_scene_fixture("Test")
    s = rt.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    W, H = 640, 357
    with rt.Context(device=0, flags=rt.FLAG_PACKET_PRIMARY | rt.FLAG_WIDE_BVH) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.compute_bvh(W, H, 1)
        full = c.read_framebuffer()
        shown = c.present()
        comm = c.comm_init(1, 0, rt.comm_unique_id())
        try:
            c.trace_tiles(W, H, 1, 0, 1, comm)
            np.testing.assert_array_equal(c.read_framebuffer(), full)
            np.testing.assert_array_equal(c.present(), shown)
        finally:
            rt.comm_destroy(comm)


def _build_outputs(s, flags, morton_mode=0, delta_mode=0):
    with rt.Context(device=0, flags=flags, morton_mode=morton_mode, delta_mode=delta_mode) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(640, 360))
        c.build()
        out = {"nodes": c.read_bvh(), "morton": c.read_morton(), "sorted": c.read_sorted()}
        if s.num_tris > 1:
            out["wide"] = c.read_wide()
    return out


@pytest.mark.parametrize("ntris", [1, 2, 3, 57, 1000, 2047, 2048, 2049, 3072, 4096, 4097, 8192, 8193])
@pytest.mark.parametrize("modes", [(0, 0), (1, 0), (0, 1)])
def test_one_workgroup_build_equals_multi_kernel_build(ntris, modes):
    """Scenes of <= 2048 triangles build in one workgroup (build.hip k_build_small): the
    exported tree, Morton codes, sorted order and every node record equal the multi-kernel
    build's, for both Morton modes and both delta modes."""
    s = rt.synthetic(ntris, seed=ntris, half_extent=(30, 30, 20))
    a = _build_outputs(s, 0, *modes)
    b = _build_outputs(s, rt.FLAG_MULTI_KERNEL_BUILD, *modes)
    np.testing.assert_array_equal(a["nodes"], b["nodes"])
    np.testing.assert_array_equal(a["morton"], b["morton"])
    for x, y in zip(a["sorted"], b["sorted"]):
        np.testing.assert_array_equal(x, y)
    if "wide" in a:
        np.testing.assert_array_equal(a["wide"], b["wide"])


def test_errors_are_reported():
    with rt.Context(device=0) as c:
        with pytest.raises(rt.RtbvhError) as e:
            c.build()
        assert e.value.status == 4   # NOT_READY
        d = load_scene_fixture("Rect")
        bad = d["indices"].copy()
        bad[0] = 10_000
        with pytest.raises(rt.RtbvhError) as e:
            c.set_scene(rt.Scene(d["vertices"], bad, d["mat_indices"], d["material_blob"]))
        assert e.value.status == 1
