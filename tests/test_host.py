"""CPU-only checks of librtbvh.so: it loads, exports every symbol include/rtbvh.h
declares, and its host-side pieces (OBJ loader, synthetic generator, camera,
band split) agree with independent restatements.  No compute call needs a GPU."""
import ctypes
import os
import re

import numpy as np
import pytest

import raytracebvh_amd as rt
from raytracebvh_amd import _lib
from oracle import lib as orc
from tests.conftest import REPO, load_scene_fixture


def test_library_exports_every_header_symbol():
    header = open(os.path.join(REPO, "include", "rtbvh.h")).read()
    declared = set(re.findall(r"\b(rtbvh_[a-z_0-9]+)\s*\(", header))
    declared -= {"rtbvh_status"}
    assert declared == set(_lib.EXPORTS), declared ^ set(_lib.EXPORTS)
    L = rt.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert L.rtbvh_abi_version() == 8


def test_layout_sizes():
    assert rt.NODE_DTYPE.itemsize == 44 and rt.MATERIAL_DTYPE.itemsize == 68


def test_stats_mirror_matches_the_library():
    # the ctypes mirror of rtbvh_stats against the struct the library was built with (a field added on one
    # side only would shift every field after it)
    assert ctypes.sizeof(_lib.Stats) == rt.lib().rtbvh_stats_size()


@pytest.mark.skipif(not os.path.isdir("/root/reference/Obj"), reason="reference not mounted")
@pytest.mark.parametrize("name", ["Rect", "Image_Test", "Test"])
def test_native_obj_loader_matches_oracle_loader(name):
    s = rt.load_obj(f"/root/reference/Obj/{name}.obj")
    f = load_scene_fixture(name)
    np.testing.assert_array_equal(s.vertices, f["vertices"])
    np.testing.assert_array_equal(s.indices, f["indices"])
    np.testing.assert_array_equal(s.mat_indices, f["mat_indices"])
    np.testing.assert_array_equal(s.material_blob, f["material_blob"])
    assert [os.path.basename(p) for p in s.texture_paths] == [str(x) for x in f["texture_names"]]


def test_obj_loader_quirks(tmp_path):
    """Dedup by position, normal z ignored (Helper.h:11-14), d sets alpha, Tr ignored."""
    (tmp_path / "q.mtl").write_text("newmtl A\nKd 0.5 0.25 0.125\nd 0.5\nTr 0.9\nNs 42\nmap_Kd t.bmp\nnewmtl B\n")
    (tmp_path / "q.obj").write_text(
        "mtllib q.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nvn 0 0 -1\nvt 0 0\n"
        "usemtl B\nf 1/1/1 2/1/1 3/1/1\nusemtl A\nf 1/1/2 2/1/2 3/1/1\n")
    s = rt.load_obj(str(tmp_path / "q.obj"), load_textures=False)
    assert len(s.vertices) == 3                      # normals differing only in z merged
    np.testing.assert_array_equal(s.indices, [0, 1, 2, 0, 1, 2])
    np.testing.assert_array_equal(s.mat_indices, [1, 0])
    a, b = s.materials
    assert a["alpha"] == np.float32(0.5) and a["shininess"] == 42 and a["tex_num"] == 0
    np.testing.assert_array_equal(a["diffuse"], np.float32([0.5, 0.25, 0.125, 1]))
    np.testing.assert_array_equal(b["ambient"], np.float32([0.2, 0.2, 0.2, 1]))   # Base_Mat
    assert b["tex_num"] == -1


def test_obj_loader_missing_file_is_io_error():
    with pytest.raises(rt.RtbvhError) as e:
        rt.load_obj("/nonexistent/x.obj")
    assert e.value.status == _lib.ERR_IO


def _synthetic_numpy(seed, ntris, half):
    """Independent numpy restatement of the SURVEY §8(d) generator."""
    M = (1 << 64) - 1
    k = np.arange(1, ntris * 12 + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + k * np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    u = u.reshape(ntris, 12)
    half = np.asarray(half, np.float32)
    c = (u[:, :3] * np.float32(2.0) - np.float32(1.0)) * half
    v = c[:, None, :] + (u[:, 3:].reshape(ntris, 3, 3) - np.float32(0.5)) * np.float32(1.0)
    return v.astype(np.float32)


def test_synthetic_generator_matches_numpy_restatement():
    s = rt.synthetic(1000, seed=0x5EED0005, half_extent=(100, 100, 50))
    v = _synthetic_numpy(0x5EED0005, 1000, (100, 100, 50))
    np.testing.assert_array_equal(s.vertices[:, :3].reshape(1000, 3, 3), v)
    np.testing.assert_array_equal(s.indices, np.arange(3000))
    n = s.vertices[:, 3:6]
    assert np.allclose(np.linalg.norm(n, axis=1), 1, atol=1e-6)
    assert s.materials[0]["shininess"] == 300 and s.materials[0]["tex_num"] == -1


def test_camera_matches_oracle():
    from oracle import lib as orc
    for W, H in ((1920, 1080), (3840, 2160), (800, 800)):
        a = rt.camera_reference(W, H)
        b = orc.camera_reference(W, H)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    wvp, _ = rt.camera_reference(1920, 1080)
    # SURVEY §8(d) quotes these WVP rows at 1920x1080
    np.testing.assert_allclose(wvp[0], [4.291935, 0, 0, 0], atol=1e-5)
    np.testing.assert_allclose(wvp[3], [0, 0, 100.03492, 100.12492], atol=1e-3)


def test_camera_orbit_is_graphics_on_key_down():
    """rtbvh_camera_orbit restates Graphics::onKeyDown (Graphics.cpp:937-960): eye = at + (eye - at) R with
    DirectXMath's RotationY(-+0.1) / RotationX(+-0.1) (row vectors, CAM_DELTA .1f, Graphics.h:14); left and
    right (up and down) undo each other; the distance to the origin is kept; camera_look at the reference
    eye is the reference camera (Graphics.cpp:44-53)."""
    eye = np.array(rt.EYE_REFERENCE, np.float32)
    for W, H in ((1920, 1080), (3840, 2160)):
        a, b = rt.camera_look(eye, W, H), rt.camera_reference(W, H)
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    c, s = np.cos(0.1), np.sin(0.1)
    ry = lambda a: np.array([[np.cos(a), 0, -np.sin(a)], [0, 1, 0], [np.sin(a), 0, np.cos(a)]])
    rx = lambda a: np.array([[1, 0, 0], [0, np.cos(a), np.sin(a)], [0, -np.sin(a), np.cos(a)]])
    want = {rt.KEY_LEFT: eye @ ry(-0.1), rt.KEY_RIGHT: eye @ ry(0.1), rt.KEY_UP: eye @ rx(0.1), rt.KEY_DOWN: eye @ rx(-0.1)}
    for key, w in want.items():
        np.testing.assert_allclose(rt.camera_orbit(eye, key), w, rtol=1e-6, atol=1e-5)
    np.testing.assert_allclose(rt.camera_orbit(rt.camera_orbit(eye, rt.KEY_LEFT), rt.KEY_RIGHT), eye, atol=1e-4)
    np.testing.assert_allclose(rt.camera_orbit(rt.camera_orbit(eye, rt.KEY_UP), rt.KEY_DOWN), eye, atol=1e-4)
    e = eye
    for _ in range(63):   # ~2 pi of left presses
        e = rt.camera_orbit(e, rt.KEY_LEFT)
    assert abs(np.linalg.norm(e) - np.linalg.norm(eye)) < 1e-3
    np.testing.assert_array_equal(rt.camera_orbit(eye, 7), eye)   # other keys: unchanged
    assert c > 0 and s > 0


@pytest.mark.parametrize("H,n", [(1080, 1), (1080, 2), (1080, 8), (2160, 8), (7, 3), (17, 4)])
def test_band_rows_partition_the_frame(H, n):
    L = rt.lib()
    rows = [L.rtbvh_band_rows(H, r, n) for r in range(n)]
    assert sum(rows) == H
    want = [sum(min(8, H - 8 * b) for b in range(r, (H + 7) // 8, n)) for r in range(n)]
    assert rows == want


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rt.RtbvhError) as e:
        rt.Context()
    assert e.value.status == _lib.ERR_NO_DEVICE


# ---------------------------------------------------------------- textures
def _bmp_cases(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, (13, 21, 3), dtype=np.uint8)          # odd width: row padding
    cases = {"rgb24.bmp": Image.fromarray(rgb, "RGB")}
    pal = Image.fromarray(rng.integers(0, 256, (9, 17), dtype=np.uint8), "L").convert("P")
    cases["pal8.bmp"] = pal
    cases["bw1.bmp"] = Image.fromarray((rng.integers(0, 2, (7, 11)) * 255).astype(np.uint8), "L").convert("1")
    out = []
    for name, im in cases.items():
        p = tmp_path / name
        im.save(p)
        out.append((str(p), np.asarray(im.convert("RGBA"))))
    return out


def test_bmp_decoder_matches_pil(tmp_path):
    """rtbvh_texture_load_bmp returns the file's rows in storage order (bottom-up), as
    DevIL does without IL_ORIGIN_SET (Image.cpp:48-49): PIL's top-down image flipped."""
    from raytracebvh_amd.scene import load_texture
    for path, want in _bmp_cases(tmp_path):
        got = load_texture(path)
        np.testing.assert_array_equal(got, want[::-1], err_msg=path)


def test_bmp_decoder_on_reference_textures():
    """The reference's own texture files (Obj/*.bmp): 8-bit paletted and 24-bit."""
    from raytracebvh_amd.scene import load_texture
    from PIL import Image
    obj = os.path.join("/root/reference", "Obj")
    if not os.path.isdir(obj):
        pytest.skip("reference tree not present")
    for name in ("Balls.bmp", "Map__1_Composite.bmp"):
        got = load_texture(os.path.join(obj, name))
        want = np.asarray(Image.open(os.path.join(obj, name)).convert("RGBA"))
        np.testing.assert_array_equal(got, want[::-1], err_msg=name)


def test_srgb_table_and_sampler_properties():
    from raytracebvh_amd.scene import srgb_table
    tab = srgb_table()
    c = np.arange(256) / 255.0
    ref = np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4).astype(np.float32)
    np.testing.assert_array_equal(tab, ref)
    assert tab[0] == 0 and tab[255] == 1 and (np.diff(tab) > 0).all()
    rng = np.random.default_rng(9)
    tex = rng.integers(0, 256, (5, 7, 4), dtype=np.uint8)
    H, W = tex.shape[:2]
    lin = np.concatenate([tab[tex[..., :3]], (tex[..., 3:4].astype(np.float32) / np.float32(255))], -1)
    for y in range(H):          # texel centres return the decoded texel exactly
        for x in range(W):
            u, v = np.float32((x + 0.5) / W), np.float32((y + 0.5) / H)
            np.testing.assert_array_equal(orc.sample_texture(tex, u, v), lin[y, x])
    for u, v in [(0.125, 0.75), (0.5, 0.5), (0.9375, 0.0625)]:   # wrap: period 1 (dyadic: exact in f32)
        np.testing.assert_array_equal(orc.sample_texture(tex, u, v), orc.sample_texture(tex, u + 2.0, v - 3.0))
    # halfway between two texel centres along x: the mean of the two (lerp at 0.5)
    u, v = np.float32(1.0 / W), np.float32(0.5 / H)
    np.testing.assert_allclose(orc.sample_texture(tex, u, v), (lin[0, 0] + lin[0, 1]) / 2, rtol=1e-6)


def test_save_bmp_roundtrip(tmp_path):
    """rtbvh_save_bmp (SaveBMP.cpp:3-62 layout): PIL reads back the image, padded and unpadded widths."""
    from PIL import Image
    rng = np.random.default_rng(11)
    for W, H in ((5, 3), (8, 4)):
        img = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
        p = str(tmp_path / f"o{W}.bmp")
        rt.save_bmp(p, img)
        back = np.asarray(Image.open(p).convert("RGB"))
        np.testing.assert_array_equal(back, img[..., :3])
        hdr = open(p, "rb").read(54)
        assert hdr[:2] == b"BM" and int.from_bytes(hdr[10:14], "little") == 0x36
        assert int.from_bytes(hdr[38:42], "little") == 0x0EC4 and hdr[28] == 24


# ---------------------------------------------------------------- textures (Image::loadImage)
def _pil_rgba(data: bytes) -> np.ndarray:
    import io

    from PIL import Image
    with Image.open(io.BytesIO(data)) as im:
        return np.asarray(im.convert("RGBA"), dtype=np.uint8)


def test_jpeg_decoder_matches_libjpeg_on_the_reference_texture(golden_dir):
    """Test.mtl:12 binds Balls.jpg (4:2:0 baseline, 1600x1000; the reference decodes it with
    DevIL/libjpeg, Image.cpp:35-61): the native decoder equals PIL's libjpeg-turbo bit for bit."""
    from raytracebvh_amd.scene import load_texture
    path = os.path.join(golden_dir, "textures", "Balls.jpg")
    got = load_texture(path)
    want = _pil_rgba(open(path, "rb").read())
    assert got.shape == (1000, 1600, 4)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("subsampling", [0, 1, 2])   # 4:4:4, 4:2:2, 4:2:0
@pytest.mark.parametrize("size", [(1, 1), (8, 17), (37, 23), (129, 77)])
@pytest.mark.parametrize("restart", [0, 3])
def test_jpeg_decoder_matches_libjpeg_synthetic(subsampling, size, restart):
    import io

    from PIL import Image

    from raytracebvh_amd.scene import decode_jpeg
    w, h = size
    rng = np.random.default_rng(w * 131 + h + subsampling)
    img = (rng.integers(0, 256, (h, w, 3)) // 3 + np.linspace(0, 150, w)[None, :, None]).astype(np.uint8)
    bio = io.BytesIO()
    kw = {"restart_marker_blocks": restart} if restart else {}
    Image.fromarray(img).save(bio, "JPEG", quality=90, subsampling=subsampling, **kw)
    data = bio.getvalue()
    np.testing.assert_array_equal(decode_jpeg(data), _pil_rgba(data))


def test_jpeg_decoder_grayscale_and_rejections():
    import io

    from PIL import Image

    from raytracebvh_amd.scene import decode_jpeg
    rng = np.random.default_rng(5)
    g = rng.integers(0, 256, (33, 45), dtype=np.uint8)
    bio = io.BytesIO()
    Image.fromarray(g).save(bio, "JPEG")
    np.testing.assert_array_equal(decode_jpeg(bio.getvalue()), _pil_rgba(bio.getvalue()))
    prog = io.BytesIO()
    Image.fromarray(np.stack([g] * 3, 2)).save(prog, "JPEG", progressive=True)
    for bad in (prog.getvalue(), b"\xff\xd8\xff\xd9", b"not a jpeg", bio.getvalue()[:40]):
        with pytest.raises(rt.RtbvhError) as e:
            decode_jpeg(bad)
        assert e.value.status == _lib.ERR_IO
    # truncated and bit-flipped files end in an error or a decoded image, never a crash
    data = bytearray(bio.getvalue())
    for cut in range(0, len(data), 17):
        try:
            decode_jpeg(bytes(data[:cut]))
        except rt.RtbvhError as e:
            assert e.status == _lib.ERR_IO
    for k in range(200):
        d = bytearray(data)
        d[int(rng.integers(2, len(d)))] ^= 1 << int(rng.integers(0, 8))
        try:
            decode_jpeg(bytes(d))
        except rt.RtbvhError as e:
            assert e.status == _lib.ERR_IO


def test_texture_load_by_magic(golden_dir, tmp_path):
    """rtbvh_texture_load: BMP (Map__1_Composite.bmp, bottom row first as DevIL keeps it) or JPEG
    by content; anything else is an I/O error (a truncated PNG also fails the PIL fallback)."""
    from raytracebvh_amd.scene import load_texture
    bmp = os.path.join(golden_dir, "textures", "Map__1_Composite.bmp")
    got = load_texture(bmp)
    np.testing.assert_array_equal(got, _pil_rgba(open(bmp, "rb").read())[::-1])
    (tmp_path / "x.png").write_bytes(b"\x89PNG\r\n\x1a\n" + b"\0" * 64)
    with pytest.raises(rt.RtbvhError) as e:
        load_texture(str(tmp_path / "x.png"))
    assert e.value.status == _lib.ERR_IO


def test_texture_load_falls_back_to_pil(tmp_path):
    """Textures the native decoders do not read (PNG, TGA, progressive JPEG) -- which DevIL
    decodes for Image::loadImage (Image.cpp:35-61) -- load through PIL in DevIL's file-order
    convention: PNG and JPEG top row first, a bottom-up TGA bottom row first."""
    from PIL import Image

    from raytracebvh_amd.scene import load_texture
    rng = np.random.default_rng(7)
    a = rng.integers(0, 256, (13, 17, 4), dtype=np.uint8)
    Image.fromarray(a, "RGBA").save(tmp_path / "t.png")
    np.testing.assert_array_equal(load_texture(str(tmp_path / "t.png")), a)
    Image.fromarray(a, "RGBA").save(tmp_path / "t.tga")
    assert not (open(tmp_path / "t.tga", "rb").read(18)[17] & 0x20)   # stored bottom-up
    np.testing.assert_array_equal(load_texture(str(tmp_path / "t.tga")), a[::-1])
    Image.fromarray(a[:, :, :3], "RGB").save(tmp_path / "p.jpg", progressive=True, quality=90)
    with Image.open(tmp_path / "p.jpg") as im:
        want = np.asarray(im.convert("RGBA"))
    np.testing.assert_array_equal(load_texture(str(tmp_path / "p.jpg")), want)
    (tmp_path / "junk.bin").write_bytes(b"not an image")
    with pytest.raises(rt.RtbvhError) as e:
        load_texture(str(tmp_path / "junk.bin"))
    assert e.value.status == _lib.ERR_IO
