"""tools/rtbvh_bench: the C++ host over include/rtbvh.h alone (SURVEY §8(b) callers)."""
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(REPO, "tools", "rtbvh_bench")


def _build_tool():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tools")], check=True)
    assert os.access(TOOL, os.X_OK)


def test_header_is_c99(tmp_path):
    """The boundary header compiles as plain C (a cgo / FFI binding sees exactly this)."""
    src = tmp_path / "t.c"
    src.write_text('#include "rtbvh.h"\nint main(void) { rtbvh_config c; rtbvh_config_default(&c); return 0; }\n')
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-fsyntax-only",
                    "-I", os.path.join(REPO, "include"), str(src)], check=True)


def test_tool_builds_and_rejects_bad_arguments():
    _build_tool()
    r = subprocess.run([TOOL, "--synthetic", "10", "--obj", "x.obj"], capture_output=True, text=True)
    assert r.returncode == 1 and "exactly one of" in r.stderr


@pytest.mark.gpu
def test_tool_frame_matches_python_path(tmp_path):
    """Same synthetic scene, camera and trace through the C++ host and through the Python
    Context: the saved BMPs are byte-identical."""
    import raytracebvh_amd as rt

    _build_tool()
    W, H, n = 320, 240, 20_000
    out = tmp_path / "cpp.bmp"
    r = subprocess.run([TOOL, "--synthetic", str(n), "--seed", "7", "--half", "30,30,20", "--width", str(W),
                        "--height", str(H), "--bounces", "2", "--iters", "2", "--warmup", "1", "--bmp", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["tris"] == n and rec["rays_this_rank"] >= W * H and rec["trace_ms_median"] > 0
    s = rt.synthetic(n, seed=7, half_extent=(30, 30, 20))
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.compute_bvh(W, H, 2)
        img = c.present()
    ref = tmp_path / "py.bmp"
    rt.save_bmp(str(ref), img)
    assert out.read_bytes() == ref.read_bytes()
    assert np.count_nonzero(img[..., :3] != 128) > 0   # not an empty (background-only) frame


@pytest.mark.gpu
def test_tool_renders_jpeg_textured_obj(tmp_path):
    """The C++ host renders an OBJ whose material binds a JPEG (map_Kd, as Test.mtl:12 binds
    Balls.jpg): the texture is decoded natively (rtbvh_texture_load) and the frame equals the
    Python path's byte for byte."""
    import shutil

    import raytracebvh_amd as rt

    _build_tool()
    shutil.copy(os.path.join(REPO, "tests", "golden", "textures", "Balls.jpg"), tmp_path / "Balls.jpg")
    (tmp_path / "q.mtl").write_text("newmtl Tex\nNs 300\nKa 0 0 0\nKd 1 1 1\nKs 1 1 1\nd 1\nmap_Kd Balls.jpg\n")
    (tmp_path / "q.obj").write_text(
        "mtllib q.mtl\nv -60 -40 10\nv 60 -40 10\nv 60 40 12\nv -60 40 12\n"
        "vt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\nvn 0 0 -1\n"
        "usemtl Tex\nf 1/1/1 2/2/1 3/3/1\nf 1/1/1 3/3/1 4/4/1\n")
    W, H = 320, 240
    out = tmp_path / "cpp.bmp"
    r = subprocess.run([TOOL, "--obj", str(tmp_path / "q.obj"), "--width", str(W), "--height", str(H),
                        "--bounces", "1", "--iters", "1", "--warmup", "0", "--bmp", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "not decoded" not in r.stderr
    s = rt.load_obj(str(tmp_path / "q.obj"))
    assert s.textures and s.textures[0].shape == (1000, 1600, 4)
    with rt.Context(device=0) as c:
        c.set_scene(s)
        c.set_camera(*rt.camera_reference(W, H))
        c.compute_bvh(W, H, 1)
        img = c.present()
    ref = tmp_path / "py.bmp"
    rt.save_bmp(str(ref), img)
    assert out.read_bytes() == ref.read_bytes()
    assert len(np.unique(img[..., :3].reshape(-1, 3), axis=0)) > 50   # textured, not flat


def test_host_code_under_asan_and_ubsan(tmp_path):
    """the host-side parsers of untrusted input (OBJ/MTL loader, BMP and JPEG
    decoders) and the CPU oracle, built with -fsanitize=address,undefined
    (-fno-sanitize-recover: any report aborts; LeakSanitizer checks the exit), run on the
    reference's files and on ~100 truncated / corrupted copies of each (tools/sanitize_host.cpp)."""
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tools"), "sanitize"], check=True)
    (tmp_path / "q.mtl").write_text("newmtl A\nKd 0.5 0.25 0.125\nd 0.5\nNs 42\nmap_Kd t.bmp\nnewmtl B\n")
    (tmp_path / "q.obj").write_text(
        "mtllib q.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nv 0 0 1\nvn 0 0 1\nvn 0 0 -1\nvt 0 0\nvt 1 1\n"
        "usemtl B\nf 1/1/1 2/1/1 3/2/1\nusemtl A\nf 1/1/2 2/2/2 4/1/1\nf 2/1/1 3/2/2 4/2/1\n")
    files = [str(tmp_path / "q.obj"), os.path.join(REPO, "tests", "golden", "textures", "Balls.jpg"),
             os.path.join(REPO, "tests", "golden", "textures", "Map__1_Composite.bmp")]
    files += [f"/root/reference/Obj/{n}.obj" for n in ("Rect", "Test") if os.path.exists(f"/root/reference/Obj/{n}.obj")]
    env = dict(os.environ, TMPDIR=str(tmp_path), ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(REPO, "tools", "sanitize_host"), "--mutations", "60"] + files,
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["runs"] == len(files) * 61 and rec["parsed"] >= len(files)
