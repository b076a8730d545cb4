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
