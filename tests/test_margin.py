"""The certified walks' rounding margin (raytracebvh_amd/csrc/margin.h) bounds how far the
point of an accepted Moller-Trumbore hit (RayTraceTraversal.hlsl:41-86) can lie outside the triangle's
box: a randomized check on the CPU (tools/margin_check.cpp restates the device arithmetic -- the
triangle test, build.hip quantize_axis, the certified slack test of trace.hip -- and includes margin.h
itself) over C5-like triangles, grazing rays whose determinant sits just above the 0.01 rejection,
flat and coplanar triangles, near-edge hits, the orthographic primary rays and several scales.  No
accepted hit may lie farther than the margin, no certified box test may prune a box holding it, and no
primary depth key may exceed its t; the per-node margins (a node's largest leaf edge bound and its margin
range, coded in its QNode) bound every such hit of the leaves below the node.  With a margin 1000x too small the check must fail: it bites."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "margin_check.cpp")
INC = os.path.join(REPO, "raytracebvh_amd", "csrc")


def _build(tmp_path, name, extra=()):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-O2", "-ffp-contract=off", f"-I{INC}", *extra, "-o", exe, SRC], check=True)
    return exe


def _run(exe, n, seed):
    p = subprocess.run([exe, str(n), str(seed)], capture_output=True, text=True, timeout=300)
    return p.returncode, json.loads(p.stdout)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_margin_contains_every_accepted_hit(tmp_path, seed):
    rc, r = _run(_build(tmp_path, "margin_check"), 400_000, seed)
    assert r["accepted"] > 1_000_000 and r["dist_checked"] > 800_000
    assert r["walk_checked"] > 500_000 and r["zkey_checked"] > 100_000
    assert r["dist_violations"] == 0 and r["dist_violations_tight"] == 0, r
    assert r["walk_violations"] == 0 and r["zkey_violations"] == 0, r
    # the per-node margins of the certified bounce walk (margin.h mt_node_codes / mt_node_rho, round 5)
    assert r["node_checked"] > 1_000_000 and r["node_walk_checked"] > 500_000
    assert r["node_violations"] == 0 and r["node_walk_violations"] == 0, r
    assert 0 < r["max_ratio"] < 1 and 0 < r["max_ratio_tight"] < 1
    assert rc == 0


def test_margin_check_detects_a_small_margin(tmp_path):
    rc, r = _run(_build(tmp_path, "margin_check_small", ["-DMARGIN_SCALE=1e-3f"]), 200_000, 1)
    assert rc == 1 and r["dist_violations"] > 0 and r["max_ratio"] > 1, r
    assert r["node_violations"] > 0, r
