"""The bounce walk's slack QNode test (trace.hip qaxis / qbox_fast) contains the
reference slab test on the exact child boxes (RayTraceTraversal.hlsl:92-104): a randomized check
on the CPU (tools/slack_check.cpp restates the device arithmetic: quantize_axis of build.hip, the
exact ray_box, the slack test), over boxes of several magnitude regimes, flat boxes, ray origins
on box planes and near-axis directions.  No exact hit may be missed or entered later.  A slack
test without the slack (E = 0) must fail the same check: the check bites."""
import json
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "tools", "slack_check.cpp")


def _build(tmp_path, name, extra=()):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-O2", "-ffp-contract=off", *extra, "-o", exe, SRC], check=True)
    return exe


def _run(exe, n, seed):
    p = subprocess.run([exe, str(n), str(seed)], capture_output=True, text=True, timeout=300)
    return p.returncode, json.loads(p.stdout)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_slack_test_contains_exact_test(tmp_path, seed):
    rc, r = _run(_build(tmp_path, "slack_check"), 400_000, seed)
    assert r["exact_hits"] > 500_000
    assert r["missed"] == 0 and r["later_entry"] == 0, r
    assert rc == 0


def test_slack_check_detects_a_missing_slack(tmp_path):
    rc, r = _run(_build(tmp_path, "slack_check_noslack", ["-DSLACK=0.0f"]), 200_000, 1)
    assert rc == 1 and r["missed"] > 0, r
