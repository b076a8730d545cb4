"""Pin the CPU oracle against the reference's own outputs (tests/golden/).

Every fixture here was produced by the reference's CPUTests programs compiled
unmodified from /root/reference (tests/golden/make_golden.py), or is a known
answer recorded in SURVEY.md §8(c).  CPU only.
"""
import json
import os

import numpy as np
import pytest

from oracle import lib as L
from tests.conftest import GOLDEN, load_scene_fixture

U32 = 0xFFFFFFFF


def fnv_u32_values(vals):
    h = 1469598103934665603
    for v in vals:
        h ^= int(v) & U32
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_morton_encoders_match_reference():
    z = np.load(os.path.join(GOLDEN, "morton_ref.npz"))
    pts = z["points"]
    # the KAT of Morton Code/main.cpp:103-104
    assert list(z["kat_stdout"]) == ["00101011110010000000000000000000"] * 2
    assert L.morton_point_cputests(.625, .4375, .75) == 0x2BC80000
    ours = np.array([L.morton_point_cputests(*p) for p in pts], dtype=np.uint32)
    np.testing.assert_array_equal(ours, z["calc"])
    np.testing.assert_array_equal(ours, z["karras"])   # both reference encoders agree
    ex = np.array([L.lib().orc_expand_bits(v) for v in range(1024)], dtype=np.uint32)
    np.testing.assert_array_equal(ex, z["expand"])


def test_blelloch_scan_matches_reference():
    z = np.load(os.path.join(GOLDEN, "scan_ref.npz"))
    flags = z["flags"].reshape(-1, 256)
    want = z["scanned"].reshape(-1, 256)
    for f, w in zip(flags, want):
        got = L.blelloch_scan256(f)
        np.testing.assert_array_equal(got, w)
        np.testing.assert_array_equal(got, np.concatenate([[0], np.cumsum(f)[:-1]]))


def test_split_sort_matches_reference_combo():
    z = np.load(os.path.join(GOLDEN, "combo.npz"))
    perm = L.split_sort(z["input_codes"])
    np.testing.assert_array_equal(z["input_codes"][perm], z["sorted_codes"])
    # stable: equal keys keep input order
    np.testing.assert_array_equal(perm, np.argsort(z["input_codes"], kind="stable"))
    np.testing.assert_array_equal(L.lsd_sort(z["input_codes"]), perm)


@pytest.mark.parametrize("n", [1, 2, 255, 256, 257, 1000, 4099])
def test_split_sort_ragged_sizes(n):
    rng = np.random.default_rng(n)
    keys = rng.integers(0, 1 << 12, size=n, dtype=np.uint32) << np.uint32(18)
    want = np.argsort(keys, kind="stable")
    np.testing.assert_array_equal(L.split_sort(keys), want)
    np.testing.assert_array_equal(L.lsd_sort(keys), want)


@pytest.mark.parametrize("mode", [L.DELTA_CPUTESTS, L.DELTA_CLZ64])
def test_karras_refit_matches_reference_combo(mode):
    """RadixBVHCombo: tree links for all 11,775 nodes + refit boxes + KATs.
    Both delta semantics give the reference's tree on this dataset."""
    z = np.load(os.path.join(GOLDEN, "combo.npz"))
    kats = json.load(open(os.path.join(GOLDEN, "combo_kats.json")))["stdout"]
    n = len(z["sorted_codes"])
    parent, cl, cr = L.karras(z["sorted_codes"], mode)
    ref_parent = z["parent"].astype(np.int64) & U32
    ref_cl = z["child_l"].astype(np.int64) & U32
    ref_cr = z["child_r"].astype(np.int64) & U32
    np.testing.assert_array_equal(parent, ref_parent)
    np.testing.assert_array_equal(cl, ref_cl)
    np.testing.assert_array_equal(cr, ref_cr)
    assert int(cr[6391]) == 6388 and kats[0] == "6388 6388"
    kat_fnv = json.load(open(os.path.join(GOLDEN, "shadersim_kats.json")))["combo_topology_fnv"]["value"]
    assert "%016x" % fnv_u32_values(np.stack([parent, cl, cr], 1).ravel()) == kat_fnv
    # refit from the reference's leaf boxes (un-permuted in that program)
    bmin = np.zeros((2 * n - 1, 3), np.float32)
    bmax = np.zeros((2 * n - 1, 3), np.float32)
    bmin[:n] = z["bb_min"][:n]
    bmax[:n] = z["bb_max"][:n]
    bmin, bmax, longest = L.refit(n, parent, cl, cr, bmin, bmax)
    np.testing.assert_array_equal(bmin, z["bb_min"])
    np.testing.assert_array_equal(bmax, z["bb_max"])
    assert longest == int(kats[1]) == 11
    root = f"{bmax[n][0]:g}, {bmax[n][1]:g}, {bmax[n][2]:g} | {bmin[n][0]:g}, {bmin[n][1]:g}, {bmin[n][2]:g}"
    assert kats[2].startswith(root)


def test_karras_matches_reference_random_sets():
    z = np.load(os.path.join(GOLDEN, "karras_ref.npz"))
    # set 0: distinct codes -> both delta semantics equal the reference
    for mode in (L.DELTA_CPUTESTS, L.DELTA_CLZ64):
        codes = z["sorted0"]
        n = len(codes)
        parent, cl, cr = L.karras(codes, mode)
        links = z["links0"].reshape(-1, 2)
        np.testing.assert_array_equal(cl[n:], links[:, 0])
        np.testing.assert_array_equal(cr[n:], links[:, 1])
    # set 1: duplicate codes -> the CPUTests delta reproduces the reference exactly ...
    codes = z["sorted1"]
    n = len(codes)
    parent, cl, cr = L.karras(codes, L.DELTA_CPUTESTS)
    links = z["links1"].reshape(-1, 2)
    np.testing.assert_array_equal(cl[n:], links[:, 0])
    np.testing.assert_array_equal(cr[n:], links[:, 1])
    # ... and the clz64 (HLSL) delta always gives a valid tree (one parent per node)
    parent, cl, cr = L.karras(codes, L.DELTA_CLZ64)
    counts = np.bincount(np.concatenate([cl[n:], cr[n:]]).astype(np.int64), minlength=2 * n - 1)
    assert counts[n] == 0 and (np.delete(counts, n) == 1).all()


def test_cputests_delta_breaks_on_heavy_duplicates():
    """with many duplicate codes the CPUTests delta (no +32 on the
    index tie-break) builds invalid trees (oracle-only: the reference program's
    size is fixed at 5,888); the default clz64 delta does not."""
    rng = np.random.default_rng(5)
    codes = np.sort(rng.integers(0, 1 << 16, size=100_000, dtype=np.uint32))
    n = len(codes)
    for mode, want_valid in ((L.DELTA_CPUTESTS, False), (L.DELTA_CLZ64, True)):
        parent, cl, cr = L.karras(codes, mode)
        counts = np.bincount(np.concatenate([cl[n:], cr[n:]]).astype(np.int64), minlength=2 * n - 1)
        valid = counts[n] == 0 and (np.delete(counts, n) == 1).all()
        assert valid == want_valid


def test_karras_paper_example_matches_bvhconstructtest():
    z = np.load(os.path.join(GOLDEN, "bvhct.npz"))
    codes = z["code"][:8]
    np.testing.assert_array_equal(codes, [1, 2, 4, 5, 19, 24, 25, 30])
    for mode in (L.DELTA_CPUTESTS, L.DELTA_CLZ64):
        parent, cl, cr = L.karras(codes, mode)
        np.testing.assert_array_equal(cl[8:], z["child_l"][8:])
        np.testing.assert_array_equal(cr[8:], z["child_r"][8:])
        # the reference never sets the root's parent in this test (prints 0)
        np.testing.assert_array_equal(parent[:8], z["parent"][:8])
        np.testing.assert_array_equal(parent[9:], z["parent"][9:])


def test_radixsort_test_has_no_err():
    assert json.load(open(os.path.join(GOLDEN, "radixsort_kat.json")))["err_lines"] == 0


@pytest.mark.parametrize("name", ["Rect", "Image_Test", "Test"])
def test_shadersim_kats(name):
    """OBJ loader + CPUTests Morton (ShaderSim) vs the recorded KATs."""
    k = json.load(open(os.path.join(GOLDEN, "shadersim_kats.json")))[name]
    d = load_scene_fixture(name)
    s = L.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    assert len(d["vertices"]) == k["verts"] and s.num_tris == k["tris"]
    codes = L.morton_tris(s, L.MORTON_CPUTESTS)
    assert int(codes[0]) == k["code0"] and int(codes[1]) == k["code1"]
    assert "%016x" % fnv_u32_values(codes) == k["fnv"]
    mask = np.uint32(sum(1 << i for i in range(18, 30)))
    assert int((((np.sort(codes & mask)) >> 18) & 1).sum()) == k["bit18_count"]


@pytest.mark.skipif(not os.path.isdir("/root/reference/Obj"), reason="reference not mounted")
@pytest.mark.parametrize("name", ["Rect", "Image_Test", "Test"])
def test_scene_fixtures_are_current(name):
    from oracle import obj_oracle
    d = obj_oracle.load_obj(f"/root/reference/Obj/{name}.obj")
    f = load_scene_fixture(name)
    for key in ("vertices", "indices", "mat_indices", "material_blob"):
        np.testing.assert_array_equal(d[key], f[key])


def test_hlsl_leading_zero_is_clz():
    """BVHConstructP1.hlsl:39-53's De Bruijn leadingZero equals clz for every
    bit length, so the HLSL delta is clz64 of index-augmented keys."""
    for b in range(33):
        for v in ([0] if b == 0 else [1 << (b - 1), (1 << b) - 1]):
            codes = np.array([0, v], dtype=np.uint32) if v else np.array([7, 7], dtype=np.uint32)
            d = L.lib().orc_delta(L.DELTA_CLZ64, codes.ctypes.data, 2, 0, 1)
            want = 32 - v.bit_length() if v else 32 + 31   # equal codes: 32 + clz(0 ^ 1)
            assert d == want, (b, v, d)
