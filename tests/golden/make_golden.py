#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container,
where the read-only reference is mounted at /root/reference).

What it does (nothing of the reference's SOURCE is copied into the repo):
  1. `make -C oracle ref` compiles the reference's own CPUTests programs
     unmodified (RadixBVHCombo, "Morton Code", BVHConstructTest, RadixSortTest)
     with thin drivers from oracle/ref_harness/ into oracle/_ref/;
  2. runs them and stores their OUTPUTS as .npz / .json fixtures:
       combo.npz        RadixBVHCombo: input codes, sorted codes, all 11,775 nodes
       combo_kats.json  its stdout KATs (main.cpp:531,576,587-600)
       karras_ref.npz   reference getChildren on two other code sets
       scan_ref.npz     reference prefixSum (Blelloch) on random flags
       morton_ref.npz   reference calcMorton / morton3D / expand on 20k points
       bvhct.npz        BVHConstructTest's 8-key Karras tree
  3. parses the reference's Obj/ meshes with the oracle OBJ loader
     (oracle/obj_oracle.py) into input fixtures scenes/<name>.npz;
  4. writes shadersim_kats.json: the ShaderSim known answers recorded in
     SURVEY.md §8(c) (that program needs DirectXMath and is unbuildable here).
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import obj_oracle  # noqa: E402

COMBO_NODE = np.dtype([("parent", "<i4"), ("childL", "<i4"), ("childR", "<i4"), ("code", "<u4"),
                       ("bbMin", "<f4", (3,)), ("bbMax", "<f4", (3,))])


def run(cmd, **kw):
    return subprocess.run(cmd, check=True, capture_output=True, text=True, **kw)


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not mounted; fixtures are committed, nothing to do")
    run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "ref"])
    refdir = os.path.join(REPO, "oracle", "_ref")
    with tempfile.TemporaryDirectory() as tmp:
        out = run([os.path.join(refdir, "combo_dump"), tmp]).stdout
        lines = [ln.strip() for ln in out.strip().splitlines() if ln.strip()]
        nodes = np.fromfile(os.path.join(tmp, "combo_nodes.bin"), dtype=COMBO_NODE)
        np.savez_compressed(
            os.path.join(HERE, "combo.npz"),
            input_codes=np.fromfile(os.path.join(tmp, "combo_input_codes.u32"), dtype="<u4"),
            sorted_codes=np.fromfile(os.path.join(tmp, "combo_sorted_codes.u32"), dtype="<u4"),
            parent=nodes["parent"], child_l=nodes["childL"], child_r=nodes["childR"],
            code=nodes["code"], bb_min=nodes["bbMin"], bb_max=nodes["bbMax"])
        with open(os.path.join(HERE, "combo_kats.json"), "w") as f:
            json.dump({"source": "CPUTests/RadixBVHCombo/RadixBVHCombo/main.cpp:531,576,587-600",
                       "stdout": lines[:3]}, f, indent=1)
        ks = {}
        for s in (0, 1):
            ks[f"sorted{s}"] = np.fromfile(os.path.join(tmp, f"combo_random{s}_sorted.u32"), dtype="<u4")
            ks[f"links{s}"] = np.fromfile(os.path.join(tmp, f"combo_random{s}_links.i32"), dtype="<i4")
        np.savez_compressed(os.path.join(HERE, "karras_ref.npz"), **ks)
        np.savez_compressed(os.path.join(HERE, "scan_ref.npz"),
                            flags=np.fromfile(os.path.join(tmp, "combo_scan_in.u32"), dtype="<u4"),
                            scanned=np.fromfile(os.path.join(tmp, "combo_scan_out.u32"), dtype="<u4"))

        out = run([os.path.join(refdir, "morton_dump"), tmp]).stdout
        np.savez_compressed(
            os.path.join(HERE, "morton_ref.npz"),
            points=np.fromfile(os.path.join(tmp, "morton_points.f32"), dtype="<f4").reshape(-1, 3),
            calc=np.fromfile(os.path.join(tmp, "morton_calc.u32"), dtype="<u4"),
            karras=np.fromfile(os.path.join(tmp, "morton_karras.u32"), dtype="<u4"),
            expand=np.fromfile(os.path.join(tmp, "morton_expand.u32"), dtype="<u4"),
            kat_stdout=np.array(out.split()[:2]))

        run([os.path.join(refdir, "bvhct_dump"), tmp])
        bv = np.fromfile(os.path.join(tmp, "bvhct_nodes.i32"), dtype="<i4").reshape(15, 4)
        np.savez_compressed(os.path.join(HERE, "bvhct.npz"), parent=bv[:, 0], child_l=bv[:, 1],
                            child_r=bv[:, 2], code=bv[:, 3].astype(np.uint32))

        rs = subprocess.run([os.path.join(refdir, "radixsort_test")], capture_output=True, text=True)
        with open(os.path.join(HERE, "radixsort_kat.json"), "w") as f:
            json.dump({"source": "CPUTests/RadixSortTest/RadixSort/main.cpp:249-256",
                       "err_lines": rs.stdout.count("ERR")}, f, indent=1)

    os.makedirs(os.path.join(HERE, "scenes"), exist_ok=True)
    for name in ("Rect", "Image_Test", "Test"):
        d = obj_oracle.load_obj(os.path.join(REF, "Obj", name + ".obj"))
        np.savez_compressed(os.path.join(HERE, "scenes", name + ".npz"), vertices=d["vertices"],
                            indices=d["indices"], mat_indices=d["mat_indices"],
                            material_blob=d["material_blob"],
                            texture_names=np.array([os.path.basename(p) for p in d["texture_paths"]]))

    kats = {
        "source": "SURVEY.md §8(c) ShaderSim KATs (CPUTests/ShaderSim/ShaderSim/main.cpp:251-320); "
                  "fnv = FNV-1a64 folding each u32 code value (h ^= code; h *= 1099511628211) "
                  "over the per-triangle codes in file order, before masking",
        "Test": {"verts": 2445, "tris": 1952, "code0": 839237106, "code1": 845160737,
                 "fnv": "6bf3b9323fa3bfbc", "bit18_count": 961},
        "Rect": {"verts": 24, "tris": 12, "code0": 681740840, "code1": 511305630,
                 "fnv": "57314e13d9be5ad1", "bit18_count": 6},
        "Image_Test": {"verts": 1734, "tris": 3072, "code0": 12483, "code1": 613558434,
                       "fnv": "f233f321e93d9963", "bit18_count": 1536},
        "combo_topology_fnv": {"value": "b7504c611d4a66c3",
                               "def": "FNV-1a64 folding u32 values parent,childL,childR per node, "
                                      "nodes 0..11774 (SURVEY §8(c), survey instrumentation)"},
    }
    with open(os.path.join(HERE, "shadersim_kats.json"), "w") as f:
        json.dump(kats, f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
