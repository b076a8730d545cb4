"""The multi-GPU path (band sharding + framebuffer gather to rank 0) on CPU with
world_size 2 over gloo.  The CPU oracle renders each rank's bands (standing in
for the GPU kernels, test only); rank 0's gathered frame must equal a full-frame
oracle render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.conftest import REPO, load_scene_fixture


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, out_path, nbuf):
    import sys
    sys.path.insert(0, REPO)
    from oracle import lib as orc
    from raytracebvh_amd.tiles import BandGather, band_row_ids

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = load_scene_fixture("Test")
    s = orc.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    wvp, wv = orc.camera_reference(W, H)
    nodes = orc.build(s, wvp)
    g = BandGather(W, H, rank, world, device="cpu", nbuf=nbuf)
    rows = band_row_ids(H, rank, world)
    mine = torch.zeros((len(rows), W, 4))
    for k, y in enumerate(rows):   # this rank's bands, compact
        rgba, _, _ = orc.trace(s, nodes, wvp, wv, W, H, 1, y, y + 1, 1)
        mine[k] = torch.from_numpy(rgba[0])
    # 3 frames with one gather in flight (the bench's loop); frame i = render + i, so a
    # buffer handed to the wrong frame shows up in the assembled values
    frames, pending = [], None
    for i in range(3):
        g.band_buffer(i)[: len(rows)] = mine + i
        if nbuf == 1:   # one buffer: synchronous gather per frame
            f = g.gather(i)
            if rank == 0:
                frames.append(f.clone())
            continue
        h = g.gather_async(i)
        if pending is not None:
            f = g.assemble(*pending)
            if rank == 0:
                frames.append(f.clone())
        pending = (i, h)
    if pending is not None:
        f = g.assemble(*pending)
        if rank == 0:
            frames.append(f.clone())
    if rank == 0:
        np.save(out_path, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("nbuf", [1, 2])
def test_band_gather_gloo_matches_full_frame(tmp_path, nbuf):
    W, H, world = 160, 77, 2   # ragged: 77 rows = 9 full bands + 5 rows
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, out, nbuf), nprocs=world, join=True,
                       start_method="spawn")
    from oracle import lib as orc
    d = load_scene_fixture("Test")
    s = orc.Scene(d["vertices"], d["indices"], d["mat_indices"], d["material_blob"])
    wvp, wv = orc.camera_reference(W, H)
    full, _, _ = orc.trace(s, orc.build(s, wvp), wvp, wv, W, H, 1)
    got = np.load(out)
    assert got.shape[0] == 3
    for i in range(3):
        np.testing.assert_array_equal(got[i], full + np.float32(i))
    assert (got[0] != 0.5).any()   # the scene is visible in this frame


def test_band_rows_python_matches_native():
    import raytracebvh_amd as rt
    from raytracebvh_amd.tiles import band_row_ids
    for H in (1, 7, 8, 77, 1080, 2160):
        for n in (1, 2, 3, 8):
            ids = [band_row_ids(H, r, n) for r in range(n)]
            assert sorted(sum(ids, [])) == list(range(H))
            assert [len(x) for x in ids] == [rt.lib().rtbvh_band_rows(H, r, n) for r in range(n)]
