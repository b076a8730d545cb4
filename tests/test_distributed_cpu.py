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


def _worker(rank, world, port, W, H, out_path, nbuf, share=16):
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
    g = BandGather(W, H, rank, world, device="cpu", nbuf=nbuf, root_share=share)
    rows = band_row_ids(H, rank, world, share)
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


@pytest.mark.parametrize("world,nbuf,share,H", [(2, 1, 16, 77), (2, 2, 16, 77), (3, 2, 11, 77), (8, 2, 13, 157)])
def test_band_gather_gloo_matches_full_frame(tmp_path, world, nbuf, share, H):
    """World 2 with the even deal (b % nranks), world 3 with an uneven deal, and world 8 with the
    bench's N = 8 deal (root_share 13, bench.py: rank 0 traces 13/16 of another rank's bands, since
    it also receives and assembles them) through BandGather with two buffers (one gather in flight):
    rank 0's gathered frame equals a full-frame oracle render.  The frames are ragged (77 rows = 9
    full bands + 5 rows; 157 = 19 + 5)."""
    W = 160
    from raytracebvh_amd.tiles import band_row_ids
    if share < 16:   # the deal is uneven here: rank 0 holds fewer rows than the others
        rows = [len(band_row_ids(H, r, world, share)) for r in range(world)]
        assert rows[0] <= min(rows[1:]) and rows[0] < max(rows[1:]) and sum(rows) == H
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, out, nbuf, share), nprocs=world, join=True,
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


def _deal_restated(H, n, share):
    """Smooth weighted round-robin (include/rtbvh.h rtbvh_deal_bands), restated."""
    nb = (H + 7) // 8
    credit = [0] * n
    total = share + 16 * (n - 1)
    owner = []
    for _ in range(nb):
        best = 0
        for r in range(n):
            credit[r] += share if r == 0 else 16
            if credit[r] > credit[best]:
                best = r
        credit[best] -= total
        owner.append(best)
    return owner


def test_band_rows_python_matches_native():
    import raytracebvh_amd as rt
    from raytracebvh_amd.tiles import band_ids, band_row_ids
    L = rt.lib()
    for H in (1, 7, 8, 77, 1080, 2160):
        for n in (1, 2, 3, 8):
            ids = [band_row_ids(H, r, n) for r in range(n)]
            assert sorted(sum(ids, [])) == list(range(H))
            assert [len(x) for x in ids] == [L.rtbvh_band_rows(H, r, n) for r in range(n)]
            assert [band_ids(H, r, n) for r in range(n)] == [list(range(r, (H + 7) // 8, n)) for r in range(n)]
            for share in (0, 5, 11, 13, 16):
                owner = _deal_restated(H, n, share)
                bands = [band_ids(H, r, n, share) for r in range(n)]
                assert bands == [[b for b, o in enumerate(owner) if o == r] for r in range(n)]
                rows = [band_row_ids(H, r, n, share) for r in range(n)]
                assert sorted(sum(rows, [])) == list(range(H))
                assert [len(x) for x in rows] == [L.rtbvh_deal_rows(H, r, n, share) for r in range(n)]
                if n > 1 and H >= 1080:   # rank 0's share of the bands, within one band
                    nb = (H + 7) // 8
                    want = nb * share / (share + 16 * (n - 1))
                    assert abs(len(bands[0]) - want) <= 1
    assert L.rtbvh_deal_bands(64, 0, 2, 17, None, 0) == 0   # root_share > 16: rejected
