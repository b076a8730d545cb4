"""Image-band sharding of a frame over ranks + the framebuffer gather.

The reference is single-GPU.  Multi-GPU here: every rank holds the same scene
and builds the same BVH (deterministic replicas); the frame's 8-row bands are
dealt by smooth weighted round-robin (rtbvh_deal_bands: rank 0 weighs root_share/16
of another rank, since it also receives and assembles every rank's bands; 16 gives
band b -> rank b % nranks; either way the bands of a rank are spread over the frame,
which balances the centre-heavy hit distribution), each rank traces its bands into a
compact buffer (rtbvh_trace_band_async), and rank 0 gathers the buffers over
torch.distributed ("nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests) and
scatters the rows into the frame.  The only collective of the path is that gather.

Frames in flight: with `nbuf=2` the band buffer of frame i+1 is a different buffer
than frame i's, so frame i's gather (on the collective's own stream) runs while
frame i+1 is traced; `assemble(i)` makes the compute stream wait for gather i before
the buffer is traced into again.
"""
from __future__ import annotations

BAND = 8


def band_ids(H: int, rank: int, nranks: int, root_share: int = 16) -> list:
    """The bands of `rank` under the deal, in order (rtbvh_deal_bands)."""
    import ctypes

    import numpy as np

    from . import _lib as _L
    n = _L.lib().rtbvh_deal_bands(H, rank, nranks, root_share, None, 0)
    out = np.zeros(max(n, 1), np.uint32)
    _L.lib().rtbvh_deal_bands(H, rank, nranks, root_share, ctypes.c_void_p(out.ctypes.data), n)
    return [int(b) for b in out[:n]]


def band_row_ids(H: int, rank: int, nranks: int, root_share: int = 16) -> list:
    """Frame rows owned by `rank`, in the order they appear in its compact buffer."""
    return [y for b in band_ids(H, rank, nranks, root_share) for y in range(BAND * b, min(BAND * b + BAND, H))]


class BandGather:
    """Band buffer(s) of this rank and, on rank 0, the assembled frame."""

    def __init__(self, W: int, H: int, rank: int, world: int, device, dtype=None, nbuf: int = 1,
                 root_share: int = 16):
        import torch

        dtype = dtype or torch.float32
        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.nbuf = nbuf
        self.root_share = root_share
        self.rows = [len(band_row_ids(H, r, world, root_share)) for r in range(world)]
        self.max_rows = max(self.rows)
        # every rank sends a buffer of the same (max) size: dist.gather needs equal shapes
        self.bands = [torch.zeros((self.max_rows, W, 4), dtype=dtype, device=device) for _ in range(self.nbuf)]
        self.band = self.bands[0]
        self.frame = None
        self.frames = None
        self.gather_lists = None
        self.row_idx = None
        if world == 1:
            self.frames = self.bands   # one rank: the band buffer of a frame is that frame
            self.frame = self.band
        elif rank == 0:
            # one assembled frame per buffer: frames in flight on different streams never
            # write the same frame buffer
            self.frames = [torch.empty((H, W, 4), dtype=dtype, device=device) for _ in range(self.nbuf)]
            self.frame = self.frames[0]
            self.gather_lists = [[torch.empty_like(self.band) for _ in range(world)] for _ in range(self.nbuf)]
            self.row_idx = [torch.tensor(band_row_ids(H, r, world, root_share), dtype=torch.long, device=device)
                            for r in range(world)]

    def band_buffer(self, i: int):
        """The buffer frame i is traced into."""
        return self.bands[i % self.nbuf]

    def gather_async(self, i: int):
        """Start gathering frame i's bands to rank 0; returns a handle for assemble()."""
        if self.world == 1:
            return None
        import torch.distributed as dist

        k = i % self.nbuf
        return dist.gather(self.bands[k], self.gather_lists[k] if self.rank == 0 else None, dst=0, async_op=True)

    def assemble(self, i: int, handle):
        """Wait (on the stream) for gather i and, on rank 0, scatter its rows into the frame."""
        if self.world == 1:
            return self.frames[i % self.nbuf]
        handle.wait()
        if self.rank == 0:
            gl = self.gather_lists[i % self.nbuf]
            f = self.frames[i % self.nbuf]
            for r in range(self.world):
                f.index_copy_(0, self.row_idx[r], gl[r][: self.rows[r]])
            return f
        return None

    def gather(self, i: int = 0):
        """Collect frame i's bands on rank 0 and assemble the frame there (synchronous)."""
        return self.assemble(i, self.gather_async(i))
