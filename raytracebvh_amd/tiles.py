"""Image-band sharding of a frame over ranks + the framebuffer gather.

The reference is single-GPU.  Multi-GPU here: every rank holds the same scene
and builds the same BVH (deterministic replicas); the frame's 8-row bands are
dealt round-robin (band b -> rank b % nranks, which balances the centre-heavy hit
distribution), each rank traces its bands into a compact buffer
(rtbvh_trace_band_async), and rank 0 gathers the buffers over torch.distributed
("nccl" = RCCL over xGMI on MI355X; "gloo" in the CPU tests) and scatters the rows
into the frame.  The only collective of the path is that gather.
"""
from __future__ import annotations

BAND = 8


def band_row_ids(H: int, rank: int, nranks: int) -> list:
    """Frame rows owned by `rank`, in the order they appear in its compact buffer."""
    return [y for b in range(rank, (H + BAND - 1) // BAND, nranks) for y in range(BAND * b, min(BAND * b + BAND, H))]


class BandGather:
    """Band buffer of this rank and, on rank 0, the assembled frame."""

    def __init__(self, W: int, H: int, rank: int, world: int, device, dtype=None):
        import torch

        dtype = dtype or torch.float32
        self.W, self.H, self.rank, self.world = W, H, rank, world
        self.rows = [len(band_row_ids(H, r, world)) for r in range(world)]
        self.max_rows = max(self.rows)
        # every rank sends a buffer of the same (max) size: dist.gather needs equal shapes
        self.band = torch.zeros((self.max_rows, W, 4), dtype=dtype, device=device)
        self.frame = None
        self.gather_list = None
        self.row_idx = None
        if world == 1:
            self.frame = self.band
        elif rank == 0:
            self.frame = torch.empty((H, W, 4), dtype=dtype, device=device)
            self.gather_list = [torch.empty_like(self.band) for _ in range(world)]
            self.row_idx = [torch.tensor(band_row_ids(H, r, world), dtype=torch.long, device=device)
                            for r in range(world)]

    def gather(self):
        """Collect every rank's bands on rank 0 and assemble the frame there."""
        if self.world == 1:
            return self.frame
        import torch.distributed as dist

        dist.gather(self.band, self.gather_list if self.rank == 0 else None, dst=0)
        if self.rank == 0:
            for r in range(self.world):
                self.frame.index_copy_(0, self.row_idx[r], self.gather_list[r][: self.rows[r]])
        return self.frame
