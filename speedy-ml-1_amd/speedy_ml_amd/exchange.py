"""Outvec exchange across ranks: one all-gather per hybrid step.

Replaces the reference's root-centric MPI traffic of sendrecievegrid
(src/mpires.f90:338-430 worker->root MPI_SEND of every region's outvec, :587-716
root->worker MPI_SEND of every region's input tile): every rank contributes its
regions' outvecs, every rank ends up with all 1152 in global region order and
builds its own overlap tiles locally (the x halo is inside the gathered grid), so
no scatter is needed.  With backend "nccl" this is RCCL over xGMI; "gloo" runs the
same code on CPU tensors (tests).
"""
from __future__ import annotations

import numpy as np

from .domain import CHUNK_PRED, processor_decomposition


class OutvecExchange:
    def __init__(self, numregions: int, world: int, rank: int, nout: int = CHUNK_PRED, device="cpu",
                 dtype=None, group=None):
        import torch

        self.world, self.rank, self.numregions, self.nout, self.group = world, rank, numregions, nout, group
        dtype = dtype or torch.float64
        decomp = [processor_decomposition(numregions, world, r) for r in range(world)]
        counts = [len(d) for d in decomp]
        self.regions = decomp[rank]
        self.nlocal = counts[rank]
        self.maxc = max(counts)
        rows = np.concatenate([np.arange(counts[r]) + r * self.maxc for r in range(world)])
        owners = np.concatenate(decomp)
        # the all-gather result is already in global order when every rank holds the
        # same number of consecutive regions (1152 over 1/2/4/8 ranks)
        self.contiguous = len(set(counts)) == 1 and np.array_equal(owners, np.arange(numregions))
        self.perm = torch.from_numpy(rows[np.argsort(owners)]).to(device)
        if world > 1:
            self.send = torch.zeros((self.maxc, nout), dtype=dtype, device=device)
            self.recv = torch.zeros((self.maxc * world, nout), dtype=dtype, device=device)
            self.glob = torch.zeros((numregions, nout), dtype=dtype, device=device)

    def __call__(self, ov_local):
        """ov_local: [nlocal, nout] outvecs of this rank's regions (region order of
        processor_decomposition).  Returns [numregions, nout] in global region order."""
        import torch
        import torch.distributed as dist

        if self.world == 1:
            return ov_local
        if (self.nlocal == self.maxc and ov_local.is_contiguous() and ov_local.shape == self.send.shape
                and ov_local.dtype == self.send.dtype):
            src = ov_local  # even shares: sent as they are, no copy on the step's critical path
        else:
            self.send[:self.nlocal].copy_(ov_local)
            src = self.send
        dist.all_gather_into_tensor(self.recv, src, group=self.group)
        if self.contiguous:
            return self.recv
        torch.index_select(self.recv, 0, self.perm, out=self.glob)
        return self.glob
