"""The library's own RCCL communicator (sml_comm_*, include/speedy_ml.h) for a Python
host: rank 0's unique id is broadcast over an initialised torch.distributed group,
then every rank joins with ncclCommInitRank.  Handed to HybridLoop, it makes the
outvec all-gather part of the native step (sml_hybrid_step: ncclAllGather on the
loop's main stream, src/mpires.f90:338-716's exchange), so it costs no cross-stream
event hops between torch's NCCL stream and the loop's.
"""
from __future__ import annotations

import ctypes

from ._lib import check, lib

UNIQUE_ID_BYTES = 128  # NCCL_UNIQUE_ID_BYTES


class NativeComm:
    def __init__(self, world: int, rank: int, group=None):
        buf = (ctypes.c_ubyte * UNIQUE_ID_BYTES)()
        if rank == 0:
            check(lib().sml_comm_unique_id(buf))
        if world > 1:
            import torch.distributed as dist

            obj = [bytes(buf) if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0, group=group)
            buf = (ctypes.c_ubyte * UNIQUE_ID_BYTES).from_buffer_copy(obj[0])
        h = ctypes.c_void_p()
        check(lib().sml_comm_create(world, rank, buf, ctypes.byref(h)))
        self._h = h
        self.world, self.rank = world, rank

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            check(lib().sml_comm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalRank:
    """Rank `rank` of `world` without a transport (sml_comm_create_local): a
    HybridLoop created with it predicts its share of processor_decomposition and
    advances from slabs the host gathered itself (HybridLoop.advance_slabs) -- the
    sharded path without RCCL, e.g. every rank of an N-rank decomposition on one GPU."""

    def __init__(self, world: int, rank: int):
        h = ctypes.c_void_p()
        check(lib().sml_comm_create_local(world, rank, ctypes.byref(h)))
        self._h = h
        self.world, self.rank = world, rank

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            check(lib().sml_comm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def exchange_plan(numregions: int, world: int):
    """sml_exchange_plan: (maxc, contiguous, perm) of the all-gather's [world][maxc]
    slabs; perm[r] = the slab row of region r."""
    import numpy as np

    from ._lib import ptr

    maxc, contig = ctypes.c_int(), ctypes.c_int()
    perm = np.zeros(numregions, dtype=np.int32)
    check(lib().sml_exchange_plan(numregions, world, ctypes.byref(maxc), ctypes.byref(contig), ptr(perm)))
    return maxc.value, bool(contig.value), perm
