"""The world > 1 exchange of the native step, through the real RCCL transport, on one
GPU (VERDICT r03 missing #2): sml_hybrid_set_force_exchange makes a world-1 loop with
an RCCL communicator send its outvec rows through ncclAllGather
(sml_comm_allgather, replacing the MPI gather/scatter of sendrecievegrid,
mpires.f90:338-430, 575-581, 644-703, 733-736) and advance from the receive slab
(sml_hybrid_advance_slabs) with the separate assembly -- exactly the code a rank of
an N-GPU run executes after its all-gather.  It must be bitwise the identity step
(the finish assembling the grids itself), with the slab ocean's sst in the rows and
the pipelined loop, over 4 steps including a slab step.

Runs in a child process: torch.distributed's NCCL group is initialised there as
bench.py does, which must not leak into the other tests."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_forced_rccl_exchange_is_bitwise_the_identity_step(cuda, tmp_path):
    out = str(tmp_path / "force.npz")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_force_exchange_child.py")
    p = subprocess.run([sys.executable, "-u", child, out], timeout=110, capture_output=True, text=True)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    got = dict(np.load(out))
    assert int(got["n_forced"]) == 4, "every forced step must go through ncclAllGather"
    assert int(got["n_ident"]) == 0
    keys = [k[len("forced_"):] for k in got if k.startswith("forced_")]
    assert len(keys) == 4 * 10
    for k in sorted(keys):
        np.testing.assert_array_equal(got["forced_" + k], got["ident_" + k], err_msg=k)
    # the slab step changed the sst grid, and the exchange rows carry it
    assert not np.array_equal(got["ident_sst3"], got["ident_sst0"])
    assert got["ident_ov3"].shape[1] == 140
