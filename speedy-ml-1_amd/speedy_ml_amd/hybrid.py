"""The hybrid prediction loop on one rank: reservoir predict for the rank's regions,
the outvec exchange, SPEEDY's 6-h window on the assembled grid, and the re-tiling
of the next step's inputs.

Reference: the time loop of src/parallelmain.f90:204-270 -- `predict` per region
(:225-234), then `sendrecievegrid` (src/mpires.f90:218-780), which gathers every
outvec at the root, assembles the global grid (:300-478), runs SPEEDY on it
(`run_model`, :1516-1628: iogrid(30), stepone + 24 leapfrog steps, iogrid(31))
and scatters the next feedback tiles and SPEEDY local vectors (:558-751).

The data dependences of one step allow an overlap the reference's serial loop
does not use.  `predict` needs `feedback` (the overlap tiles of the assembled
grid) for the state update and for W_out(:, ncs+1:) x~, and SPEEDY's local vector
only for W_out(:, 1:ncs) local_model -- the split the reference itself computes
under `outvec_component_contribs` (mod_reservoir.f90:1456-1459).  So each step is
issued on two HIP streams:

    main   : begin(fb_t) ........ wait(lm_t) finish -> exchange -> assemble -> tile fb_t+1
    speedy :   [iogrid(30) + window + iogrid(31) + tile lm_t+1 of step t-1]   wait(grid_t) ...

The reservoir's update and ~98 % of its readout bytes run while SPEEDY
integrates the previous step's window.  Results are identical to the one-stream
schedule (`overlap=False`, which uses the one-pass readout with the same sums).

Measured on MI355X: with the window at 3 launches per step the overlap did not
pay (profiles/r01h_*: under the readout's ~6 TB/s stream SPEEDY's small
latency-bound kernels waited far longer on memory); with the window at 2 leaner
launches per step it does: 496 vs 482 steps/s at 1 GPU and +0.6-1 % for the 2/4/8-
rank shares (profiles/r01o).  bench.py uses it by default.

The two streams are also given disjoint CUs (`speedy_cus`, default 64: SPEEDY on
CUs [0, 64), the reservoir on the other 192; sml_stream_create_cu_range).  Without
the split, SPEEDY's blocks (146-150 KB of LDS each) wait for a CU whose LDS the
update's blocks have left, and then share that CU's memory pipeline with readout
waves: the window ran 1.57 ms beside the readout vs 1.16 ms alone.  With it the
overlapped step went 1.66 -> 1.43 ms (tools/probe_host_calls.py; 48 or fewer CUs
for SPEEDY are slower: the 48 latitude-row blocks no longer have a CU each).
"""
from __future__ import annotations

import os

import torch

from ._lib import check, lib


class HybridLoop:
    """Owns the device-resident step buffers and the two streams of one rank.

    res: Reservoirs (this rank's regions), dyn: Dynamics with physics set,
    exchange: OutvecExchange, tisr: [nlocal, 16] standardized tisr inputs (device)
    or None (feedback tisr entries left as they are)."""

    def __init__(self, res, dyn, exchange, device, tisr=None, overlap: bool = True, nleap: int = 24,
                 side_priority: int = -1, speedy_cus: int | None = None):
        self.res, self.dyn, self.exchange, self.tisr = res, dyn, exchange, tisr
        self.overlap, self.nleap = overlap, nleap
        self.dev = torch.device(device)
        self.fb, self.lm, self.ov = res.alloc_io(self.dev)
        z = lambda *s: torch.zeros(s, dtype=torch.float64, device=self.dev)  # noqa: E731
        # variables3d(4, 96, 48, 8) / logp(96, 48) / precip(96, 48) in Fortran order
        self.g4, self.g2, self.pr = z(8, 48, 96, 4), z(48, 96), z(48, 96)
        self.f4, self.f2 = z(8, 48, 96, 4), z(48, 96)
        # two non-default streams: the legacy NULL stream synchronises implicitly with
        # every blocking stream, which would serialise the two chains again.  SPEEDY's
        # chain is latency-bound: its high-priority stream keeps its small launches
        # ahead of the readout's blocks
        self._owned = []
        if speedy_cus is None:
            speedy_cus = int(os.environ.get("SML_SPEEDY_CUS", "64"))
        ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count if overlap else 0
        if overlap and 0 < speedy_cus < ncu:
            with torch.cuda.device(self.dev):
                self.side = self._cu_stream(0, speedy_cus)
                self.main = self._cu_stream(speedy_cus, ncu - speedy_cus)
            res.set_read_waves(0)  # pacing the readout only pays when it shares CUs with SPEEDY
        else:
            self.main = torch.cuda.Stream(self.dev)
            self.side = torch.cuda.Stream(self.dev, priority=side_priority) if overlap else self.main
        self.ev_grid = torch.cuda.Event()
        self.ev_lm = torch.cuda.Event()

    def _cu_stream(self, first: int, count: int):
        import ctypes

        h = ctypes.c_void_p()
        check(lib().sml_stream_create_cu_range(first, count, ctypes.byref(h)))
        self._owned.append(h)
        return torch.cuda.ExternalStream(h.value, device=self.dev)

    def close(self):
        """Wait for the loop's work and release the CU-range streams it created."""
        if self._owned:
            torch.cuda.synchronize(self.dev)
            for h in self._owned:
                check(lib().sml_stream_destroy(h))
            self._owned = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def start(self, g4, g2, pr, f4, f2):
        """start_prediction analogue: inputs of the first step from an analysis grid
        (g4, g2, pr) and a SPEEDY forecast from it (f4, f2)."""
        self.main.wait_stream(torch.cuda.current_stream(self.dev))
        with torch.cuda.stream(self.main):
            self.g4.copy_(g4)
            self.g2.copy_(g2)
            self.pr.copy_(pr)
            self.f4.copy_(f4)
            self.f2.copy_(f2)
        self.res.tile_inputs(self.g4, self.g2, self.pr, self.f4, self.f2, self.tisr, self.fb, self.lm,
                             stream=self.main)
        self.ev_lm.record(self.main)

    def step(self):
        """One hybrid time step (asynchronous; `sync()` waits for it)."""
        m, s = self.main, self.side
        if self.overlap:
            self.res.predict_begin(self.fb, stream=m)
            m.wait_event(self.ev_lm)  # SPEEDY's forecast grids of the previous window
            # tile_local_model fused into the finish: one launch fewer on the critical path
            self.res.predict_finish_grid(self.f4, self.f2, self.lm, self.ov, stream=m)
        else:  # one pass (kReadFull): the same sums as begin + finish, one launch fewer
            self.res.predict(self.fb, self.lm, self.ov, stream=m)
        with torch.cuda.stream(m):
            glob = self.exchange(self.ov)  # RCCL all-gather over xGMI when world > 1
        self.res.assemble(glob, self.g4, self.g2, self.pr, stream=m)
        if self.overlap:  # (one stream: stream order suffices, and an event record costs ~7 us of GPU idle)
            self.ev_grid.record(m)
        self.res.tile_feedback(self.g4, self.g2, self.pr, self.tisr, self.fb, stream=m)
        if self.overlap:
            s.wait_event(self.ev_grid)
        self.dyn.from_grid(self.g4, self.g2, stream=s)   # iogrid(30)
        self.dyn.window(self.nleap, stream=s)            # stepone + 24 x step(2,2), physics on
        self.dyn.to_grid(self.f4, self.f2, stream=s)     # iogrid(31)
        if self.overlap:
            self.ev_lm.record(s)
        else:
            self.res.tile_local_model(self.f4, self.f2, self.lm, stream=s)

    def sync(self):
        if self.overlap:
            self.main.wait_event(self.ev_lm)
            # the local model of the last window, as the one-stream loop leaves it (the
            # overlapped steps tile it inside the next step's finish)
            self.res.tile_local_model(self.f4, self.f2, self.lm, stream=self.main)
        torch.cuda.synchronize(self.dev)
