"""Host-side decomposition logic (speedy_ml_amd.domain) against the oracle's
restatement of res_domain.f90 and the reference's known shape classes."""
import numpy as np

import oracle
from speedy_ml_amd import domain


def test_geometry_matches_oracle_all_regions():
    for r in range(1152):
        g = domain.region_geometry(r)
        o = oracle.region_geometry(r)
        assert (g.res_xstart, g.res_xend, g.res_ystart, g.res_yend) == (
            o["res_xstart"], o["res_xend"], o["res_ystart"], o["res_yend"])
        assert (g.in_xstart, g.in_xend, g.in_ystart, g.in_yend, g.inx, g.iny) == (
            o["input_xstart"], o["input_xend"], o["input_ystart"], o["input_yend"], o["inputxchunk"],
            o["inputychunk"])
        assert (g.pole, g.periodic) == (bool(o["pole"]), bool(o["periodic"]))


def test_periodic_wrap_and_poles():
    g0 = domain.region_geometry(0)  # first x-row, southern pole
    assert [g0.input_x(lx) for lx in range(1, 5)] == [96, 1, 2, 3]
    assert g0.iny == 3 and g0.in_ystart == 1
    g_last = domain.region_geometry(1151)  # last x-row, northern pole
    assert [g_last.input_x(lx) for lx in range(1, 5)] == [94, 95, 96, 1]
    assert g_last.iny == 3 and g_last.in_yend == 48
    g_mid = domain.region_geometry(24 * 10 + 5)
    assert [g_mid.input_x(lx) for lx in range(1, 5)] == [20, 21, 22, 23]


def test_reservoir_shape_classes():
    # 4x4+sst 576/5760/33177, 4x4 560/6160/37945,
    # polar+sst 432/6048/36578, polar 420/5880/34574
    cases = {(5, True): (576, 5760, 33177), (5, False): (560, 6160, 37945),
             (0, True): (432, 6048, 36578), (0, False): (420, 5880, 34574)}
    for (region, sst), (ninp, n, k) in cases.items():
        s = domain.reservoir_sizes(region, sst)
        assert (s.ninp, s.n, s.k) == (ninp, n, k)
        o = oracle.reservoir_sizes(region, sst)
        assert (o["ninp"], o["n"], o["k"], o["chunk_pred"], o["chunk_speedy"]) == (ninp, n, k, 136, 132)


def test_sst_mask_classes():
    m = domain.load_sst_mask()
    polar = np.array([domain.region_geometry(r).pole for r in range(1152)])
    assert int((~polar & (m == 1)).sum()) == 976
    assert int((~polar & (m == 0)).sum()) == 80
    assert int((polar & (m == 1)).sum()) == 51
    assert int((polar & (m == 0)).sum()) == 45


def test_processor_decomposition_partitions():
    for nproc in (1, 2, 3, 4, 5, 7, 8, 16, 96):
        allr = []
        for rank in range(nproc):
            allr += domain.processor_decomposition(1152, nproc, rank)
        assert sorted(allr) == list(range(1152)), nproc
    # 8 ranks: contiguous blocks of 144 (res_domain.f90:37-52)
    assert domain.processor_decomposition(1152, 8, 3) == list(range(432, 576))


def test_radius_by_region_matches_oracle():
    for r in range(0, 1152, 7):
        assert domain.radius_by_region(r) == oracle.radius_by_region(r)


def test_native_decomposition_matches_python():
    """sml_processor_decomposition (the native loop's check of its communicator's
    rank, sml_hybrid_create) gives every rank the regions the Python host loads."""
    import ctypes

    from speedy_ml_amd._lib import check, lib

    buf = (ctypes.c_int * 1152)()
    cnt = ctypes.c_int()
    for nproc in (1, 2, 3, 4, 7, 8, 16):
        for rank in range(nproc):
            check(lib().sml_processor_decomposition(1152, nproc, rank, buf, ctypes.byref(cnt)))
            assert list(buf[:cnt.value]) == domain.processor_decomposition(1152, nproc, rank), (nproc, rank)
