"""map_rect's multi-rank executor over RCCL on the GPU.

The box has one GPU, so the job is a one-rank RCCL communicator: the executor
takes its distributed path (chunking, the status / outputs exchange and the
per-job column exchange are real ncclAllGather calls through
smg_comm_allgather) and must return exactly what the single-process path
returns, which the real reference pins (fixtures map_rect_hier_J*).  The
W > 1 partition / exchange logic runs under gloo in tests/test_sharding.py.
"""
import ctypes
import os

import numpy as np
import pytest

import gen
from _util import ROOT, golden, near_rel, prebuilt

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tests", "cpp", "_bin", "libmaprect_dist.so")
_AG = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.c_longlong, ctypes.POINTER(ctypes.c_double),
                       ctypes.c_void_p)
_TAIL = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
         ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
         ctypes.c_char_p, ctypes.c_int]


def _lib():
    lib = ctypes.CDLL(prebuilt(LIB))
    lib.maprect_hier.restype = ctypes.c_int
    lib.maprect_hier.argtypes = [ctypes.c_int, ctypes.c_int, _AG, ctypes.c_void_p] + _TAIL
    lib.maprect_hier_rccl.restype = ctypes.c_int
    lib.maprect_hier_rccl.argtypes = _TAIL
    return lib


def _call(lib, rccl, xr, xi, th, mode):
    J = xr.shape[0]
    fx = ctypes.c_double()
    grad = np.zeros(2 + J)
    vals = np.zeros(3 * J + 3)
    nv = ctypes.c_int()
    err = ctypes.create_string_buffer(512)
    xrf = np.ascontiguousarray(xr, dtype=np.float64)
    xif = np.ascontiguousarray(xi, dtype=np.int32)
    thf = np.ascontiguousarray(th, dtype=np.float64)
    tail = (J, xrf.ctypes.data_as(ctypes.c_void_p), xr.shape[1], xif.ctypes.data_as(ctypes.c_void_p),
            thf.ctypes.data_as(ctypes.c_void_p), mode, ctypes.byref(fx), grad.ctypes.data_as(ctypes.c_void_p),
            vals.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nv), err, 512)
    if rccl:
        rc = lib.maprect_hier_rccl(*tail)
    else:
        rc = lib.maprect_hier(1, 0, _AG(lambda *a: None), None, *tail)
    return rc, fx.value, grad, vals[:nv.value], err.value.decode()


@pytest.mark.parametrize("J", [1, 7, 16])
def test_map_rect_rccl_one_rank(J):
    lib = _lib()
    xr, xi, th = gen.maprect_inputs(J)
    d = golden(f"map_rect_hier_J{J}")
    for mode in range(4):
        rc, fx, g, v, err = _call(lib, True, xr, xi, th, mode)
        rc1, fx1, g1, v1, _ = _call(lib, False, xr, xi, th, mode)
        assert rc == 0 and rc1 == 0, err
        assert fx == fx1 and np.array_equal(g, g1) and np.array_equal(v, v1), mode
        near_rel(fx, d["fx"], 1e-12, what="fx")
        near_rel(v, d["values"], 1e-12, what="values")
        if mode == 0:
            near_rel(g, d["grad"], 1e-10, what="grad")


def test_map_rect_rccl_failing_job():
    lib = _lib()
    xr, xi, th = gen.maprect_inputs(7)
    xi[3, 1] = 1
    rc, _, _, _, err = _call(lib, True, xr, xi, th, 0)
    assert rc == 1 and err == "Error during MPI evaluation.", (rc, err)
    # the communicator was left cleanly: a following call works
    xi[3, 1] = 0
    rc, fx, _, _, err = _call(lib, True, xr, xi, th, 0)
    assert rc == 0, err
    near_rel(fx, golden("map_rect_hier_J7")["fx"], 1e-12, what="fx after failure")


def test_comm_scatterv_one_rank():
    """smg_comm_scatterv on a one-rank communicator: the grouped point-to-point
    calls (none to make) and the root's own block copied on the device --
    the map_rect job data scatter's RCCL entry (W > 1 scatter logic: gloo in
    tests/test_sharding.py::test_map_rect_job_data_cache_gloo)."""
    from math_amd import hip
    with hip.Context(0, 1 << 26) as c:
        idb = ctypes.create_string_buffer(128)
        assert c.lib.smg_comm_unique_id(idb) == 0
        c.call("smg_comm_init", 1, 0, idb)
        try:
            a = np.arange(37, dtype=np.float64) * 0.5 - 3.0
            src = c.put(a)
            dst = c.alloc(a.nbytes)
            counts = (ctypes.c_longlong * 1)(37)
            c.call("smg_comm_scatterv", src, counts, dst, 0)
            assert np.array_equal(c.get(dst, 37), a)
            counts0 = (ctypes.c_longlong * 1)(0)
            c.call("smg_comm_scatterv", src, counts0, dst, 0)  # an empty block is a no-op
            assert c.lib.smg_comm_scatterv(c.ptr, src, counts, dst, 1) != 0  # root outside the job
        finally:
            c.call("smg_comm_destroy")
