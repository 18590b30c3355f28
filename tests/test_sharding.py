"""Row sharding of the GLM reducer and the multi-rank
map_rect executor (§8(f) row 1) on CPU, world_size 2 and 3, gloo.

The multi-GPU path partitions the R rows with stan::math::row_partition (the
C++ header function, called here through libsmg_bench.so), generates each
rank's block of the config-4 streams in place (a SplitMix64 stream started k
elements later is the stream of seed + k*GOLDEN, math_amd/bench/smg_bench.cpp),
computes the block's [logp, alpha', beta'] and sums them with ONE all-reduce.
Here every rank computes its block with the oracle (CPU restatement) and the
all-reduce is gloo's; the result must equal the reference's single-call
fixture (glm_R100000_M256, real Stan Math) within 1e-10 -- the decomposition
the RCCL path uses is exact up to summation order.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gen
from _util import ROOT, f64, golden, near_rel, oracle, ptr, prebuilt

GOLDEN_INC = 0x9E3779B97F4A7C15
BENCH_LIB = os.path.join(ROOT, "math_amd", "lib", "libsmg_bench.so")


def _partition(R, world, rank, lib=None):
    """stan::math::row_partition, through the bench library or (in a process
    that already loaded it) the glm_dist test library."""
    b0, b1 = ctypes.c_longlong(), ctypes.c_longlong()
    if lib is None:
        ctypes.CDLL(prebuilt(BENCH_LIB)).smg_bench_row_partition(ctypes.c_longlong(R), world, rank, ctypes.byref(b0),
                                                       ctypes.byref(b1))
    else:
        lib.glm_dist_row_partition(ctypes.c_longlong(R), world, rank, ctypes.byref(b0), ctypes.byref(b1))
    return b0.value, b1.value


def _offset_seed(seed, k):
    return (seed + k * GOLDEN_INC) % (1 << 64)


def _block(R, M, b0, b1):
    """rows [b0, b1) of the config-4 data generated from offset streams only."""
    rows = b1 - b0
    x = np.empty((rows, M), order="F")
    for j in range(M):
        x[:, j] = gen.unif(_offset_seed(gen.SEED + 41, b0 + j * R), rows, -1.0, 1.0) * np.sqrt(3.0)
    y = gen.bernoulli(_offset_seed(gen.SEED + 42, b0), rows, 0.5)
    return x, y


def _rank_main(rank, world, port, R, M, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = _partition(R, world, rank)
    x, y = _block(R, M, b0, b1)
    _, _, th = gen.glm_inputs(1, M)
    ga, gb = np.zeros(1), np.zeros(M)
    yy = np.ascontiguousarray(y, dtype=np.int32)
    lp = oracle().oracle_glm(ptr(yy), ptr(f64(x.ravel(order="F"))), b1 - b0, M, th[0], ptr(f64(th[1:])),
                             ptr(ga), ptr(gb))
    buf = torch.tensor(np.concatenate([[lp], ga, gb]), dtype=torch.float64)
    dist.all_reduce(buf)  # the one exchange of the sharded path
    if rank == 0:
        np.save(out, buf.numpy())
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _spawn(fn, world, *args):
    """mp.start_processes with a fresh rendezvous port: fn(rank, world, port, *args).
    The port is free when probed but can be taken by another process on a
    shared host before rank 0 binds it (EADDRINUSE); only that case is retried,
    with a new port."""
    for attempt in range(3):
        try:
            mp.start_processes(fn, args=(world, _free_port()) + args, nprocs=world, join=True,
                               start_method="spawn")
            return
        except mp.ProcessRaisedException as e:
            if "EADDRINUSE" not in str(e) or attempt == 2:
                raise


def test_partition_tiles_rows():
    for R in (0, 1, 7, 100000, 10_000_000):
        for world in (1, 2, 3, 8):
            blocks = [_partition(R, world, r) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == R
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))
            sizes = [b1 - b0 for b0, b1 in blocks]
            assert max(sizes) - min(sizes) <= 1


def test_offset_streams_equal_global_stream():
    R, M = 1000, 3
    full = gen.unif(gen.SEED + 41, R * M, -1.0, 1.0).reshape(M, R).T * np.sqrt(3.0)
    yfull = gen.bernoulli(gen.SEED + 42, R, 0.5)
    for b0, b1 in ((0, 1000), (0, 333), (333, 1000), (517, 518)):
        x, y = _block(R, M, b0, b1)
        assert np.array_equal(x, full[b0:b1])
        assert np.array_equal(y, yfull[b0:b1])


def test_glm_two_ranks_gloo_matches_reference(tmp_path):
    d = golden("glm_R100000_M256")
    R, M = int(d["R"]), int(d["M"])
    out = str(tmp_path / "r0.npy")
    _spawn(_rank_main, 2, R, M, out)
    res = np.load(out)
    near_rel(res[0], d["fx"], 1e-12, what="fx")
    near_rel(res[1:], d["grad"], 1e-10, what="grad")


# ---------------------------------------------------------------- map_rect executor
MAPRECT_LIB = os.path.join(ROOT, "tests", "cpp", "_bin", "libmaprect_dist.so")
_AG = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.c_longlong, ctypes.POINTER(ctypes.c_double),
                       ctypes.c_void_p)


def _maprect_call(lib, world, rank, cb, xr, xi, th, mode):
    J = xr.shape[0]
    fx = ctypes.c_double()
    grad = np.zeros(2 + J)
    vals = np.zeros(3 * J + 3)
    nv = ctypes.c_int()
    err = ctypes.create_string_buffer(512)
    xrf = np.ascontiguousarray(xr, dtype=np.float64)
    xif = np.ascontiguousarray(xi, dtype=np.int32)
    thf = np.ascontiguousarray(th, dtype=np.float64)
    rc = lib.maprect_hier(world, rank, cb, None, J, xrf.ctypes.data_as(ctypes.c_void_p), xr.shape[1],
                          xif.ctypes.data_as(ctypes.c_void_p), thf.ctypes.data_as(ctypes.c_void_p), mode,
                          ctypes.byref(fx), grad.ctypes.data_as(ctypes.c_void_p),
                          vals.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nv), err, 512)
    return rc, fx.value, grad, vals[:nv.value], err.value.decode()


def _maprect_lib():
    lib = ctypes.CDLL(prebuilt(MAPRECT_LIB))
    lib.maprect_hier.restype = ctypes.c_int
    lib.maprect_hier.argtypes = [ctypes.c_int, ctypes.c_int, _AG, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_double), ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    return lib


def _maprect_rank(rank, world, port, cases, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def allgather(send, count, recv, _user):
        t = torch.from_numpy(np.ctypeslib.as_array(send, shape=(count,)).copy())
        parts = [torch.empty(count, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, t)
        np.ctypeslib.as_array(recv, shape=(count * world,))[:] = torch.cat(parts).numpy()
        calls.append(count)

    cb = _AG(allgather)
    lib = _maprect_lib()
    res = {}
    for J, fail in cases:
        xr, xi, th = gen.maprect_inputs(J)
        if fail >= 0:
            xi[fail, 1] = 1
        for mode in range(4):
            rc, fx, grad, vals, err = _maprect_call(lib, world, rank, cb, xr, xi, th, mode)
            res[f"{J}_{fail}_{mode}"] = dict(rc=rc, fx=fx, grad=grad, vals=vals, err=err)
    res["collectives"] = len(calls)
    np.save(out + f".{rank}.npy", np.array(res, dtype=object), allow_pickle=True)
    dist.destroy_process_group()


MAPRECT_CASES = [(7, -1), (1, -1), (16, -1), (7, 5), (16, 0)]


@pytest.mark.parametrize("world", [2, 3])
def test_map_rect_executor_gloo(tmp_path, world):
    """map_rect over W gloo ranks (each evaluates its mpi_map_chunks share and
    two all-gathers exchange the per-job columns) == the same executor in one
    process, bit for bit, and == the real reference's map_rect (fixtures
    map_rect_hier_J*, jobs with 1..3 outputs each) within 1e-12 / 1e-10; every
    operand combination (var/var, var/data, data/var, data/data); a job that
    throws on one rank makes every rank throw the reference's
    "Error during MPI evaluation."."""
    out = str(tmp_path / "mr")
    _spawn(_maprect_rank, world, MAPRECT_CASES, out)
    ranks = [np.load(out + f".{r}.npy", allow_pickle=True).item() for r in range(world)]
    lib = _maprect_lib()
    cb = _AG(lambda *a: None)
    for J, fail in MAPRECT_CASES:
        xr, xi, th = gen.maprect_inputs(J)
        if fail >= 0:
            xi[fail, 1] = 1
        for mode in range(4):
            key = f"{J}_{fail}_{mode}"
            rc1, fx1, g1, v1, err1 = _maprect_call(lib, 1, 0, cb, xr, xi, th, mode)
            for r in range(world):
                got = ranks[r][key]
                if fail >= 0:
                    assert rc1 == 1 and err1 == "hier_job: job failed", (key, rc1, err1)
                    assert got["rc"] == 1 and got["err"] == "Error during MPI evaluation.", (key, r, got)
                    continue
                assert rc1 == 0 and got["rc"] == 0, (key, r, got["err"], err1)
                assert got["fx"] == fx1 and np.array_equal(got["grad"], g1) and np.array_equal(got["vals"], v1), (key, r)
            if fail < 0:
                d = golden(f"map_rect_hier_J{J}")
                near_rel(fx1, d["fx"], 1e-12, what=f"{key} fx")
                near_rel(v1, d["values"], 1e-12, what=f"{key} values")
                want = np.array(d["grad"])
                if mode == 1:
                    want[2:] = 0.0
                if mode == 2:
                    want[:2] = 0.0
                if mode == 3:
                    want[:] = 0.0
                near_rel(g1, want, 1e-10, what=f"{key} grad")
    # per call (each with a cleared job data cache): the cache's size exchange,
    # then two all-gathers; a failed evaluation stops after the status exchange
    n_ok = sum(1 for _, fail in MAPRECT_CASES if fail < 0)
    want = 4 * (3 * n_ok + 2 * (len(MAPRECT_CASES) - n_ok))
    assert all(rk["collectives"] == want for rk in ranks), [rk["collectives"] for rk in ranks]


_SC = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                       ctypes.POINTER(ctypes.c_double), ctypes.c_void_p)


def _maprect_ex(lib, world, rank, cb, sc, xr, xi, th, mode, fresh, root_only):
    J = xr.shape[0]
    fx = ctypes.c_double()
    grad = np.zeros(2 + J)
    vals = np.zeros(3 * J + 3)
    nv = ctypes.c_int()
    err = ctypes.create_string_buffer(512)
    xrf = np.ascontiguousarray(xr, dtype=np.float64)
    xif = np.ascontiguousarray(xi, dtype=np.int32)
    thf = np.ascontiguousarray(th, dtype=np.float64)
    lib.maprect_hier_ex.restype = ctypes.c_int
    rc = lib.maprect_hier_ex(world, rank, cb, sc, None, J, xrf.ctypes.data_as(ctypes.c_void_p), xr.shape[1],
                             xif.ctypes.data_as(ctypes.c_void_p), thf.ctypes.data_as(ctypes.c_void_p), mode, fresh,
                             root_only, ctypes.byref(fx), grad.ctypes.data_as(ctypes.c_void_p),
                             vals.ctypes.data_as(ctypes.c_void_p), ctypes.byref(nv), err, 512)
    return rc, fx.value, grad, vals[:nv.value], err.value.decode()


def _maprect_cache_rank(rank, world, port, use_hook, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []

    def allgather(send, count, recv, _user):
        t = torch.from_numpy(np.ctypeslib.as_array(send, shape=(count,)).copy())
        parts = [torch.empty(count, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, t)
        np.ctypeslib.as_array(recv, shape=(count * world,))[:] = torch.cat(parts).numpy()
        log.append(("ag", count))

    def scatterv(send, counts, recv, _user):  # point to point from rank 0
        cn = [counts[r] for r in range(world)]
        if rank == 0:
            flat = np.ctypeslib.as_array(send, shape=(sum(cn),)) if sum(cn) else np.zeros(0)
            off = cn[0]
            for r in range(1, world):
                if cn[r]:
                    dist.send(torch.from_numpy(flat[off:off + cn[r]].copy()), dst=r)
                off += cn[r]
            if cn[0]:
                np.ctypeslib.as_array(recv, shape=(cn[0],))[:] = flat[:cn[0]]
        elif cn[rank]:
            t = torch.empty(cn[rank], dtype=torch.float64)
            dist.recv(t, src=0)
            np.ctypeslib.as_array(recv, shape=(cn[rank],))[:] = t.numpy()
        log.append(("sc", cn[rank]))

    cb, sc = _AG(allgather), _SC(scatterv)
    lib = _maprect_lib()
    res = {}
    for J in (7, 16):
        xr, xi, th = gen.maprect_inputs(J)
        for mode in range(4):
            for call in (0, 1):  # the first call fills the cache, the second reuses it
                n0 = len(log)
                got = _maprect_ex(lib, world, rank, cb, sc if use_hook else _SC(), xr, xi, th, mode,
                                  int(call == 0 and mode == 0), 1)
                res[f"{J}_{mode}_{call}"] = dict(rc=got[0], fx=got[1], grad=got[2], vals=got[3], err=got[4],
                                                 log=log[n0:])
    np.save(out + f".{rank}.npy", np.array(res, dtype=object), allow_pickle=True)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,use_hook", [(2, True), (3, True), (3, False)])
def test_map_rect_job_data_cache_gloo(tmp_path, world, use_hook):
    """The per-call_id job data cache (prim/mat/functor/mpi_parallel_call.hpp:
    170-181, 423-450): only rank 0 holds x_r / x_i (the other ranks pass empty
    arrays).  The first call of each call_id exchanges the sizes and scatters
    each rank's block from rank 0 (a scatterv hook, or without one an
    all-gather of the root's buffer); the second call exchanges NO job data --
    only the two result all-gathers -- and both calls equal the one-process
    executor bit for bit."""
    out = str(tmp_path / "mc")
    _spawn(_maprect_cache_rank, world, use_hook, out)
    ranks = [np.load(out + f".{r}.npy", allow_pickle=True).item() for r in range(world)]
    lib = _maprect_lib()
    cb = _AG(lambda *a: None)
    for J in (7, 16):
        xr, xi, th = gen.maprect_inputs(J)
        for mode in range(4):
            rc1, fx1, g1, v1, err1 = _maprect_call(lib, 1, 0, cb, xr, xi, th, mode)
            assert rc1 == 0, err1
            for r in range(world):
                for call in (0, 1):
                    got = ranks[r][f"{J}_{mode}_{call}"]
                    assert got["rc"] == 0, (J, mode, call, r, got["err"])
                    assert got["fx"] == fx1 and np.array_equal(got["grad"], g1) and np.array_equal(got["vals"], v1)
                    kinds = [k for k, _ in got["log"]]
                    if call == 1:
                        assert kinds == ["ag", "ag"], (J, mode, r, got["log"])
                    elif use_hook:
                        assert kinds == ["ag", "sc", "sc", "ag", "ag"], (J, mode, r, got["log"])
                    else:
                        assert kinds == ["ag"] * 5, (J, mode, r, got["log"])


def _maprect_ragged_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(send, count, recv, _user):
        t = torch.from_numpy(np.ctypeslib.as_array(send, shape=(count,)).copy())
        parts = [torch.empty(count, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, t)
        np.ctypeslib.as_array(recv, shape=(count * world,))[:] = torch.cat(parts).numpy()

    cb = _AG(allgather)
    lib = _maprect_lib()
    xr, xi, th = gen.maprect_inputs(7)
    res = {}
    # (a) the first call of a call_id: the checks travel in the cache's size exchange
    lib.maprect_set_ragged(1)
    res["fill"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 1, 1)
    # (b) a cached call_id: they travel in the status exchange
    lib.maprect_set_ragged(0)
    res["good"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 1, 1)
    lib.maprect_set_ragged(1)
    res["cached"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 0, 1)
    # (c) a later good call still agrees (no rank left behind in a collective)
    lib.maprect_set_ragged(0)
    res["after"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 0, 1)
    np.save(out + f".{rank}.npy", np.array(res, dtype=object), allow_pickle=True)
    dist.destroy_process_group()


def test_map_rect_argument_checks_agree_gloo(tmp_path):
    """Rank 0 passes a ragged x_r, rank 1 leaves the job data to the root
    (empty x_r / x_i): both ranks throw rank 0's invalid_argument -- on the
    first call of the call_id (the job data cache's size exchange carries the
    checks) and on a cached one (the status exchange carries them) -- instead
    of rank 1 waiting in a collective rank 0 never reaches; the reference's
    root checks before it dispatches (prim/mat/functor/map_rect.hpp:133-167)."""
    out = str(tmp_path / "rg")
    _spawn(_maprect_ragged_rank, 2, out)
    ranks = [np.load(out + f".{r}.npy", allow_pickle=True).item() for r in range(2)]
    xr, _, _ = gen.maprect_inputs(7)
    n = xr.shape[1]
    msg = (f"map_rect: Size of one of the arrays of the job specific real data ({n - 1}) and size of another "
           f"array of the job specifc real data ({n}) must match in size")
    for r in range(2):
        for key in ("fill", "cached"):
            rc, _, _, _, err = ranks[r][key]
            assert rc == 2 and err == msg, (r, key, rc, err)
        for key in ("good", "after"):
            assert ranks[r][key][0] == 0, (r, key, ranks[r][key][4])
        assert ranks[r]["good"][1] == ranks[r]["after"][1]


def _maprect_jobcount_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(send, count, recv, _user):
        t = torch.from_numpy(np.ctypeslib.as_array(send, shape=(count,)).copy())
        parts = [torch.empty(count, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, t)
        np.ctypeslib.as_array(recv, shape=(count * world,))[:] = torch.cat(parts).numpy()

    cb = _AG(allgather)
    lib = _maprect_lib()
    xr, xi, th = gen.maprect_inputs(7)
    short = (xr[:0], xi[:0], th[:2])  # rank 1 passes no jobs at all
    res = {}
    # (a) the first call of the call_id: the cache's size exchange sees the counts
    res["fill"] = _maprect_ex(lib, world, rank, cb, _SC(), *(short if rank == 1 else (xr, xi, th)), 0, 1, 0)
    # (b) a cached call_id: the status exchange carries it (sized by the cached count on every rank)
    res["good"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 1, 0)
    res["cached"] = _maprect_ex(lib, world, rank, cb, _SC(), *(short if rank == 1 else (xr, xi, th)), 0, 0, 0)
    res["after"] = _maprect_ex(lib, world, rank, cb, _SC(), xr, xi, th, 0, 0, 0)
    np.save(out + f".{rank}.npy", np.array(res, dtype=object), allow_pickle=True)
    dist.destroy_process_group()


def test_map_rect_job_count_mismatch_throws_on_every_rank_gloo(tmp_path):
    """Rank 1 passes J = 0 jobs, rank 0 J = 7: every rank throws the same
    invalid_argument -- on the first call of the call_id and on a cached one --
    instead of rank 1 returning early while rank 0 waits in a collective;
    good calls before and after agree."""
    out = str(tmp_path / "jc")
    _spawn(_maprect_jobcount_rank, 2, out)
    ranks = [np.load(out + f".{r}.npy", allow_pickle=True).item() for r in range(2)]
    for r in range(2):
        rc, _, _, _, err = ranks[r]["fill"]
        assert rc == 2 and err == "map_rect: every rank must pass the same number of jobs", (r, err)
        rc, _, _, _, err = ranks[r]["cached"]
        assert rc == 2 and err.startswith("map_rect: every rank must pass the same number of jobs"), (r, err)
        for key in ("good", "after"):
            assert ranks[r][key][0] == 0, (r, key, ranks[r][key][4])
        assert ranks[r]["good"][1] == ranks[r]["after"][1]


# ---------------------------------------------------------------- product GLM reducers, W = 2
GLMDIST_LIB = os.path.join(ROOT, "tests", "cpp", "_bin", "libglm_dist.so")
_AR = ctypes.CFUNCTYPE(None, ctypes.POINTER(ctypes.c_double), ctypes.c_longlong, ctypes.c_void_p)

# (kind, fixture, bad global row or -1): kind 0 bernoulli (bad y = 2), 1 poisson (bad y = -1)
GLM_DIST_CASES = [(0, "glm_R100000_M256", -1), (1, "poisson_log_glm_R20000_M64", -1),
                  (0, "glm_R100000_M256", 77777), (1, "poisson_log_glm_R20000_M64", 123)]


def _glm_case_block(kind, name, b0, b1):
    d = golden(name)
    R, M = int(d["R"]), int(d["M"])
    if kind == 0:
        x, y = _block(R, M, b0, b1)
        th = gen.glm_inputs(1, M)[2]
    else:
        xf, yf, th = gen.glm2_inputs(R, M, "poisson")
        x, y = xf[b0:b1], yf[b0:b1]
    return R, M, np.asfortranarray(x), np.ascontiguousarray(y, dtype=np.int32), f64(th)


def _glm_dist_rank(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []

    def allgather(send, count, recv, _user):  # unused by the reducers
        raise RuntimeError("allgather called")

    def allreduce(buf, count, _user):
        a = np.ctypeslib.as_array(buf, shape=(count,))
        t = torch.from_numpy(a.copy())
        dist.all_reduce(t)
        a[:] = t.numpy()
        calls.append(count)

    ag, ar = _AG(allgather), _AR(allreduce)
    lib = ctypes.CDLL(prebuilt(GLMDIST_LIB))
    lib.glm_dist_eval.restype = ctypes.c_int
    res = {}
    for kind, name, bad in GLM_DIST_CASES:
        R = int(golden(name)["R"])
        b0, b1 = _partition(R, world, rank, lib)
        R, M, x, y, th = _glm_case_block(kind, name, b0, b1)
        if b0 <= bad < b1:
            y[bad - b0] = 2 if kind == 0 else -1
        fx = ctypes.c_double()
        g = np.zeros(M + 1)
        err = ctypes.create_string_buffer(512)
        rc = lib.glm_dist_eval(world, rank, ag, ar, None, kind, ctypes.c_longlong(R), ctypes.c_longlong(b0),
                               ctypes.c_longlong(b1 - b0), M, x.ctypes.data_as(ctypes.c_void_p),
                               y.ctypes.data_as(ctypes.c_void_p), th.ctypes.data_as(ctypes.c_void_p),
                               ctypes.byref(fx), g.ctypes.data_as(ctypes.c_void_p), err, 512)
        res[f"{kind}_{bad}"] = dict(rc=rc, fx=fx.value, g=g, err=err.value.decode(), own=b0 <= bad < b1)
    res["allreduce_counts"] = calls
    np.save(out + f".{rank}.npy", np.array(res, dtype=object), allow_pickle=True)
    dist.destroy_process_group()


@pytest.mark.gpu
def test_glm_reducers_two_ranks_product_path(tmp_path):
    """The product's row-sharded reducers (reduce_sum_bernoulli_logit_glm,
    poisson_log_glm_lpmf on a glm_shard) in W = 2 processes sharing the GPU,
    joined by a gloo all-reduce hook (amd::set_host_collective): each rank's
    row block on the device, ONE all-reduce of [logp, alpha', beta' | y flag]
    per call.  Both ranks return the reference's single-call result
    (glm_R100000_M256 / poisson_log_glm_R20000_M64, real Stan Math) within
    1e-12 / 1e-10, bitwise equal to each other; an out-of-support y on one
    rank makes BOTH ranks throw domain_error (the owner with the reference's
    message and the global index)."""
    out = str(tmp_path / "gd")
    _spawn(_glm_dist_rank, 2, out)
    ranks = [np.load(out + f".{r}.npy", allow_pickle=True).item() for r in range(2)]
    for kind, name, bad in GLM_DIST_CASES:
        key = f"{kind}_{bad}"
        r0, r1 = ranks[0][key], ranks[1][key]
        if bad < 0:
            assert r0["rc"] == 0 and r1["rc"] == 0, (key, r0["err"], r1["err"])
            assert r0["fx"] == r1["fx"] and np.array_equal(r0["g"], r1["g"]), key
            d = golden(name)
            near_rel(r0["fx"], d["fx"], 1e-12, what=f"{key} fx")
            near_rel(r0["g"], d["grad"], 1e-10, what=f"{key} grad")
        else:
            assert r0["rc"] == 1 and r1["rc"] == 1, (key, r0, r1)
            owner = r0 if r0["own"] else r1
            fn = "bernoulli_logit_glm_lpmf" if kind == 0 else "poisson_log_glm_lpmf"
            want = (f"{fn}: Vector of dependent variables[{bad + 1}] is 2, but must be in the interval [0, 1]"
                    if kind == 0 else f"{fn}: Vector of dependent variables[{bad + 1}] is -1, but must be >= 0!")
            assert owner["err"] == want, owner["err"]
    # one all-reduce per call on every rank (M + 3 bernoulli, M + 4 poisson)
    for rk in ranks:
        assert rk["allreduce_counts"] == [259, 68, 259, 68], rk["allreduce_counts"]
