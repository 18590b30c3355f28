"""Row sharding of the GLM reducer on CPU, world_size 2, gloo.

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
from _util import ROOT, f64, golden, near_rel, oracle, ptr

GOLDEN_INC = 0x9E3779B97F4A7C15
BENCH_LIB = os.path.join(ROOT, "math_amd", "lib", "libsmg_bench.so")


def _partition(R, world, rank):
    lib = ctypes.CDLL(BENCH_LIB)
    b0, b1 = ctypes.c_longlong(), ctypes.c_longlong()
    lib.smg_bench_row_partition(ctypes.c_longlong(R), world, rank, ctypes.byref(b0), ctypes.byref(b1))
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
    mp.start_processes(_rank_main, args=(2, _free_port(), R, M, out), nprocs=2, join=True,
                       start_method="spawn")
    res = np.load(out)
    near_rel(res[0], d["fx"], 1e-12, what="fx")
    near_rel(res[1:], d["grad"], 1e-10, what="grad")
