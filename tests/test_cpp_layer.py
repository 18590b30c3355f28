"""The header-only C++ stan::math layer (math_amd/include) driven end to end.

CPU part: the C++ test programs build and the C-ABI library exports every
symbol include/smg_hip.h declares.  GPU part: the programs run the GP
gradient through stan::math::gradient (device tape) and are compared with the
reference's golden values at 1e-10 relative (expect_near_rel semantics).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from _util import ROOT, golden, near_rel, prebuilt

BIN = os.path.join(ROOT, "tests", "cpp", "_bin")
LIB = os.path.join(ROOT, "math_amd", "lib", "libsmg_hip.so")


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "smg_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(smg_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build() must produce math_amd/lib/libsmg_hip.so"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (smg_[a-z0-9_]+)", out))
    missing = [s for s in _declared_symbols() if s not in exported]
    assert not missing, f"declared but not exported: {missing}"


def test_python_binding_covers_header():
    from math_amd import hip
    missing = [s for s in _declared_symbols() if s not in hip.exported_symbols()]
    assert not missing, missing


def test_prebuilt_binaries_match_sources():
    """Every prebuilt binary the GPU box runs but cannot rebuild carries the
    hash of the sources it was built from (math_amd/srchash.py), equal to the
    tree's: libsmg_bench.so, tests/cpp/_bin/*, oracle/_ref/*."""
    import glob
    bins = [os.path.join(ROOT, "math_amd", "lib", "libsmg_bench.so")] + sorted(glob.glob(os.path.join(BIN, "*")))
    bins += sorted(glob.glob(os.path.join(ROOT, "oracle", "_ref", "ref_harness*")))
    assert len(bins) >= 6
    for b in bins:
        prebuilt(b)


def test_stream_panel_bounds_tile_the_columns():
    """smg_cholesky_stream_panel_cols (host-only, no GPU): the streamed
    factor's panels are contiguous, at most 512 columns wide, and tile
    [0, n) -- the bounds the Eigen boundary's cholesky_decompose builds each
    panel's host varis from (one definition with the device side)."""
    import ctypes
    from math_amd import hip
    lib = hip.lib()
    j0, j1 = ctypes.c_int(), ctypes.c_int()
    for n in (1, 65, 511, 512, 513, 1536, 4096, 4100):
        npan = lib.smg_cholesky_stream_panels(n)
        end = 0
        for p in range(npan):
            assert lib.smg_cholesky_stream_panel_cols(n, p, ctypes.byref(j0), ctypes.byref(j1)) == 0
            assert j0.value == end and 0 < j1.value - j0.value <= 512
            end = j1.value
        assert end == n
        assert lib.smg_cholesky_stream_panel_cols(n, npan, ctypes.byref(j0), ctypes.byref(j1)) != 0


def test_sweep_bridges_linear_in_tape_length():
    """The reverse sweep with materialised host blocks (CPU, no device call):
    each block's bridge learns whether a later node touched its varis from the
    sweep's touch log (grad.hpp log_host_touches), not a rescan of the rest of
    the tape -- exactly the touched block is stamped, and the sweep's time
    grows linearly with bridges x tape (1,000 -> 4,000 bridges: < 8x, a
    rescan is ~16x)."""
    def run(B):
        out = _run("test_tape_cpu", "", args=("check", str(B)))
        b, tape, sec, touched, xadj, gel = out.split()
        assert int(touched) == 1 and float(gel) == 2.0
        return int(tape), float(sec)
    run(100)  # warm
    t1 = min(run(1000)[1] for _ in range(3))
    tape4, t4 = min((run(4000) for _ in range(3)), key=lambda r: r[1])
    assert tape4 > 4 * 4000
    assert t4 < 8 * t1 + 2e-3, (t1, t4)


def test_cpp_programs_built():
    for name in ("test_gp_tape", "test_functors", "test_tape_cpu"):
        assert os.path.exists(os.path.join(BIN, name)), f"{name} not built (run __graft_entry__.build())"


def _run(name, stdin, args=(), env=None):
    e = None if env is None else {**os.environ, **env}
    p = subprocess.run([prebuilt(os.path.join(BIN, name)), *args], input=stdin, capture_output=True, text=True, timeout=300,
                       env=e)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout


def _gp_stdin(d):
    N = len(d["x"])
    stdin = f"{N} " + " ".join(repr(float(v)) for v in d["theta"]) + "\n"
    return stdin + " ".join(repr(float(v)) for v in d["x"]) + "\n" + " ".join(repr(float(v)) for v in d["y"]) + "\n"


def _gp_rows(out):
    return np.array([[float(v) for v in l.split()] for l in out.strip().splitlines()[:3]])


@pytest.mark.gpu
@pytest.mark.parametrize("N", [16, 256, 1024, 4096])
def test_gp_gradient_through_tape(N):
    d = golden(f"gp_N{N}")
    lines = [l.split() for l in _run("test_gp_tape", _gp_stdin(d)).strip().splitlines()]
    for row in lines[:3]:  # std::vector twice (re-use of recovered arenas) + Eigen::VectorXd
        vals = np.array([float(v) for v in row])
        near_rel(vals[0], d["fx"], 1e-12, what="fx")
        near_rel(vals[1:], d["grad"], 1e-10, what="grad")
    assert lines[3] == ["stack", "0", "0"]  # nested tape fully recovered


@pytest.mark.gpu
@pytest.mark.parametrize("split_b", ["1", "0"])
@pytest.mark.parametrize("N", [1024, 4096])
def test_gp_gradient_fused_lookahead(N, split_b):
    """The opt-in look-ahead inside the next panel's launch (SMG_FUSED_A=1:
    the diagonal block's tiles and the rows below column block by column
    block, published per tile; the resident rows load each block at its
    step), with the trailing update split or whole: the reference's golden
    gradient at 1e-10, three evaluations each."""
    d = golden(f"gp_N{N}")
    lines = [l.split() for l in _run("test_gp_tape", _gp_stdin(d),
                                     env={"SMG_FUSED_A": "1", "SMG_SPLIT_B": split_b}).strip().splitlines()]
    for row in lines[:3]:
        vals = np.array([float(v) for v in row])
        near_rel(vals[0], d["fx"], 1e-12, what="fx")
        near_rel(vals[1:], d["grad"], 1e-10, what="grad")
    assert lines[3] == ["stack", "0", "0"]


@pytest.mark.gpu
@pytest.mark.parametrize("N", [64, 1024])
def test_gp_cholesky_reverse_closed_form_vs_murray(N):
    """The GP's factor has one consumer, the MVN: cholesky_decompose's reverse
    takes the closed form adj Phi(s s^T - K^{-1}) (smg_cholesky_mvn_rev; N = 64
    the blocked-solve inverse, N = 1024 the doubling from the 512-row block
    inverses); SMG_CHOL_MVN_CLOSED_FORM=0 forces the dense adjoint + Murray's
    reverse.  Both match the reference's golden gradient at 1e-10 and each
    other at 1e-11."""
    d = golden(f"gp_N{N}")
    a = _gp_rows(_run("test_gp_tape", _gp_stdin(d)))
    b = _gp_rows(_run("test_gp_tape", _gp_stdin(d), env={"SMG_CHOL_MVN_CLOSED_FORM": "0"}))
    for r in (a, b):
        near_rel(r[:, 1:], np.tile(d["grad"], (3, 1)), 1e-10, what="grad")
    near_rel(a, b, 1e-11, what="closed form vs Murray")


@pytest.mark.gpu
@pytest.mark.parametrize("N", [64, 1024])
def test_gp_cholesky_second_consumer_takes_dense_path(N):
    """lp + 1e-3 sum(L): the factor's adjoint is no longer the MVN's alone, so
    the deposited MVN partials are expanded into the dense adjoint and Murray's
    reverse runs on the sum -- equal to the run that never deposits."""
    d = golden(f"gp_N{N}")
    a = _gp_rows(_run("test_gp_tape", _gp_stdin(d), args=("mixed",)))
    b = _gp_rows(_run("test_gp_tape", _gp_stdin(d), args=("mixed",), env={"SMG_CHOL_MVN_CLOSED_FORM": "0"}))
    near_rel(a, b, 1e-12, what="mixed consumers")
    assert abs(a[0, 0] - d["fx"]) > 1e-9  # the extra term is really there
