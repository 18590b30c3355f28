"""Shared test helpers: golden fixtures, tolerance checks, oracle bindings.

The oracle (oracle/_build/libsmg_oracle.so) is the CPU restatement of the
reference: it is imported ONLY here, in tests, as the checker.
"""
import ctypes
import json
import math
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def golden(name: str) -> dict:
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        d = json.load(f)

    def conv(v):
        if isinstance(v, list):
            return np.array([conv(e) for e in v], dtype=np.float64) if v and not isinstance(v[0], list) else v
        if v == "nan":
            return math.nan
        if v == "inf":
            return math.inf
        if v == "-inf":
            return -math.inf
        return v

    return {k: conv(v) for k, v in d.items()}


def near_rel(actual, expected, rtol, atol=None, what=""):
    """expect_near_rel semantics (test/unit/math/expect_near_rel.hpp:33-52):
    each entry passes when its relative error 2|a-b|/(|a|+|b|) <= rtol or its
    absolute error |a-b| <= atol (atol defaults to rtol, the reference's
    absolute fallback near zero; callers pass a norm-scaled atol for matrices
    whose small entries carry cancellation).  NaN/inf must match exactly."""
    a = np.asarray(actual, dtype=np.float64).ravel()
    b = np.asarray(expected, dtype=np.float64).ravel()
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    atol = rtol if atol is None else atol
    fin = np.isfinite(a) & np.isfinite(b)
    same_nonfinite = (np.isnan(a) & np.isnan(b)) | (a == b)
    assert np.all(fin | same_nonfinite), f"{what}: non-finite mismatch at {np.where(~(fin | same_nonfinite))[0][:5]}"
    a, b = a[fin], b[fin]
    small = (np.abs(a) < atol) | (np.abs(b) < atol)
    absdiff = np.abs(a - b)
    rel = absdiff / np.maximum(0.5 * (np.abs(a) + np.abs(b)), 1e-300)
    bad = (absdiff > atol) & (rel > rtol)
    if np.any(bad):
        i = np.where(bad)[0][0]
        raise AssertionError(
            f"{what}: {bad.sum()} / {bad.size} entries off; first at {i}: "
            f"{a[i]!r} vs {b[i]!r} (rel {rel[i]:.3e}, abs {absdiff[i]:.3e}, rtol {rtol}, atol {atol})")
    return float(rel[~small].max()) if np.any(~small) else 0.0


# --------------------------------------------------------------- prebuilt binaries
def prebuilt(path):
    """path, after checking that the binary was built from the tree's sources
    (math_amd/srchash.py): the GPU box runs these container-built binaries and
    cannot rebuild them (no /root/reference there for Eigen)."""
    import sys
    sys.path.insert(0, ROOT)
    from math_amd import srchash
    name = os.path.basename(path)
    if name == "libsmg_bench.so":
        group = "bench"
    elif name.startswith("ref_harness"):
        group = "ref"
    else:
        group = "cpp:" + (name[3:-3] if name.startswith("lib") and name.endswith(".so") else name)
    srchash.check(path, group)
    return path


# --------------------------------------------------------------- oracle
_ORACLE = None
_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)


def ptr(a):
    if a is None:
        return None
    if a.dtype == np.int32:
        return a.ctypes.data_as(_I)
    return a.ctypes.data_as(_D)


def oracle():
    global _ORACLE
    if _ORACLE is None:
        path = os.path.join(ROOT, "oracle", "_build", "libsmg_oracle.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "cpu"])
        lib = ctypes.CDLL(path)
        dd = ctypes.c_double
        ii = ctypes.c_int
        sig = {
            "oracle_gp_cov": (None, [_D, ii, dd, dd, _D]),
            "oracle_gp_cov_rev": (None, [_D, ii, dd, dd, _D, _D, _D]),
            "oracle_cholesky": (ii, [_D, ii, _D]),
            "oracle_cholesky_rev": (None, [_D, _D, ii, _D]),
            "oracle_mvn_cholesky": (None, [_D, _D, _D, ii, _D, _D, _D, _D]),
            "oracle_multiply": (None, [_D, _D, ii, ii, ii, _D]),
            "oracle_multiply_rev": (None, [_D, _D, _D, ii, ii, ii, _D, _D]),
            "oracle_mdivide_left_tri": (None, [ii, _D, _D, ii, ii, _D]),
            "oracle_mdivide_left_tri_rev": (None, [ii, _D, _D, _D, ii, ii, _D, _D]),
            "oracle_log_sum_exp": (dd, [_D, ii]),
            "oracle_log_sum_exp_rev": (None, [_D, ii, dd, dd, _D]),
            "oracle_lgamma": (dd, [dd]),
            "oracle_digamma": (dd, [dd]),
            "oracle_trigamma": (dd, [dd]),
            "oracle_normal_lpdf": (dd, [_D, ii, _D, ii, _D, ii, ii, _D, _D, _D]),
            "oracle_glm": (dd, [_I, _D, ctypes.c_longlong, ii, dd, _D, _D, _D]),
            "oracle_normal_id_glm": (dd, [_D, _D, ctypes.c_longlong, ii, dd, _D, dd, _D]),
            "oracle_poisson_log_glm": (dd, [_I, _D, ctypes.c_longlong, ii, dd, _D, _D]),
            "oracle_categorical_logit_glm": (dd, [_I, _D, ctypes.c_longlong, ii, ii, _D, _D, _D]),
            "oracle_gp_marginal": (None, [_D, _D, ii, _D, _D, _D]),
            "oracle_mdivide_left_spd": (ii, [_D, _D, ii, ii, _D, _D, _D, _D]),
            "oracle_log_determinant_spd": (ii, [_D, ii, _D, _D]),
            "oracle_mlt_self_transpose": (None, [_D, ii, ii, _D, _D, _D]),
            "oracle_quad_form_sym": (None, [_D, _D, ii, ii, _D, ii, _D, _D, _D]),
            "oracle_mulchol": (None, [_D, ii, _D, _D]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _ORACLE = lib
    return _ORACLE


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def glm2_oracle(kind, x, y, th, M):
    """(logp, gradient) of the restated normal_id / poisson_log GLM."""
    R = len(y)
    g = np.zeros(M + 2 if kind == "normal" else M + 1)
    xf = f64(x.ravel(order="F"))
    if kind == "normal":
        lp = oracle().oracle_normal_id_glm(ptr(f64(y)), ptr(xf), R, M, th[0], ptr(f64(th[1:M + 1])), th[M + 1], ptr(g))
    else:
        lp = oracle().oracle_poisson_log_glm(ptr(np.ascontiguousarray(y, dtype=np.int32)), ptr(xf), R, M, th[0],
                                             ptr(f64(th[1:])), ptr(g))
    return lp, g


def glm_cat_oracle(x, y, th, M, C):
    """(logp, [alpha'(C), beta'(M x C col-major)]) of the restated categorical GLM."""
    R = len(y)
    g = np.zeros(C + M * C)
    xf = f64(x.ravel(order="F"))
    lp = oracle().oracle_categorical_logit_glm(ptr(np.ascontiguousarray(y, dtype=np.int32)), ptr(xf), R, M, C,
                                               ptr(f64(th[:C])), ptr(f64(th[C:])), ptr(g))
    return lp, g


def spd_oracle(kind, args, n, k, sym=1):
    """(f, gradient over every argument entry, col-major, concatenated) of the
    restated SURVEY 8(f) row-3 functor `kind` (gen.spd_inputs order)."""
    fx = np.zeros(1)
    F = lambda a: np.ascontiguousarray(np.asarray(a, dtype=np.float64).ravel(order="F"))  # noqa: E731
    if kind == 0:
        A, B, W = args
        gA, gB = np.zeros(n * n), np.zeros(n * k)
        assert oracle().oracle_mdivide_left_spd(ptr(F(A)), ptr(F(B)), n, k, ptr(F(W)), ptr(fx), ptr(gA), ptr(gB)) == 0
        return fx[0], np.concatenate([gA, gB])
    if kind == 1:
        (A,) = args
        gA = np.zeros(n * n)
        assert oracle().oracle_log_determinant_spd(ptr(F(A)), n, ptr(fx), ptr(gA)) == 0
        return fx[0], gA
    if kind == 2:
        L, W = args
        gL = np.zeros(n * k)
        oracle().oracle_mlt_self_transpose(ptr(F(L)), n, k, ptr(F(W)), ptr(fx), ptr(gL))
        return fx[0], gL
    A, B, W = args
    gA, gB = np.zeros(n * n), np.zeros(n * k)
    oracle().oracle_quad_form_sym(ptr(F(A)), ptr(F(B)), n, k, ptr(F(W)), sym, ptr(fx), ptr(gA), ptr(gB))
    return fx[0], np.concatenate([gA, gB])


def check_against_fixture(d, fx, g, rtol, what=""):
    """fx and the gradient (full, or its sum / L2 / sampled entries)."""
    near_rel(fx, d["fx"], 1e-12, what=what + " fx")
    if "grad" in d:
        near_rel(g, d["grad"], rtol, what=what + " grad")
    else:
        idx = np.array(d["sample_index"], dtype=np.int64)
        near_rel(g[idx], d["sample_grad"], rtol, what=what + " sampled grad")
    near_rel(np.sum(g), d["grad_sum"], 1e-9, atol=1e-9 * np.abs(g).sum(), what=what + " grad sum")
    near_rel(np.linalg.norm(g), d["grad_l2"], 1e-11, what=what + " grad l2")
