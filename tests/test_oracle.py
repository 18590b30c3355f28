"""Pin the CPU restatement (oracle/cpu_ref.cpp) against golden vectors that the
real reference produced (oracle/ref_harness.cpp -> tests/golden/).  CPU only.

Tolerances: values and gradients 1e-10 relative (expect_near_rel semantics)
unless a case states otherwise; the restatement uses the same algorithms as
the reference, so differences are round-off only.
"""
import glob
import math
import os

import numpy as np
import pytest

import gen
from _util import GOLDEN, f64, golden, near_rel, oracle, ptr

RTOL = 1e-10


def test_generator_matches_harness():
    # glm_R1000_M8 inputs are regenerated from seeds; value pins the generator
    d = golden("glm_R1000_M8")
    x, y, th = gen.glm_inputs(1000, 8)
    ga = np.zeros(1)
    gb = np.zeros(8)
    lp = oracle().oracle_glm(ptr(y), ptr(f64(x.ravel(order="F"))), 1000, 8, th[0], ptr(f64(th[1:])), ptr(ga), ptr(gb))
    near_rel(lp, d["fx"], 1e-13, what="glm fx")
    near_rel(np.concatenate([ga, gb]), d["grad"], RTOL, what="glm grad")


@pytest.mark.parametrize("name", ["glm_R10000_M256", "glm_R100000_M256"])
def test_oracle_glm(name):
    d = golden(name)
    R, M = int(d["R"]), int(d["M"])
    x, y, th = gen.glm_inputs(R, M)
    ga, gb = np.zeros(1), np.zeros(M)
    lp = oracle().oracle_glm(ptr(y), ptr(f64(x.ravel(order="F"))), R, M, th[0], ptr(f64(th[1:])), ptr(ga), ptr(gb))
    near_rel(lp, d["fx"], 1e-12, what="fx")
    near_rel(np.concatenate([ga, gb]), d["grad"], RTOL, what="grad")
    if "fx_map_rect32" in d:  # map_rect over 32 shards == single call
        near_rel(d["fx_map_rect32"], d["fx"], 1e-12, what="map_rect fx")
        near_rel(d["grad_map_rect32"], d["grad"], RTOL, what="map_rect grad")


def test_oracle_glm_extreme():
    d = golden("glm_extreme")
    R, M = int(d["R"]), int(d["M"])
    x = f64(d["x"])
    y = np.array(d["y"], dtype=np.int32)
    th = d["theta"]
    ga, gb = np.zeros(1), np.zeros(M)
    lp = oracle().oracle_glm(ptr(y), ptr(x), R, M, th[0], ptr(f64(th[1:])), ptr(ga), ptr(gb))
    near_rel(lp, d["fx"], 1e-12, what="fx")
    near_rel(np.concatenate([ga, gb]), d["grad"], RTOL, what="grad")


@pytest.mark.parametrize("N", [16, 64, 256, 1024])
def test_oracle_gp(N):
    d = golden(f"gp_N{N}")
    fx = np.zeros(1)
    g = np.zeros(3)
    oracle().oracle_gp_marginal(ptr(f64(d["x"])), ptr(f64(d["y"])), N, ptr(f64(d["theta"])), ptr(fx), ptr(g))
    near_rel(fx, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, what="grad")


@pytest.mark.parametrize("N", [8, 40, 128])
def test_oracle_mulchol(N):
    d = golden(f"mulchol_N{N}")
    A = f64(gen.mulchol_input(N))
    fx = np.zeros(1)
    g = np.zeros(N * N)
    oracle().oracle_mulchol(ptr(A), N, ptr(fx), ptr(g))
    near_rel(fx, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, atol=RTOL * np.abs(d["grad"]).max(), what="grad")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "cholesky_N*.json"))))
def test_oracle_cholesky(path):
    d = golden(os.path.basename(path)[:-5])
    N = int(d["N"])
    A = f64(d["A"])
    L = np.zeros(N * N)
    assert oracle().oracle_cholesky(ptr(A), N, ptr(L)) == 0
    near_rel(L, d["L"], 1e-12, what="L")
    W = d["W"].reshape(N, N).T  # W[(j*N)+i] -> (i, j)
    Ladj = np.tril(W).ravel(order="F").copy()
    Aadj = np.zeros(N * N)
    oracle().oracle_cholesky_rev(ptr(f64(d["L"])), ptr(Ladj), N, ptr(Aadj))
    near_rel(Aadj, d["grad_A"], RTOL, atol=RTOL * np.abs(d["grad_A"]).max(), what="grad_A")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "mvn_cholesky_N*.json"))))
def test_oracle_mvn(path):
    d = golden(os.path.basename(path)[:-5])
    N = int(d["N"])
    lp = np.zeros(1)
    gy, gm, gL = np.zeros(N), np.zeros(N), np.zeros(N * N)
    oracle().oracle_mvn_cholesky(ptr(f64(d["y"])), ptr(f64(d["mu"])), ptr(f64(d["L"])), N, ptr(lp), ptr(gy), ptr(gm), ptr(gL))
    near_rel(lp, d["fx"], 1e-12, what="lp")
    near_rel(gy, d["grad_y"], RTOL, what="gy")
    near_rel(gm, d["grad_mu"], RTOL, what="gmu")
    near_rel(gL, d["grad_L"], RTOL, atol=RTOL * np.abs(d["grad_L"]).max(), what="gL")


def test_oracle_mvn_known_answer():
    d = golden("mvn_cholesky_known")
    S = d["Sigma"].reshape(3, 3)
    L = np.linalg.cholesky(S)
    lp = np.zeros(1)
    oracle().oracle_mvn_cholesky(ptr(f64(d["y"])), ptr(f64(d["mu"])), ptr(f64(L.ravel(order="F"))), 3, ptr(lp), None, None, None)
    assert abs(lp[0] - d["expected"]) < 1e-5  # EXPECT_FLOAT_EQ in the reference


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "multiply_*.json"))))
def test_oracle_multiply(path):
    d = golden(os.path.basename(path)[:-5])
    m, k, n, kind = (int(d[s]) for s in ("m", "k", "n", "kind"))
    C = np.zeros(m * n)
    oracle().oracle_multiply(ptr(f64(d["A"])), ptr(f64(d["B"])), m, k, n, ptr(C))
    near_rel(C, d["C"], 1e-12, atol=1e-14, what="C")
    Ag, Bg = np.zeros(m * k), np.zeros(k * n)
    oracle().oracle_multiply_rev(ptr(f64(d["A"])), ptr(f64(d["B"])), ptr(f64(d["W"])), m, k, n, ptr(Ag), ptr(Bg))
    if kind != 2:
        near_rel(Ag, d["grad_A"], RTOL, atol=1e-13, what="gA")
    if kind != 1:
        near_rel(Bg, d["grad_B"], RTOL, atol=1e-13, what="gB")


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "mdivide_left_tri_*.json"))))
def test_oracle_mdivide(path):
    d = golden(os.path.basename(path)[:-5])
    m, n, lower, kind = (int(d[s]) for s in ("m", "n", "lower", "kind"))
    C = np.zeros(m * n)
    oracle().oracle_mdivide_left_tri(lower, ptr(f64(d["A"])), ptr(f64(d["B"])), m, n, ptr(C))
    near_rel(C, d["C"], 1e-12, atol=1e-13, what="C")
    Ag, Bg = np.zeros(m * m), np.zeros(m * n)
    oracle().oracle_mdivide_left_tri_rev(lower, ptr(f64(d["A"])), ptr(C), ptr(f64(d["W"])), m, n, ptr(Ag), ptr(Bg))
    if kind != 1:
        near_rel(Ag, d["grad_A"], RTOL, atol=1e-12, what="gA")
    if kind != 2:
        near_rel(Bg, d["grad_B"], RTOL, atol=1e-12, what="gB")


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_oracle_lse(kind):
    d = golden(f"log_sum_exp_{kind}")
    x = f64(d["x"])
    n = len(x)
    lse = oracle().oracle_log_sum_exp(ptr(x), n)
    near_rel(lse, d["fx"], 1e-14, what="lse")
    g = np.zeros(n)
    oracle().oracle_log_sum_exp_rev(ptr(x), n, lse, 1.0, ptr(g))
    near_rel(g, d["grad"], 1e-12, atol=1e-15, what="grad")


def test_oracle_special():
    d = golden("special")
    o = oracle()
    xs = d["x"]
    lg = [o.oracle_lgamma(x) for x in xs]
    dg = [o.oracle_digamma(x) for x in xs]
    tg = [o.oracle_trigamma(x) for x in xs]
    near_rel(lg, d["lgamma"], 1e-15, atol=1e-15, what="lgamma")  # same libm
    near_rel(dg, d["digamma"], 1e-14, atol=1e-14, what="digamma")
    near_rel(tg, d["trigamma"], 1e-14, what="trigamma")
    near_rel(dg, d["grad_lgamma"], 1e-14, atol=1e-14, what="d lgamma")
    near_rel(tg, d["grad_digamma"], 1e-14, what="d digamma")


def test_oracle_normal():
    o = oracle()
    d = golden("normal_N1024")
    th = f64(d["theta"])
    zero, one = f64([0.0]), f64([1.0])
    g = np.zeros(1024)
    lp = o.oracle_normal_lpdf(ptr(th), 1, ptr(zero), 0, ptr(one), 0, 1024, ptr(g), None, None)
    near_rel(lp, d["fx"], 1e-13, what="fx")
    near_rel(g, d["grad"], 1e-14, what="grad")
    d = golden("normal_vec9")
    gy, gm, gs = np.zeros(9), np.zeros(9), np.zeros(9)
    lp = o.oracle_normal_lpdf(ptr(f64(d["y"])), 1, ptr(f64(d["mu"])), 1, ptr(f64(d["sigma"])), 1, 9, ptr(gy), ptr(gm), ptr(gs))
    near_rel(lp, d["fx"], 1e-13, what="fx")
    near_rel(gy, d["grad_y"], 1e-13, what="gy")
    near_rel(gm, d["grad_mu"], 1e-13, what="gmu")
    near_rel(gs, d["grad_sigma"], 1e-13, what="gsigma")
    d = golden("normal_known")
    for y, m, s, e in zip(d["y"], d["mu"], d["sigma"], d["expected"]):
        lp = o.oracle_normal_lpdf(ptr(f64([y])), 0, ptr(f64([m])), 0, ptr(f64([s])), 0, 1, None, None, None)
        assert abs(lp - e) < 1e-8  # test_fixture_distr.hpp:120


def test_oracle_gp_cov_rev_matches_chain():
    """gp cov rev restatement vs finite differences at tight step (sanity)."""
    o = oracle()
    n = 12
    x = gen.unif(7, n, -3, 3)
    W = gen.unif(8, n * n, -1, 1)
    K = np.zeros(n * n)
    ga, gl = np.zeros(1), np.zeros(1)
    o.oracle_gp_cov_rev(ptr(x), n, 1.3, 0.7, ptr(W), ptr(ga), ptr(gl))

    def f(s, l):
        o.oracle_gp_cov(ptr(x), n, s, l, ptr(K))
        return float(W @ K)

    h = 1e-6
    fd_s = (f(1.3 + h, 0.7) - f(1.3 - h, 0.7)) / (2 * h)
    fd_l = (f(1.3, 0.7 + h) - f(1.3, 0.7 - h)) / (2 * h)
    assert abs(ga[0] - fd_s) < 1e-6 * max(1, abs(fd_s))
    assert abs(gl[0] - fd_l) < 1e-6 * max(1, abs(fd_l))
