"""The drop-in boundary's overload sets, on the device.

tests/cpp/boundary_cases.hpp holds the reference's call forms once; the
reference harness compiled it against Stan Math 3.0.0 to write
tests/golden/boundary_forms.json / boundary_errors.json / gp_nd_D3_N*.json,
and tests/cpp/test_boundary.cpp compiles the SAME source against math_amd
(the compile probe, built by __graft_entry__.build()).  Values at 1e-12
relative, gradients at 1e-10 (expect_near_rel semantics), error messages
character for character.
"""
import os
import subprocess

import numpy as np
import pytest

from _util import ROOT, golden, near_rel, prebuilt

BIN = os.path.join(ROOT, "tests", "cpp", "_bin", "test_boundary")
RTOL = 1e-10


def _run(stdin, timeout=600, env=None):
    e = None if env is None else {**os.environ, **env}
    p = subprocess.run([prebuilt(BIN)], input=stdin, capture_output=True, text=True, timeout=timeout, env=e)
    assert p.returncode == 0, p.stderr[-3000:]
    return p.stdout


def _num(vals):
    return " ".join(repr(float(v)) for v in np.ravel(vals))


def _parse(out):
    res = {}
    for line in out.strip().splitlines():
        tag, *vals = line.split()
        res[tag] = np.array([float(v) for v in vals])
    return res


EIGEN = "/root/reference/lib/eigen_3.3.3"


@pytest.mark.skipif(not os.path.isdir(EIGEN), reason="Eigen (vendored with the reference) not present")
def test_compile_probe():
    """Every reference call form of boundary_cases.hpp compiles against
    math_amd/include (a missing or ambiguous overload fails here)."""
    src = os.path.join(ROOT, "tests", "cpp", "test_boundary.cpp")
    p = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I" + os.path.join(ROOT, "math_amd", "include"),
                        "-I" + os.path.join(ROOT, "include"), "-isystem", EIGEN, src],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-4000:]


@pytest.mark.gpu
def test_boundary_forms():
    d = golden("boundary_forms")
    inp = [int(d["m"]), int(d["k"]), int(d["n"]), int(d["s"]), int(d["nobs"])]
    stdin = "forms " + " ".join(map(str, inp)) + " " + " ".join(
        _num(d[k]) for k in ("A", "B", "v", "r", "r5", "S", "d", "L", "ys", "mu", "W")) + " " + repr(d["c"]) + "\n"
    res = _parse(_run(stdin))
    names = sorted(k[:-3] for k in d if k.endswith("_fx"))
    assert len(names) >= 28, names
    for name in names:
        got = res[name]
        near_rel(got[0], d[name + "_fx"], 1e-12, what=name + " f")
        want = np.atleast_1d(d[name + "_grad"]) if len(np.atleast_1d(d[name + "_grad"])) else np.zeros(0)
        near_rel(got[1:], want, RTOL, what=name + " grad")
    assert list(res["stack"]) == [0.0, 0.0]  # every case recovered its tape and host blocks


@pytest.mark.gpu
def test_boundary_errors():
    want = golden("boundary_errors")
    out = _run("errors\n")
    got = {}
    for line in out.strip().splitlines():
        tag, _, rest = line.partition(" ")
        got[tag] = rest
    for k, v in want.items():
        assert got.get(k) == v, (k, got.get(k), v)


@pytest.mark.gpu
@pytest.mark.parametrize("N", [64, 256])
@pytest.mark.parametrize("form", [0, 1, 2])
def test_gp_nd_codegen_shape(N, form):
    """The Stan-codegen-shaped GP marginal (Eigen::Matrix<var> K, Kd, L) with
    D = 3 inputs: (var, var), (double, var) and 5 observations with a var
    mean, against the reference's gradient()."""
    d = golden(f"gp_nd_D3_N{N}")
    th = d[f"theta_f{form}"]
    stdin = (f"gp_nd {N} 3 5 {_num(d['x'])} {_num(d['ys'])} {form} {len(th)} {_num(th)} 2\n")
    res = _parse(_run(stdin))
    near_rel(res["gp_nd"][0], d[f"fx_f{form}"], 1e-12, what="fx")
    near_rel(res["gp_nd"][1:], d[f"grad_f{form}"], RTOL, what="grad")
    assert list(res["stack"]) == [0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("touch", [0, 1])
def test_bridge_round_trip(touch):
    """device -> Eigen -> device hands back the materialised node (no bridge
    vari, no upload); a modified copy is gathered; L's upper triangle is the
    one dummy vari; the gradient equals the all-device one, plus the closed
    form of the host-side terms when a host node touches the blocks (their
    gathers then run; the dummy's adjoint is dropped like the reference's)."""
    N = 40
    r = _parse(_run(f"bridge {N} {touch}\n"))
    for k in ("same_node", "no_bridge_pushed", "modified_copy_new_node", "lower_dummy"):
        assert r[k][0] == 1.0, k
    assert r["blocks_after"][0] == 0.0
    g_eig, g_dev = r["grad_eigen"][1:], r["grad_device"][1:].copy()
    if touch:
        i, j = np.indices((N, N))
        a = (np.where(i == j, 2.0, 0.0) + 1.0 / (1.0 + i + j)).T.ravel()  # column-major like the C++ side
        K00, K10 = a[0] + 1.0, a[1]
        g_dev[0] += 2.0 + 3.0 * (-K10 / (2.0 * K00 ** 1.5))  # dL10/dK00
        g_dev[1] += 3.0 / np.sqrt(K00)                          # dL10/dK10
        near_rel(r["L10"][0], K10 / np.sqrt(K00), 1e-15, what="L10")
    near_rel(g_eig, g_dev, 1e-12, what="grad")


@pytest.mark.gpu
def test_cholesky_gradient_after_nan_poisoned_arena():
    """the Murray reverse reads its work matrix's strict
    upper triangle as stored zeros; with the arena pre-filled with NaN bytes
    and recovered, the gradient at n > 2 * 512 (the two-level reverse) must
    be finite and bit-identical to the clean one."""
    r = _parse(_run("chol_nan_arena 1100\n"))
    assert r["nan_entries"][0] == 0
    assert r["diff_entries"][0] == 0


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1024, 2048])
def test_cholesky_mvn_closed_form_predicted_across_failure(N):
    """The closed-form Cholesky reverse under an MVN at one tape position:
    evaluation 2 forms K^{-1} alongside the factorisation (the history says
    the closed form), 3 fails with a not-positive-definite input while that
    work is queued, 4 runs normally again -- 2 and 4 equal the unpredicted 1."""
    r = _parse(_run(f"chol_mvn_predicted {N}\n"))
    assert r["threw3"][0] == 1
    assert r["finite"][0] == 1
    assert r["rel2"][0] < 1e-12 and r["rel4"][0] < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("N", [300, 1024])
def test_cholesky_factor_adjoint_readable_after_closed_form(N):
    """After a sweep whose Cholesky reverse took the closed form (L's dense
    adjoint never formed), L.adj() still returns the MVN's partials, and A's
    adjoint is unchanged: equal to the dense path's (SMG_CHOL_MVN_CLOSED_FORM=0)."""
    def rows(env):
        out = _run(f"chol_mvn_ladj {N}\n", env=env)
        return np.array([[float(v) for v in l.split()[1:]] for l in out.strip().splitlines()])
    a, b = rows(None), rows({"SMG_CHOL_MVN_CLOSED_FORM": "0"})
    near_rel(a, b, 1e-11, what="L / A adjoint sums")
    assert abs(a[0, 0]) > 0


def _gpi_split(v, N):
    t = N * (N + 1) // 2
    o = [3, t, N, t, t, 7]
    parts, k = [], 0
    for n in o:
        parts.append(np.asarray(v[k:k + n]))
        k += n
    assert k == len(v)
    return parts


@pytest.mark.gpu
@pytest.mark.parametrize("closed", ["1", "0"])
@pytest.mark.parametrize("N,variant", [(64, 0), (64, 1), (64, 2), (256, 0), (256, 1)])
def test_gp_intermediate_adjoints(N, variant, closed):
    """After a top-level lp.grad() of the Stan-codegen GP (Eigen::Matrix<var>
    K, Kd, L), the intermediate varis hold what the reference's do
    (tests/golden/gp_intermediate_N*.json, written by the real Stan Math from
    the same bnd::run_gp_intermediate): K(i, j).adj() (K(i, j) and K(j, i)
    one vari, rev/mat/fun/gp_exp_quad_cov.hpp:235), Kd's own diagonal varis
    (add_diag shares K's off-diagonal varis, prim/mat/fun/add_diag.hpp:25-27),
    L's lower adjoints (the MVN's partials; one dummy above the diagonal,
    cholesky_decompose.hpp:34-48) and the same number of distinct varis.
    Variant 1 adds host consumers of L (the factor's adjoint has a second
    writer: the dense reverse), variant 2 of K's shared varis and Kd's
    diagonal (the bridges gather them); closed = "0" forces the dense
    Cholesky reverse throughout.  1e-10 relative (matrix entries with a
    1e-10 * max-norm absolute floor: they carry cancellation)."""
    d = golden(f"gp_intermediate_N{N}")
    th = d["theta"]
    env = None if closed == "1" else {"SMG_CHOL_MVN_CLOSED_FORM": "0"}
    res = _parse(_run(f"gp_inter {N} {variant} {_num(d['x'])} {_num(d['y'])} {_num(th)}\n", env=env))
    got, want = res["gpi"], np.concatenate([[d[f"fx_v{variant}"]], d[f"v{variant}"]])
    near_rel(got[0], want[0], 1e-12, what="lp")
    g, w = _gpi_split(got[1:], N), _gpi_split(want[1:], N)
    near_rel(g[0], w[0], RTOL, what="grad theta")
    for name, a, b in zip(("K adj", "Kd diag adj", "L adj", "L val"), g[1:5], w[1:5]):
        near_rel(a, b, RTOL, atol=RTOL * float(np.abs(b).max()), what=name)
    assert list(g[5]) == list(w[5]), ("identity", list(g[5]), list(w[5]))
    assert list(res["stack"]) == [0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("N", [300, 1024])
def test_gp_kernel_two_inverse_consumers(N, mode):
    """One gp_exp_quad_cov output with two consumers that each take the
    Cholesky closed form's inverse-form adjoint (mode 0: two add_diag ->
    cholesky -> MVN terms; mode 1: K factored directly and through add_diag)
    and a nested sweep whose window holds only the factor and the MVN (mode 2:
    the deposit's receivers are not chained, Kd.adj() must still hold it).
    Two evaluations (the second on the predicted closed form, at N = 1024
    with the progressive K^{-1}); the hyperparameter gradient and the K / Kd
    adjoint sums equal the dense Cholesky reverse's (SMG_CHOL_MVN_CLOSED_FORM=0)
    at 1e-10 relative."""
    def run(env):
        return _parse(_run(f"gp_share {N} {mode} 2\n", env=env))
    a, b = run(None), run({"SMG_CHOL_MVN_CLOSED_FORM": "0"})
    tag = f"share{mode}"
    near_rel(a[tag][0], b[tag][0], 1e-12, what="lp")
    near_rel(a[tag][1:], b[tag][1:], RTOL, what="theta' and adjoint sums")
    assert abs(b[tag][8]) > 0  # Kd's adjoint holds the deposit
    if mode != 2:
        assert np.all(np.abs(b[tag][5:9]) > 0)
    assert list(a["stack"]) == [0.0, 0.0] and list(b["stack"]) == [0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 1, 2])
def test_gp_intermediate_adjoints_N1024(variant):
    """bnd::run_gp_intermediate at N = 1024 (a 512-multiple: the second
    evaluation forms K^{-1} progressively with the panels and deposits the
    inverse-form adjoint through add_diag into gp_exp_quad_cov), with the
    intermediate adjoints read after the sweep (variant 0), host consumers of
    L (variant 1: the dense reverse) and of K / Kd (variant 2: the deposit
    expanded into K's dense adjoint on the progressive path).  The theta
    gradient of variant 0 against the reference's (gp_N1024.json, the same
    model) and every intermediate adjoint against the dense Cholesky reverse
    (SMG_CHOL_MVN_CLOSED_FORM=0), 1e-10."""
    N = 1024
    d = golden(f"gp_N{N}")
    cmd = f"gp_inter_rep {N} {variant} 2 {_num(d['x'])} {_num(d['y'])} {_num(d['theta'])}\n"
    a = _parse(_run(cmd))
    b = _parse(_run(cmd, env={"SMG_CHOL_MVN_CLOSED_FORM": "0"}))
    ga, gb = _gpi_split(a["gpi"][1:], N), _gpi_split(b["gpi"][1:], N)
    near_rel(a["gpi"][0], b["gpi"][0], 1e-12, what="lp")
    if variant == 0:
        near_rel(a["gpi"][0], d["fx"], 1e-12, what="lp vs reference")
        near_rel(ga[0], d["grad"], RTOL, what="grad theta vs reference")
    near_rel(ga[0], gb[0], RTOL, what="grad theta")
    for name, x, y in zip(("K adj", "Kd diag adj", "L adj", "L val"), ga[1:5], gb[1:5]):
        near_rel(x, y, RTOL, atol=RTOL * float(np.abs(y).max()), what=name)
    assert list(ga[5]) == list(gb[5])
    assert list(a["stack"]) == [0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("closed", ["1", "0"])
@pytest.mark.parametrize("N", [64, 256])
def test_gp_intermediate_replaced_element(N, closed):
    """cholesky_decompose of an Eigen matrix that is a materialised node but
    for one replaced element (Kd(N-1, N/2) = 0.5 (x + x), a new vari of the
    same value): the factorisation started speculatively on the node is
    discarded once the host's pointer check fails, and the gathered copy's
    result is the reference's unmodified one (gp_intermediate_N*.json
    variant 0, 1e-10): the same lp, theta gradient, K / Kd / L adjoints and
    L values; the identity entries but those of Kd's sharing (one new vari)."""
    d = golden(f"gp_intermediate_N{N}")
    th = d["theta"]
    env = None if closed == "1" else {"SMG_CHOL_MVN_CLOSED_FORM": "0"}
    res = _parse(_run(f"gp_inter {N} 3 {_num(d['x'])} {_num(d['y'])} {_num(th)}\n", env=env))
    got, want = res["gpi"], np.concatenate([[d["fx_v0"]], d["v0"]])
    near_rel(got[0], want[0], 1e-12, what="lp")
    g, w = _gpi_split(got[1:], N), _gpi_split(want[1:], N)
    near_rel(g[0], w[0], RTOL, what="grad theta")
    for name, a, b in zip(("K adj", "Kd diag adj", "L adj", "L val"), g[1:5], w[1:5]):
        near_rel(a, b, RTOL, atol=RTOL * float(np.abs(b).max()), what=name)
    gi, wi = list(g[5]), list(w[5])
    assert [gi[q] for q in (0, 3, 4, 6)] == [wi[q] for q in (0, 3, 4, 6)], ("identity", gi, wi)
    assert gi[1] == 0.0 and gi[5] == wi[5] + 1  # (Kd no longer shares K's vari there: one more vari)
    assert list(res["stack"]) == [0.0, 0.0]


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1024, 4096])
def test_gp_codegen_1d_golden(N):
    """The Stan-codegen GP marginal (1-D x, Eigen::Matrix<var> K, Kd, L, the
    path Stan models take) through gradient() at N = 1024 and the north-star
    N = 4096, twice (the second evaluation forms K^{-1} alongside the
    factorisation: the predicted closed form), against the reference's
    gradient (gp_N*.json) at 1e-10."""
    d = golden(f"gp_N{N}")
    res = _parse(_run(f"gp_1d {N} 2 {_num(d['x'])} {_num(d['y'])} {_num(d['theta'])}\n", timeout=600))
    for r in range(2):
        got = res[f"gp1d_{r}"]
        near_rel(got[0], d["fx"], 1e-12, what=f"fx {r}")
        near_rel(got[1:], d["grad"], RTOL, what=f"grad {r}")
    assert list(res["stack"]) == [0.0, 0.0]
