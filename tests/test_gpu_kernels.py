"""GPU parity tests of every C-ABI entry point (libsmg_hip.so through ctypes)
against the golden vectors produced by the real reference and against the
CPU restatement (oracle) on seeded inputs.

Tolerances are written per test: 1e-10 relative (expect_near_rel semantics)
for values and gradients unless stated; plain BLAS products are checked at
1e-13 relative to the operand norms.
"""
import glob
import os

import numpy as np
import pytest

import gen
from _util import GOLDEN, check_against_fixture, f64, glm2_oracle, glm_cat_oracle, golden, near_rel, oracle, ptr, spd_oracle

pytestmark = pytest.mark.gpu
RTOL = 1e-10


@pytest.fixture(scope="module")
def ctx():
    from math_amd import hip
    c = hip.Context(0, 1 << 30)
    yield c
    c.close()


@pytest.fixture(autouse=True)
def _rewind(ctx):
    m = ctx.mark()
    yield
    assert ctx.status() == 0
    ctx.rewind(m)


def F(a):  # column-major flat
    return np.asfortranarray(a).ravel(order="F")


# ------------------------------------------------------------------ GEMM
@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(16, 16, 4), (70, 33, 45), (130, 257, 64), (64, 64, 4096), (512, 384, 300)])
def test_gemm(ctx, ta, tb, m, n, k):
    rng = np.random.default_rng(m * 7 + n * 3 + k)
    A = rng.standard_normal((k, m) if ta else (m, k))
    B = rng.standard_normal((n, k) if tb else (k, n))
    C = rng.standard_normal((m, n))
    ref = 1.5 * (A.T if ta else A) @ (B.T if tb else B) - 0.5 * C
    dA, dB, dC = ctx.put(F(A)), ctx.put(F(B)), ctx.put(F(C))
    ctx.call("smg_gemm", ta, tb, 0, m, n, k, 1.5, dA, A.shape[0], dB, B.shape[0], -0.5, dC, m)
    out = ctx.get(dC, m * n).reshape(n, m).T
    scale = np.abs(A).max() * np.abs(B).max() * k + np.abs(C).max()
    assert np.abs(out - ref).max() <= 1e-13 * scale


@pytest.mark.parametrize("uplo", [1, 2])
def test_gemm_triangle(ctx, uplo):
    rng = np.random.default_rng(5)
    n, k = 200, 77
    A = rng.standard_normal((n, k))
    C = rng.standard_normal((n, n))
    ref = C - A @ A.T
    dA, dC = ctx.put(F(A)), ctx.put(F(C))
    ctx.call("smg_gemm", 0, 1, uplo, n, n, k, -1.0, dA, n, dA, n, 1.0, dC, n)
    out = ctx.get(dC, n * n).reshape(n, n).T
    mask = np.tril(np.ones((n, n), bool)) if uplo == 1 else np.triu(np.ones((n, n), bool))
    assert np.abs(out[mask] - ref[mask]).max() < 1e-12
    assert np.array_equal(out[~mask], C[~mask])  # other triangle untouched


@pytest.mark.parametrize("n,k", [(64, 64), (200, 77), (512, 512), (1000, 300)])
def test_gemm_symmetric_output(ctx, n, k):
    """uplo 3: the lower half of C = A A^T - C0 computed, written mirrored."""
    rng = np.random.default_rng(n + k)
    A = rng.standard_normal((n, k))
    C0 = rng.standard_normal((n, n))
    C0 = C0 + C0.T
    ref = A @ A.T - C0
    dA, dC = ctx.put(F(A)), ctx.put(F(C0))
    ctx.call("smg_gemm", 0, 1, 3, n, n, k, 1.0, dA, n, dA, n, -1.0, dC, n)
    out = ctx.get(dC, n * n).reshape(n, n).T
    assert np.array_equal(out, out.T)
    assert np.abs(out - ref).max() < 1e-12 * (np.abs(A).max() ** 2 * k + np.abs(C0).max())


@pytest.mark.parametrize("m,n,k,ta", [(512, 512, 3584, 1), (512, 2560, 1536, 1), (130, 70, 5000, 0), (64, 64, 4096, 1)])
def test_gemm_split_k_deterministic(ctx, m, n, k, ta):
    """Split-K products (small output grid, long K): fixed-order partial slabs,
    three runs bitwise equal."""
    rng = np.random.default_rng(m + n + k)
    A = rng.standard_normal((k, m) if ta else (m, k))
    B = rng.standard_normal((k, n))
    C0 = rng.standard_normal((m, n))
    ref = -(A.T if ta else A) @ B + C0
    outs = []
    for _ in range(3):
        dA, dB, dC = ctx.put(F(A)), ctx.put(F(B)), ctx.put(F(C0))
        ctx.call("smg_gemm", ta, 0, 0, m, n, k, -1.0, dA, A.shape[0], dB, k, 1.0, dC, m)
        outs.append(ctx.get(dC, m * n).reshape(n, m).T)
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])
    assert np.abs(outs[0] - ref).max() <= 1e-13 * (np.abs(A).max() * np.abs(B).max() * k + np.abs(C0).max())


@pytest.mark.parametrize("case", ["c_is_a_right", "c_is_b_left", "c_in_a_general", "disjoint_blocks"])
def test_gemm_in_place(ctx, case):
    """In-place products of the blocked TRSMs (C = C W, C = W C) and general
    aliasing must be race-free whatever tile size the dispatcher picks."""
    rng = np.random.default_rng(11)
    if case == "c_is_a_right":      # C (2000 x 64) = C W (64 x 64), like C_adj D^{-1}
        m, n = 2000, 64
        X = rng.standard_normal((m, n)); W = rng.standard_normal((n, n))
        dX, dW = ctx.put(F(X)), ctx.put(F(W))
        ctx.call("smg_gemm", 0, 1, 0, m, n, n, 1.0, dX, m, dW, n, 0.0, dX, m)
        ref = X @ W.T
        out = ctx.get(dX, m * n).reshape(n, m).T
    elif case == "c_is_b_left":     # C (64 x 300) = W^T C, like X_p = W_p^T B_p
        m, n = 64, 300
        X = rng.standard_normal((m, n)); W = rng.standard_normal((m, m))
        dX, dW = ctx.put(F(X)), ctx.put(F(W))
        ctx.call("smg_gemm", 1, 0, 0, m, n, m, 1.0, dW, m, dX, m, 0.0, dX, m)
        ref = W.T @ X
        out = ctx.get(dX, m * n).reshape(n, m).T
    elif case == "c_in_a_general":  # C (300 x 200) = 2 C B - C, beta != 0: out-of-place fallback
        m, n = 300, 200
        X = rng.standard_normal((m, n)); B = rng.standard_normal((n, n))
        dX, dB = ctx.put(F(X)), ctx.put(F(B))
        ctx.call("smg_gemm", 0, 0, 0, m, n, n, 2.0, dX, m, dB, n, -1.0, dX, m)
        ref = 2.0 * X @ B - X
        out = ctx.get(dX, m * n).reshape(n, m).T
    else:                            # disjoint sub-blocks of one matrix (Murray's R/D/B/C)
        N = 400
        Lm = rng.standard_normal((N, N))
        dL = ctx.put(F(Lm))
        j, k = 128, 192                   # La[j:k, 0:k] -= La[k:, j:k]^T La[k:, 0:k]
        at = lambda r, c: dL + 8 * (r + c * N)  # noqa: E731  (device address of L[r, c])
        ctx.call("smg_gemm", 1, 0, 0, k - j, k, N - k, -1.0, at(k, j), N, at(k, 0), N, 1.0, at(j, 0), N)
        ref = Lm.copy()
        ref[j:k, 0:k] -= Lm[k:, j:k].T @ Lm[k:, 0:k]
        out = ctx.get(dL, N * N).reshape(N, N).T
    assert np.abs(out - ref).max() <= 1e-11 * (np.abs(ref).max() + 1.0)


def test_mfma_layout_asymmetric(ctx):
    """A = I with an asymmetric B catches a transposed D layout."""
    n = 16
    B = np.arange(n * n, dtype=np.float64).reshape(n, n)
    I = np.eye(n)
    dA, dB, dC = ctx.put(F(I)), ctx.put(F(B)), ctx.zeros(n * n)
    ctx.call("smg_gemm", 0, 0, 0, n, n, n, 1.0, dA, n, dB, n, 0.0, dC, n)
    out = ctx.get(dC, n * n).reshape(n, n).T
    assert np.array_equal(out, B)


# ------------------------------------------------------- gp_exp_quad_cov
@pytest.mark.parametrize("n,ld", [(1, 1), (33, 35), (300, 300), (301, 302), (2050, 2050), (300, 301)])
@pytest.mark.parametrize("vec", [0, 1])
def test_add_diag_fwd(ctx, n, ld, vec):
    """add_diag (prim/mat/fun/add_diag.hpp:20-55) bit for bit, through the
    16-byte column form (even n and ld) and the element form."""
    rng = np.random.default_rng(n + ld + vec)
    A = rng.uniform(-1, 1, (n, n))
    d = rng.uniform(0, 2, n)
    Ap = np.zeros((n, ld)); Ap[:, :n] = A.T        # column-major with leading dimension ld
    B = np.full(n * ld, 5.0)
    dB = ctx.put(B)
    ctx.call("smg_add_diag_fwd", ctx.put(Ap.ravel()), ld, n, 0.25, ctx.put(d) if vec else None, dB, ld)
    out = ctx.get(dB, n * ld).reshape(n, ld)
    ref = A + np.diag(d if vec else np.full(n, 0.25))
    assert np.array_equal(out[:, :n].T, ref)
    assert np.all(out[:, n:] == 5.0)


@pytest.mark.parametrize("m,n,ld", [(1, 1, 1), (33, 20, 35), (300, 300, 300), (300, 301, 302),
                                    (2050, 2050, 2050), (64, 200, 64), (301, 300, 301)])
def test_copy_tril(ctx, m, n, ld):
    """Y = tril(X) over the m x n block (column form for even m and ld): the
    lower trapezoid copied, the strict upper stored as zeros even where Y held
    NaN (recycled arena memory), the rows past m untouched."""
    rng = np.random.default_rng(m + 7 * n + ld)
    X = rng.uniform(-1, 1, n * ld)
    Y0 = rng.uniform(-1, 1, n * ld)
    Y0[::3] = np.nan
    dY = ctx.put(Y0)
    ctx.call("smg_copy_tril", m, n, ctx.put(X), ld, dY, ld)
    out = ctx.get(dY, n * ld).reshape(n, ld).T          # out[i, j] = Y(i, j)
    Xm, Ym = X.reshape(n, ld).T, Y0.reshape(n, ld).T
    i, j = np.indices((ld, n))
    ref = np.where(i >= m, Ym, np.where(i >= j, Xm, 0.0))
    assert np.array_equal(out, ref, equal_nan=True)


@pytest.mark.parametrize("n,ld", [(1, 1), (33, 35), (300, 300), (301, 302), (2050, 2050)])
def test_add_diag_rev(ctx, n, ld):
    """add_diag's reverse: A's adjoint += B's adjoint (column form for even n
    and ld, element form otherwise), the scalar diagonal's adjoint = trace."""
    rng = np.random.default_rng(3 * n + ld)
    Ba = rng.uniform(-1, 1, n * ld)
    Aa0 = rng.uniform(-1, 1, n * ld)
    dAa, dd = ctx.put(Aa0), ctx.zeros(1)
    ctx.call("smg_add_diag_rev", ctx.put(Ba), ld, n, dAa, ld, dd, 0)
    out = ctx.get(dAa, n * ld).reshape(n, ld)
    ref = (Aa0 + Ba).reshape(n, ld)
    assert np.array_equal(out[:, :n], ref[:, :n])
    assert np.array_equal(out[:, n:], Aa0.reshape(n, ld)[:, n:])
    near_rel(ctx.get(dd, 1)[0], np.trace(Ba.reshape(n, ld)[:, :n]), 1e-13, what="diag adj")


@pytest.mark.parametrize("n", [1, 2, 33, 300, 2050, 4096])
def test_gp_cov(ctx, n):
    x = gen.unif(11 + n, n, -10, 10)
    K_ref = np.zeros(n * n)
    oracle().oracle_gp_cov(ptr(x), n, 1.3, 0.7, ptr(K_ref))
    dx, dK = ctx.put(x), ctx.zeros(n * n)
    ctx.call("smg_gp_exp_quad_cov_fwd", dx, n, 1.3, 0.7, dK, n)
    near_rel(ctx.get(dK, n * n), K_ref, 1e-14, atol=1e-300, what="K")
    W = gen.unif(12 + n, n * n, -1, 1)
    ga, gl = np.zeros(1), np.zeros(1)
    oracle().oracle_gp_cov_rev(ptr(x), n, 1.3, 0.7, ptr(W), ptr(ga), ptr(gl))
    dW, dout = ctx.put(W), ctx.zeros(2)
    ctx.call("smg_gp_exp_quad_cov_rev", dx, n, 1.3, 0.7, dW, n, dout)
    out = ctx.get(dout, 2)
    near_rel(out, [ga[0], gl[0]], 1e-11, what="gp rev")


@pytest.mark.parametrize("n,D", [(1, 3), (2, 2), (33, 3), (300, 1), (300, 5), (2051, 3), (64, 200)])
def test_gp_cov_nd(ctx, n, D):
    """D-dimensional gp_exp_quad_cov (rev/mat/fun/gp_exp_quad_cov.hpp:158-184,
    96-112) against float64 numpy over the same squared distances (summed in
    coordinate order) and, for D = 1, bit-equal to the scalar-x entries."""
    X = gen.unif(31 + n + D, n * D, -5, 5).reshape(n, D)  # point i = row i (device: D x n column-major)
    s, l = 1.3, 0.9
    d2 = np.zeros((n, n))
    for d in range(D):
        d2 = d2 + (X[:, d][:, None] - X[:, d][None, :]) ** 2
    K_ref = s * s * np.exp(-d2 * (0.5 / (l * l)))
    np.fill_diagonal(K_ref, s * s)
    dx, dK = ctx.put(X.ravel()), ctx.zeros(n * n)
    ctx.call("smg_gp_exp_quad_cov_nd_fwd", dx, D, n, s, l, dK, n)
    near_rel(ctx.get(dK, n * n), F(K_ref), 1e-13, atol=1e-300, what="K")
    W = gen.unif(32 + n, n * n, -1, 1)
    Wm = W.reshape(n, n).T
    off = ~np.eye(n, dtype=bool)
    prod = Wm * K_ref
    g_s = 2.0 / s * (prod[off].sum() + np.trace(Wm) * s * s)
    g_l = (prod * d2)[off].sum() / l ** 3
    dW, dout = ctx.put(W), ctx.zeros(2)
    ctx.call("smg_gp_exp_quad_cov_nd_rev", dx, D, n, s, l, dW, n, dout)
    near_rel(ctx.get(dout, 2), [g_s, g_l], 1e-11, what="gp nd rev")
    if D == 1:
        dK1 = ctx.zeros(n * n)
        ctx.call("smg_gp_exp_quad_cov_fwd", dx, n, s, l, dK1, n)
        assert np.array_equal(ctx.get(dK1, n * n), ctx.get(dK, n * n))


# ------------------------------------------------------------- cholesky
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "cholesky_N*.json"))))
def test_cholesky_golden(ctx, path):
    d = golden(os.path.basename(path)[:-5])
    N = int(d["N"])
    dA, dL, dD = ctx.put(f64(d["A"])), ctx.zeros(N * N), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_check_symmetric", dA, N, N)
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    assert ctx.status() == 0
    near_rel(ctx.get(dL, N * N), d["L"], 1e-12, atol=1e-300, what="L")
    W = d["W"].reshape(N, N).T
    dLa, dAa = ctx.put(F(np.tril(W))), ctx.zeros(N * N)
    ctx.call("smg_cholesky_rev", dL, N, dD, dLa, N, N, dAa, N)
    g = ctx.get(dAa, N * N)
    near_rel(g, d["grad_A"], RTOL, atol=RTOL * np.abs(d["grad_A"]).max(), what="grad_A")


@pytest.mark.parametrize("N", [65, 300, 1000])
def test_cholesky_vs_oracle(ctx, N):
    rng = np.random.default_rng(N)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + np.eye(N)
    A = 0.5 * (A + A.T)
    Lref = np.zeros(N * N)
    assert oracle().oracle_cholesky(ptr(F(A)), N, ptr(Lref)) == 0
    dA, dL, dD = ctx.put(F(A)), ctx.zeros(N * N), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    L = ctx.get(dL, N * N)
    near_rel(L, Lref, 1e-11, atol=1e-11 * np.abs(Lref).max(), what="L")
    W = np.tril(rng.uniform(-1, 1, (N, N)))
    Aref = np.zeros(N * N)
    oracle().oracle_cholesky_rev(ptr(Lref), ptr(F(W)), N, ptr(Aref))
    dLa, dAa = ctx.put(F(W)), ctx.zeros(N * N)
    ctx.call("smg_cholesky_rev", dL, N, dD, dLa, N, N, dAa, N)
    g = ctx.get(dAa, N * N)
    near_rel(g, Aref, 1e-10, atol=1e-10 * np.abs(Aref).max(), what="grad_A")


@pytest.mark.parametrize("N", [300, 1000, 2048])
def test_cholesky_aux_block_inverses(ctx, N):
    """smg_cholesky_fwd's aux: every full 64/128/256/512-row diagonal block's
    inverse (the 64 level and, since round 4, the 128 level from the panel
    kernel's inverter workgroup; 256 / 512 by doubling after the panels) times
    that block of L is the identity, with stored zeros above the diagonal."""
    rng = np.random.default_rng(N + 11)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + np.eye(N)
    A = 0.5 * (A + A.T)
    lib = ctx.lib
    dA, dL = ctx.put(F(A)), ctx.zeros(N * N)
    naux = lib.smg_cholesky_aux_doubles(N)
    dD = ctx.zeros(naux)
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    L = ctx.get(dL, N * N).reshape(N, N).T
    aux = ctx.get(dD, naux).reshape(-1, N).T  # N rows, column blocks of the levels
    off = 0
    for s in (64, 128, 256, 512):
        for b in range(0, N - s + 1, s):
            X = aux[b:b + s, off:off + s]
            assert np.abs(np.triu(X, 1)).max() == 0.0, (s, b)
            E = X @ L[b:b + s, b:b + s] - np.eye(s)
            assert np.abs(E).max() < 1e-11, (s, b, np.abs(E).max())
        off += s


@pytest.mark.parametrize("N,with_ws", [(65, False), (600, False), (1536, True), (2048, False)])
def test_cholesky_fwd_stream(ctx, N, with_ws):
    """smg_cholesky_fwd_checked_mark_stream: the factor streamed to pinned
    host memory panel by panel (the Eigen boundary's cholesky_decompose) --
    every panel's marker lands, the host copy is the packed lower triangle of
    the device factor bit for bit, and the factor equals the unstreamed entry's
    bit for bit (with and without the progressive K^{-1} workspace)."""
    import ctypes
    rng = np.random.default_rng(N + 7)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + np.eye(N)
    A = 0.5 * (A + A.T)
    T = N * (N + 1) // 2
    lib = ctx.lib
    dA = ctx.put(F(A))
    dL0, dD0 = ctx.zeros(N * N), ctx.zeros(lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_cholesky_fwd_checked", dA, N, N, dL0, N, dD0)
    L0 = ctx.get(dL0, N * N)
    dL, dD, dP = ctx.zeros(N * N), ctx.zeros(lib.smg_cholesky_aux_doubles(N)), ctx.zeros(T)
    ws = ctx.zeros(lib.smg_cholesky_mvn_rev_ws_doubles(N)) if with_ws else None
    host = lib.smg_host_scratch(ctx.ptr, T * 8)
    assert host
    started = ctypes.c_int(-1)
    ctx.call("smg_cholesky_fwd_checked_mark_stream", dA, N, N, dL, N, dD, ws, ctypes.byref(started), dP, host, 3)
    npan = lib.smg_cholesky_stream_panels(N)
    assert npan == (1 if N <= 512 else -(-N // 512))
    for p in range(npan):
        ctx.call("smg_marker_wait", 3 + p)
    h = np.ctypeslib.as_array(ctypes.cast(host, ctypes.POINTER(ctypes.c_double)), shape=(T,)).copy()
    st = ctypes.c_int(-1)
    ctx.call("smg_status_mark_wait", ctypes.byref(st))
    assert st.value == 0
    ctx.call("smg_join_async")
    L = ctx.get(dL, N * N)
    assert np.array_equal(L, L0)
    Lm = L.reshape(N, N).T  # row-major view of the column-major factor
    packed = np.concatenate([Lm[j:, j] for j in range(N)])
    assert np.array_equal(h, packed)
    assert started.value == (2 if with_ws else 0)


@pytest.mark.parametrize("N,mu", [(64, False), (320, True), (1000 // 64 * 64, False), (2048, True)])
def test_mvn_cholesky_fwd_inv(ctx, N, mu):
    """smg_mvn_cholesky_fwd_inv: w = W (y - mu), s = W^T w on an explicit
    inverse W = L^{-1} (the reference's arithmetic, inv_L products) -- against
    the solve-based smg_mvn_cholesky_fwd on the same factor (1e-12) and the
    oracle's value (1e-10).  W's strict upper outside its diagonal 64 x 64
    tiles holds NaN: it must never be read."""
    rng = np.random.default_rng(N + 3)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.3 * np.eye(N)
    A = 0.5 * (A + A.T)
    y = rng.uniform(-1, 1, N)
    m = rng.uniform(-0.5, 0.5, N) if mu else None
    dA, dL, dD = ctx.put(F(A)), ctx.zeros(N * N), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    L = ctx.get(dL, N * N).reshape(N, N).T
    W = np.linalg.inv(np.tril(L))
    W = np.tril(W)
    blk = np.arange(N) // 64
    W[blk[:, None] < blk[None, :]] = np.nan  # above the diagonal tiles: never read
    dy, dmu = ctx.put(y), (ctx.put(m) if mu else None)
    ws0, lp0 = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd", dy, dmu, dL, N, dD, N, ws0, lp0)
    ws1, lp1 = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd_inv", dy, dmu, dL, N, ctx.put(F(W)), N, N, ws1, lp1)
    a0, a1 = ctx.get(ws0, 2 * N), ctx.get(ws1, 2 * N)
    near_rel(a1, a0, 1e-12, atol=1e-12 * np.abs(a0).max(), what="[w, s]")
    v0, v1 = ctx.get(lp0, 1)[0], ctx.get(lp1, 1)[0]
    near_rel(np.array([v1]), np.array([v0]), 1e-12, what="lp")
    r = y - (m if mu else 0.0)
    w = np.linalg.solve(np.tril(L), r)
    lp_ref = -0.5 * N * np.log(2 * np.pi) - 0.5 * w @ w - np.log(np.diag(L)).sum()
    near_rel(np.array([v1]), np.array([lp_ref]), 1e-10, what="lp vs numpy")
    assert ctx.lib.smg_mvn_cholesky_fwd_inv(ctx.ptr, dy, dmu, dL, N, ctx.put(F(W)), N - 1, N, ws1, lp1) != 0


def test_mvn_inverse_from_progressive_factorisation(ctx):
    """The factorisation's progressive W = L^{-1} (smg_cholesky_fwd_checked_mark_inv,
    *started == 2) is what smg_mvn_cholesky_fwd_inv reads after
    smg_cholesky_inverse_wait: the same [w, s] and lp as the solves (1e-12)."""
    import ctypes
    N = 2048
    rng = np.random.default_rng(99)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.2 * np.eye(N)
    A = 0.5 * (A + A.T)
    y = rng.uniform(-1, 1, N)
    lib = ctx.lib
    dA, dL, dD = ctx.put(F(A)), ctx.zeros(N * N), ctx.zeros(lib.smg_cholesky_aux_doubles(N))
    ws = ctx.zeros(lib.smg_cholesky_mvn_rev_ws_doubles(N))
    started = ctypes.c_int(-1)
    ctx.call("smg_cholesky_fwd_checked_mark_inv", dA, N, N, dL, N, dD, ws, ctypes.byref(started))
    assert started.value == 2
    st = ctypes.c_int(-1)
    ctx.call("smg_status_mark_wait", ctypes.byref(st))
    assert st.value == 0
    ctx.call("smg_cholesky_inverse_wait")
    dy = ctx.put(y)
    ws1, lp1 = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd_inv", dy, None, dL, N, ws, N, N, ws1, lp1)
    ws0, lp0 = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd", dy, None, dL, N, dD, N, ws0, lp0)
    ctx.call("smg_join_async")
    a0, a1 = ctx.get(ws0, 2 * N), ctx.get(ws1, 2 * N)
    near_rel(a1, a0, 1e-12, atol=1e-12 * np.abs(a0).max(), what="[w, s]")
    near_rel(ctx.get(lp1, 1), ctx.get(lp0, 1), 1e-12, what="lp")


def test_progressive_w_only_and_tangent_from_it(ctx):
    """smg_cholesky_fwd_checked_mark_winv (*started == 3): W = L^{-1} formed
    beside the panels without K^{-1} -- from a NaN workspace, its lower
    triangle bit-identical to the K^{-1} mode's W (the same parts in the same
    order) and within 1e-10 of numpy's inverse; then smg_chol_tangent_fwd_w on
    that W (its strict upper outside the 512-row diagonal blocks left NaN, so
    any read of it would poison the outputs) against smg_chol_tangent_fwd,
    which forms its own zero-padded W: Ld, Y, P within 1e-10 (P from a NaN
    buffer: L P reads only what the fused Y / Phi(Y) epilogue writes)."""
    import ctypes
    N = 2048
    rng = np.random.default_rng(5)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.2 * np.eye(N)
    A = 0.5 * (A + A.T)
    Ad = rng.uniform(-1, 1, (N, N))
    Ad = 0.5 * (Ad + Ad.T)
    lib = ctx.lib
    nw = lib.smg_cholesky_mvn_rev_ws_doubles(N)
    nan_ws = np.full(nw, np.nan)
    dA = ctx.put(F(A))
    outs = {}
    for fn, want in (("smg_cholesky_fwd_checked_mark_winv", 3), ("smg_cholesky_fwd_checked_mark_inv", 2)):
        dL, dD, ws = ctx.zeros(N * N), ctx.zeros(lib.smg_cholesky_aux_doubles(N)), ctx.put(nan_ws)
        started = ctypes.c_int(-1)
        ctx.call(fn, dA, N, N, dL, N, dD, ws, ctypes.byref(started))
        assert started.value == want
        st = ctypes.c_int(-1)
        ctx.call("smg_status_mark_wait", ctypes.byref(st))
        assert st.value == 0
        ctx.call("smg_cholesky_inverse_wait")
        ctx.call("smg_join_async")
        W = ctx.get(ws, N * N).reshape(N, N, order="F")
        outs[fn] = (dL, dD, ws, W)
    Lh = ctx.get(outs["smg_cholesky_fwd_checked_mark_winv"][0], N * N).reshape(N, N, order="F")
    W3 = np.tril(outs["smg_cholesky_fwd_checked_mark_winv"][3])
    W2 = np.tril(outs["smg_cholesky_fwd_checked_mark_inv"][3])
    assert np.array_equal(W3, W2), "W differs between the W-only and the K^{-1} modes"
    Wref = np.linalg.inv(np.tril(Lh))
    near_rel(W3, Wref, 1e-10, atol=1e-10 * np.abs(Wref).max(), what="W vs numpy")
    dL, dD, ws, _ = outs["smg_cholesky_fwd_checked_mark_winv"]
    dAd = ctx.put(F(Ad))
    res = []
    for given in (True, False):
        Wt, Y, Ld = (ctx.zeros(N * N) for _ in range(3))
        P = ctx.put(np.full(N * N, np.nan))  # (P = Phi(Y) is written lower plus the diagonal blocks' zero upper)
        if given:
            ctx.call("smg_chol_tangent_fwd_w", dL, N, ws, dAd, N, N, Wt, Y, P, Ld, N)
        else:
            Wn = ctx.zeros(N * N)
            ctx.call("smg_chol_tangent_fwd", dL, N, dD, dAd, N, N, Wn, Wt, Y, P, Ld, N)
        res.append([np.tril(ctx.get(x, N * N).reshape(N, N, order="F")) for x in (Ld, Y, P)])
    for a, b, what in zip(res[0], res[1], ("Ld", "Y", "P")):
        assert np.isfinite(a).all(), what
        near_rel(a, b, 1e-10, atol=1e-10 * np.abs(b).max(), what=what)


@pytest.mark.parametrize("trans", [0, 1])
def test_trmv_inv_vs_numpy(ctx, trans):
    """smg_trmv_inv: y = W x / W^T x over W's lower triangle (the whole
    strict upper NaN: never read, the diagonal tiles' masked), against numpy
    at 1e-13; run twice, bit-identical (fixed-order partial sums)."""
    N = 1024
    rng = np.random.default_rng(17)
    W = np.tril(rng.uniform(-1, 1, (N, N)))
    Wd = W.copy()
    Wd[np.triu_indices(N, 1)] = np.nan
    x = rng.uniform(-1, 1, N)
    dW, dx = ctx.put(F(Wd)), ctx.put(x)
    outs = []
    for _ in range(2):
        dy = ctx.zeros(N)
        ctx.call("smg_trmv_inv", trans, dW, N, N, dx, dy)
        outs.append(ctx.get(dy, N))
    ref = (W.T if trans else W) @ x
    near_rel(outs[0], ref, 1e-13, atol=1e-13 * np.abs(ref).max(), what="trmv")
    assert np.array_equal(outs[0], outs[1])
    assert ctx.lib.smg_trmv_inv(ctx.ptr, trans, dW, N, N - 1, dx, dx) != 0  # n % 64 != 0


@pytest.mark.parametrize("n", [1, 63, 1024])
def test_rank1_lower(ctx, n):
    """smg_rank1_lower: A += alpha x y^T on the lower triangle only (the
    strict upper untouched), against numpy at 1e-15."""
    rng = np.random.default_rng(n)
    A = rng.uniform(-1, 1, (n, n))
    x, y = rng.uniform(-1, 1, n), rng.uniform(-1, 1, n)
    dA = ctx.put(F(A))
    ctx.call("smg_rank1_lower", n, -0.75, ctx.put(x), ctx.put(y), dA, n)
    out = ctx.get(dA, n * n).reshape(n, n).T
    ref = A - 0.75 * np.tril(np.outer(x, y))
    lo = np.tril(np.ones((n, n), bool))
    near_rel(out[lo], ref[lo], 1e-15, atol=1e-15, what="lower")
    assert np.array_equal(out[~lo], A[~lo])


@pytest.mark.parametrize("mode", [0, 1])
def test_progressive_inverses_from_nan_workspace(ctx, mode):
    """The progressive factorisation's by-products against numpy, from a
    workspace and an aux buffer that start as NaN: every 512-row block row's
    256- and 512-level diagonal-block inverses (aux columns 64 + 128 .. and
    64 + 128 + 256 .., ld N), W = L^{-1} (lower) and C = K^{-1} (lower: the
    shares and Y accumulate with beta = 0 on their first contribution, nothing
    is cleared beforehand).  1e-10.  mode 0: one k_inv_block512 launch per
    row (its occupancy guard must pass on an MI355X), running beside the
    panels and the trailing-update GEMMs; mode 1: the six-launch chain, the
    fallback when the guard fails."""
    ctx.call("smg_set_inv_block_mode", mode)
    try:
        if mode == 0:
            assert ctx.lib.smg_inv_block_fused(ctx.ptr, 2048) == 1 and ctx.lib.smg_inv_block_fused(ctx.ptr, 4096) == 1
        _progressive_inverses_check(ctx)
    finally:
        ctx.call("smg_set_inv_block_mode", 0)


def _progressive_inverses_check(ctx):
    import ctypes
    N = 2048
    rng = np.random.default_rng(7)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.2 * np.eye(N)
    A = 0.5 * (A + A.T)
    lib = ctx.lib
    naux = lib.smg_cholesky_aux_doubles(N)
    nws = lib.smg_cholesky_mvn_rev_ws_doubles(N)
    dA, dL = ctx.put(F(A)), ctx.zeros(N * N)
    dD, ws = ctx.put(np.full(naux, np.nan)), ctx.put(np.full(nws, np.nan))
    started = ctypes.c_int(-1)
    ctx.call("smg_cholesky_fwd_checked_mark_inv", dA, N, N, dL, N, dD, ws, ctypes.byref(started))
    assert started.value == 2
    st = ctypes.c_int(-1)
    ctx.call("smg_status_mark_wait", ctypes.byref(st))
    assert st.value == 0
    ctx.call("smg_cholesky_inverse_wait")
    ctx.call("smg_join_async")
    L = np.tril(ctx.get(dL, N * N).reshape(N, N, order="F"))
    aux = ctx.get(dD, naux).reshape(-1, N).T  # aux[:, c]: column c of the n x SMG_AUX_COLS strip set
    for off, s2 in ((64 + 128, 256), (64 + 128 + 256, 512)):
        for r0 in range(0, N, s2):
            got = aux[r0:r0 + s2, off:off + s2]
            want = np.linalg.inv(L[r0:r0 + s2, r0:r0 + s2])
            assert np.all(np.isfinite(got)), (s2, r0)
            near_rel(np.tril(got), np.tril(want), 1e-10, atol=1e-10 * np.abs(want).max(), what=f"W{s2} row {r0}")
            assert not np.any(np.triu(got, 1)), (s2, r0)  # stored zeros above
    W = ctx.get(ws, N * N).reshape(N, N, order="F")
    Winv = np.linalg.inv(L)
    near_rel(np.tril(W), np.tril(Winv), 1e-10, atol=1e-10 * np.abs(Winv).max(), what="W")
    C = ctx.get(ws + 8 * N * N, N * N).reshape(N, N, order="F")
    Kinv = np.linalg.inv(A)
    assert np.all(np.isfinite(np.tril(C)))
    near_rel(np.tril(C), np.tril(Kinv), 1e-9, atol=1e-10 * np.abs(Kinv).max(), what="K^-1")


@pytest.mark.parametrize("N", [64, 300, 1024, 2048])
def test_cholesky_rev_inverse_vs_murray(ctx, N):
    """smg_cholesky_rev_inverse (the closed form on W = L^{-1}: Abar lower +=
    tril(G + G^T) - diag(G), G = W^T Phi(L^T tril(Lbar)) W) against the blocked
    Murray reverse smg_cholesky_rev on the same factor and adjoint (1e-10,
    the lower triangle; the strict upper of Lbar carries junk both ignore).
    The workspace starts as NaN: a stale value the products read would show."""
    rng = np.random.default_rng(N + 5)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.5 * np.eye(N)
    A = 0.5 * (A + A.T)
    dA, dL, dD = ctx.put(F(A)), ctx.zeros(N * N), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    L = ctx.get(dL, N * N).reshape(N, N).T
    W = np.tril(np.linalg.inv(np.tril(L)))
    Lbar = rng.uniform(-1, 1, (N, N))
    G0 = rng.uniform(-1, 1, (N, N))
    # Murray (the reference's algorithm): overwrites its adjoint input
    dLa, dG = ctx.put(F(Lbar)), ctx.put(F(G0))
    ctx.call("smg_cholesky_rev", dL, N, dD, dLa, N, N, dG, N)
    Gm = ctx.get(dG, N * N).reshape(N, N).T
    dG2 = ctx.put(F(G0))
    ctx.call("smg_cholesky_rev_inverse", dL, N, ctx.put(F(W)), ctx.put(F(W.T)), N, ctx.put(F(Lbar)), N, N, dG2, N,
             ctx.put(np.full(2 * N * N, np.nan)))
    Gi = ctx.get(dG2, N * N).reshape(N, N).T
    low = np.tril(np.ones((N, N), bool))
    ref = Gm[low] - G0[low]
    near_rel(Gi[low] - G0[low], ref, 1e-10, atol=1e-10 * np.abs(ref).max(), what="Abar")
    assert np.array_equal(Gi[~low], G0[~low])


@pytest.mark.parametrize("n", [1, 2, 63, 300, 2049])
def test_sum_strict_upper(ctx, n):
    """smg_sum_strict_upper: the sum a Cholesky factor's dummy vari collects
    from the strict upper triangle (fixed order; 1e-13 against numpy)."""
    rng = np.random.default_rng(n)
    A = rng.uniform(-1, 1, (n, n))
    out = ctx.zeros(1)
    ctx.call("smg_sum_strict_upper", n, ctx.put(F(A)), n, out)
    ref = np.triu(A, 1).sum()
    assert abs(ctx.get(out, 1)[0] - ref) <= 1e-13 * max(1.0, np.abs(np.triu(A, 1)).sum())


@pytest.mark.parametrize("N,D,k", [(64, 1, 1), (301, 1, 1), (512, 3, 1), (1024, 1, 2), (257, 2, 3)])
def test_gp_inverse_adjoint_vs_composition(ctx, N, D, k):
    """smg_gp_inverse_adjoint (the GP marginal's three reverses in one pass
    over K^{-1}) against their composition on the device: the closed form's
    epilogue into Kd's adjoint (smg_cholesky_inverse_adjoint), add_diag's
    reverse, gp_exp_quad_cov's reverse -- d', sigma', l' at 1e-12."""
    rng = np.random.default_rng(N * 7 + D + k)
    M = rng.uniform(-1, 1, (N, N))
    C = M @ M.T / N + np.eye(N)
    s = rng.uniform(-1, 1, (k, 2 * N))  # observation o's s at o * 2N (the MVN's [w, s] blocks: s_stride 2N)
    x = rng.uniform(-3, 3, (N, D))
    sig, ell, adj = 1.3, 0.7, 0.8
    dC, ds, dx = ctx.put(F(C)), ctx.put(s.ravel()), ctx.put(x.ravel())
    dK = ctx.zeros(N * N)
    ctx.call("smg_gp_exp_quad_cov_nd_fwd", dx, D, N, sig, ell, dK, N)
    # composition
    dKd, dKa, dd0, o0 = ctx.zeros(N * N), ctx.zeros(N * N), ctx.zeros(1), ctx.zeros(2)
    ctx.call("smg_cholesky_inverse_adjoint", dC, N, N, ds, k, 2 * N, adj, dKd, N)
    ctx.call("smg_add_diag_rev", dKd, N, N, dKa, N, dd0, 0)
    ctx.call("smg_gp_exp_quad_cov_nd_rev", dx, D, N, sig, ell, dKa, N, o0)
    # fused
    dd1, o1 = ctx.zeros(1), ctx.zeros(2)
    ctx.call("smg_gp_inverse_adjoint", dC, N, N, ds, k, 2 * N, adj, dK, N, dx, D, sig, ell, dd1, o1)
    dd2 = ctx.zeros(1)  # the diagonal sum alone (K0, x unused)
    ctx.call("smg_gp_inverse_adjoint", dC, N, N, ds, k, 2 * N, adj, None, N, None, 1, 1.0, 1.0, dd2, None)
    r0 = np.concatenate([ctx.get(dd0, 1), ctx.get(o0, 2)])
    r1 = np.concatenate([ctx.get(dd1, 1), ctx.get(o1, 2)])
    near_rel(r1, r0, 1e-12, what="[d', sigma', l']")
    near_rel(ctx.get(dd2, 1), r0[:1], 1e-12, what="d' alone")
    # the epilogue against numpy: Phi(sum_o s_o s_o^T - k C) adj on the lower triangle
    S = sum(np.outer(s[o, :N], s[o, :N]) for o in range(k))
    G = adj * (S - k * C)
    G = np.tril(G, -1) + 0.5 * np.diag(np.diag(G))
    Kd = ctx.get(dKd, N * N).reshape(N, N).T
    near_rel(Kd, G, 1e-12, atol=1e-12 * np.abs(G).max(), what="epilogue")


@pytest.mark.parametrize("N", [65, 300, 1024, 2048])
def test_cholesky_mvn_closed_form_vs_oracle(ctx, N):
    """smg_cholesky_mvn_rev: cholesky_decompose's reverse for the MVN's
    lower-only partials Lbar = adj (tril(s w^T) - diag(1/L_ii)), in closed form
    adj Phi(s s^T - K^{-1}), against the oracle's Murray reverse of that Lbar
    (N = 65, 300: L^{-1} by the blocked solve; 1024, 2048: the doubling from
    the 512-row block inverses, with and without the factorisation's aux)."""
    rng = np.random.default_rng(N + 11)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + 0.2 * np.eye(N)
    A = 0.5 * (A + A.T)
    y = rng.uniform(-1, 1, N)
    dA, dL, dD = ctx.put(F(A)), ctx.zeros(N * N), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N))
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, dD)
    ws, dlp = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd", ctx.put(y), None, dL, N, dD, N, ws, dlp)
    L = ctx.get(dL, N * N).reshape(N, N).T
    w, s = np.split(ctx.get(ws, 2 * N), 2)
    adj = 0.75
    Lbar = adj * (np.tril(np.outer(s, w)) - np.diag(1.0 / np.diag(L)))
    Aref = np.zeros(N * N)
    oracle().oracle_cholesky_rev(ptr(F(L)), ptr(F(Lbar)), N, ptr(Aref))
    Aref = Aref.reshape(N, N).T
    wsz = ctx.lib.smg_cholesky_mvn_rev_ws_doubles(N)
    for aux in (dD, None):
        G0 = rng.uniform(-1, 1, (N, N))  # accumulates into the lower triangle only
        dG = ctx.put(F(G0))
        ctx.call("smg_cholesky_mvn_rev", dL, N, aux, N, ws + 8 * N, 1, 0, adj, dG, N, ctx.zeros(wsz))
        G = ctx.get(dG, N * N).reshape(N, N).T
        low = np.tril(np.ones((N, N), bool))
        near_rel(G[low] - G0[low], Aref[low], 1e-10, atol=1e-10 * np.abs(Aref).max(), what="grad_A")
        assert np.array_equal(G[~low], G0[~low])


def test_cholesky_not_pd_and_not_symmetric(ctx):
    N = 70
    A = np.eye(N)
    A[40, 40] = -1.0
    dA, dL = ctx.put(F(A)), ctx.zeros(N * N)
    ctx.call("smg_cholesky_fwd", dA, N, N, dL, N, ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(N)))
    assert ctx.status() & 2
    A = np.eye(N)
    A[5, 3] = 1e-7
    dA = ctx.put(F(A))
    ctx.call("smg_check_symmetric", dA, N, N)
    assert ctx.status() & 4
    A[5, 3] = 5e-9  # within CONSTRAINT_TOLERANCE
    dA = ctx.put(F(A))
    ctx.call("smg_check_symmetric", dA, N, N)
    assert ctx.status() == 0


@pytest.mark.parametrize("N,i,j,v,bad", [(200, 150, 10, 1e-7, True), (200, 10, 150, 1e-7, True),
                                         (200, 130, 129, -2e-8, True), (200, 63, 64, 1e-9, False),
                                         (129, 128, 0, float("nan"), True), (64, 63, 62, 0.0, False)])
def test_check_symmetric_tiles(ctx, N, i, j, v, bad):
    """Tile-pair symmetric check: one perturbed entry anywhere (either
    triangle, across tile boundaries, ragged last tile, NaN)."""
    rng = np.random.default_rng(N + i + j)
    B = rng.standard_normal((N, N))
    A = B + B.T
    A[i, j] += v
    ctx.call("smg_check_symmetric", ctx.put(F(A)), N, N)
    assert bool(ctx.status() & 4) == bad


# ------------------------------------------------------ mdivide_left_tri
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "mdivide_left_tri_*.json"))))
def test_mdivide_golden(ctx, path):
    d = golden(os.path.basename(path)[:-5])
    m, n, lower, kind = (int(d[s]) for s in ("m", "n", "lower", "kind"))
    dA, dB, dC = ctx.put(f64(d["A"])), ctx.put(f64(d["B"])), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_fwd", lower, dA, m, dB, m, m, n, dC, m)
    near_rel(ctx.get(dC, m * n), d["C"], 1e-12, atol=1e-13, what="C")
    dW, dAa, dBa, ws = ctx.put(f64(d["W"])), ctx.zeros(m * m), ctx.zeros(m * n), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_rev", lower, dA, m, dC, m, dW, m, m, n,
             dAa if kind != 1 else None, m, dBa if kind != 2 else None, m, ws)
    if kind != 1:
        near_rel(ctx.get(dAa, m * m), d["grad_A"], RTOL, atol=1e-12, what="gA")
    if kind != 2:
        near_rel(ctx.get(dBa, m * n), d["grad_B"], RTOL, atol=1e-12, what="gB")


def test_mdivide_large_vs_oracle(ctx):
    m, n = 300, 7
    rng = np.random.default_rng(3)
    S = rng.uniform(-1, 1, (m, m))
    S = S @ S.T / m + np.eye(m)
    L = np.linalg.cholesky(S)
    for lower, T in ((1, L), (0, L.T.copy())):
        B = rng.uniform(-1, 1, (m, n))
        Cref = np.zeros(m * n)
        oracle().oracle_mdivide_left_tri(lower, ptr(F(T)), ptr(F(B)), m, n, ptr(Cref))
        dA, dB, dC = ctx.put(F(T)), ctx.put(F(B)), ctx.zeros(m * n)
        ctx.call("smg_mdivide_left_tri_fwd", lower, dA, m, dB, m, m, n, dC, m)
        near_rel(ctx.get(dC, m * n), Cref, 1e-11, atol=1e-13, what="C")


# ------------------------------------------------------------- multiply
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "multiply_[0-9]*.json"))))
def test_multiply_golden(ctx, path):
    d = golden(os.path.basename(path)[:-5])
    m, k, n, kind = (int(d[s]) for s in ("m", "k", "n", "kind"))
    dA, dB, dC = ctx.put(f64(d["A"])), ctx.put(f64(d["B"])), ctx.zeros(m * n)
    ctx.call("smg_multiply_fwd", dA, m, dB, k, m, k, n, dC, m)
    near_rel(ctx.get(dC, m * n), d["C"], 1e-12, atol=1e-14, what="C")
    dW, dAa, dBa = ctx.put(f64(d["W"])), ctx.zeros(m * k), ctx.zeros(k * n)
    ctx.call("smg_multiply_rev", dA, m, dB, k, dW, m, m, k, n, dAa if kind != 2 else None, m,
             dBa if kind != 1 else None, k)
    if kind != 2:
        near_rel(ctx.get(dAa, m * k), d["grad_A"], RTOL, atol=1e-13, what="gA")
    if kind != 1:
        near_rel(ctx.get(dBa, k * n), d["grad_B"], RTOL, atol=1e-13, what="gB")


# ------------------------------------------------------------------ mvn
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "mvn_cholesky_N*.json"))))
def test_mvn_golden(ctx, path):
    d = golden(os.path.basename(path)[:-5])
    N = int(d["N"])
    dy, dmu, dL = ctx.put(f64(d["y"])), ctx.put(f64(d["mu"])), ctx.put(f64(d["L"]))
    ws, dlp = ctx.zeros(2 * N), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd", dy, dmu, dL, N, None, N, ws, dlp)
    near_rel(ctx.get(dlp, 1), [d["fx"]], 1e-12, what="lp")
    gy, gm, gL = ctx.zeros(N), ctx.zeros(N), ctx.zeros(N * N)
    ctx.call("smg_mvn_cholesky_rev", dL, N, None, N, ws, 1.0, 0, gy, gm, gL, N)
    near_rel(ctx.get(gy, N), d["grad_y"], RTOL, what="gy")
    near_rel(ctx.get(gm, N), d["grad_mu"], RTOL, what="gmu")
    gref = d["grad_L"]
    near_rel(ctx.get(gL, N * N), gref, RTOL, atol=RTOL * np.abs(gref).max(), what="gL")
    # lower_only mode == the lower triangle of the full partials
    gL2 = ctx.zeros(N * N)
    ctx.call("smg_mvn_cholesky_rev", dL, N, None, N, ws, 1.0, 1, None, None, gL2, N)
    low = np.tril(np.ones((N, N), bool)).ravel(order="F")
    g2 = ctx.get(gL2, N * N)
    near_rel(g2[low], gref[low], RTOL, atol=RTOL * np.abs(gref).max(), what="gL lower")
    assert np.all(g2[~low] == 0.0)


def test_mvn_known_answer(ctx):
    d = golden("mvn_cholesky_known")
    L = np.linalg.cholesky(d["Sigma"].reshape(3, 3))
    dy, dmu, dL = ctx.put(f64(d["y"])), ctx.put(f64(d["mu"])), ctx.put(F(L))
    ws, dlp = ctx.zeros(6), ctx.zeros(1)
    ctx.call("smg_mvn_cholesky_fwd", dy, dmu, dL, 3, None, 3, ws, dlp)
    assert abs(ctx.get(dlp, 1)[0] - d["expected"]) < 1e-5  # EXPECT_FLOAT_EQ


# ------------------------------------------------- lse / special / normal
@pytest.mark.parametrize("kind", [0, 1, 2])
def test_log_sum_exp(ctx, kind):
    d = golden(f"log_sum_exp_{kind}")
    x = f64(d["x"])
    n = len(x)
    dx, dout, dg = ctx.put(x), ctx.zeros(1), ctx.zeros(n)
    ctx.call("smg_log_sum_exp_fwd", dx, n, dout)
    lse = ctx.get(dout, 1)[0]
    near_rel(lse, d["fx"], 1e-14, what="lse")
    ctx.call("smg_log_sum_exp_rev", dx, n, lse, 1.0, dg)
    near_rel(ctx.get(dg, n), d["grad"], 1e-12, atol=1e-15, what="grad")


def test_log_sum_exp_edge(ctx):
    dout = ctx.zeros(1)
    ctx.call("smg_log_sum_exp_fwd", ctx.zeros(1), 0, dout)
    assert ctx.get(dout, 1)[0] == -np.inf
    x = np.array([1.0, np.inf, 3.0])
    ctx.call("smg_log_sum_exp_fwd", ctx.put(x), 3, dout)
    assert ctx.get(dout, 1)[0] == np.inf


def test_special(ctx):
    d = golden("special")
    x = f64(d["x"])
    n = len(x)
    dx = ctx.put(x)
    outs = {}
    for f in ("lgamma", "digamma", "trigamma"):
        dy = ctx.zeros(n)
        ctx.call(f"smg_{f}_fwd", dx, n, dy)
        outs[f] = ctx.get(dy, n)
    # lgamma: ROCm libm vs glibc lgamma_r, both faithful: 1e-13 relative
    # (absolute 1e-13 near the roots at 1 and 2)
    near_rel(outs["lgamma"], d["lgamma"], 1e-13, atol=1e-13, what="lgamma")
    near_rel(outs["digamma"], d["digamma"], 1e-13, atol=1e-13, what="digamma")
    near_rel(outs["trigamma"], d["trigamma"], 1e-13, what="trigamma")
    ones = ctx.put(np.ones(n))
    g1, g2 = ctx.zeros(n), ctx.zeros(n)
    ctx.call("smg_lgamma_rev", dx, n, ones, g1)
    ctx.call("smg_digamma_rev", dx, n, ones, g2)
    near_rel(ctx.get(g1, n), d["grad_lgamma"], 1e-13, atol=1e-13, what="dlgamma")
    near_rel(ctx.get(g2, n), d["grad_digamma"], 1e-13, what="ddigamma")


def test_normal(ctx):
    d = golden("normal_N1024")
    th = f64(d["theta"])
    dth, d0, d1 = ctx.put(th), ctx.put(np.zeros(1)), ctx.put(np.ones(1))
    out, gy = ctx.zeros(1), ctx.zeros(1024)
    ctx.call("smg_normal_lpdf", dth, 1, d0, 0, d1, 0, 1024, 7, out, gy, None, None)
    near_rel(ctx.get(out, 1), [d["fx"]], 1e-13, what="fx")
    near_rel(ctx.get(gy, 1024), d["grad"], 1e-14, what="grad")
    d = golden("normal_vec9")
    dy, dm, ds = ctx.put(f64(d["y"])), ctx.put(f64(d["mu"])), ctx.put(f64(d["sigma"]))
    out, gy, gm, gs = ctx.zeros(1), ctx.zeros(9), ctx.zeros(9), ctx.zeros(9)
    ctx.call("smg_normal_lpdf", dy, 1, dm, 1, ds, 1, 9, 7, out, gy, gm, gs)
    near_rel(ctx.get(out, 1), [d["fx"]], 1e-13, what="fx")
    near_rel(ctx.get(gy, 9), d["grad_y"], 1e-13, what="gy")
    near_rel(ctx.get(gm, 9), d["grad_mu"], 1e-13, what="gmu")
    near_rel(ctx.get(gs, 9), d["grad_sigma"], 1e-13, what="gs")
    out = ctx.zeros(1)  # propto: only sigma and quadratic terms (all operands var)
    ctx.call("smg_normal_lpdf", dy, 1, dm, 1, ds, 1, 9, 6, out, None, None, None)
    near_rel(ctx.get(out, 1), [d["fx_propto"]], 1e-13, what="fx propto")


# --------------------------------------------------------------- GLM
def _glm(ctx, x, y, th, R, M):
    dx, dy, dab = ctx.put(F(x) if x.ndim == 2 else x), ctx.put(y.astype(np.int32)), ctx.put(f64(th))
    ws = ctx.zeros(int(ctx.lib.smg_glm_ws_doubles(R, M)))
    out = ctx.zeros(M + 2)
    ctx.call("smg_bernoulli_logit_glm", dy, dx, R, M, R, dab, ws, out)
    return ctx.get(out, M + 2)


@pytest.mark.parametrize("name", ["glm_R1000_M8", "glm_R10000_M256", "glm_R100000_M256"])
def test_glm_golden(ctx, name):
    d = golden(name)
    R, M = int(d["R"]), int(d["M"])
    x, y, th = gen.glm_inputs(R, M)
    out = _glm(ctx, x, y, th, R, M)
    near_rel(out[0], d["fx"], 1e-12, what="fx")
    near_rel(out[1:], d["grad"], RTOL, what="grad")


def _glm2(ctx, kind, x, y, th, R, M):
    """Device normal_id / poisson_log GLM -> (logp, gradient) assembled as the
    host layer does (normal: logp = -N log sqrt(2 pi) - N log sigma - sq/2,
    sigma' = (sq - N)/sigma; poisson: logp = sum(y theta - e^theta) - sum lgamma(y+1))."""
    dx, dab = ctx.put(F(x)), ctx.put(f64(th))
    ws = ctx.zeros(int(ctx.lib.smg_glm_ws_doubles(R, M)))
    out = ctx.zeros(M + 3)
    if kind == "normal":
        ctx.call("smg_normal_id_glm", ctx.put(f64(y)), dx, R, M, R, dab, ws, out)
        o = ctx.get(out, M + 2)
        sig = th[M + 1]
        lp = -0.91893853320467274178 * R - R * np.log(sig) - 0.5 * o[0]
        return lp, np.concatenate([o[1:], [(o[0] - R) / sig]])
    ctx.call("smg_poisson_log_glm", ctx.put(np.ascontiguousarray(y, dtype=np.int32)), dx, R, M, R, dab, ws, out)
    o = ctx.get(out, M + 3)
    return o[0] - o[M + 2], o[1:M + 2]


@pytest.mark.parametrize("name", ["normal_id_glm_R1000_M8", "normal_id_glm_R20000_M64",
                                  "poisson_log_glm_R1000_M8", "poisson_log_glm_R20000_M64"])
def test_glm2_golden(ctx, name):
    d = golden(name)
    R, M = int(d["R"]), int(d["M"])
    kind = "normal" if name.startswith("normal") else "poisson"
    x, y, th = gen.glm2_inputs(R, M, kind)
    lp, g = _glm2(ctx, kind, x, y, th, R, M)
    near_rel(lp, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, what="grad")


@pytest.mark.parametrize("kind", ["normal", "poisson"])
def test_glm2_vs_oracle_ragged(ctx, kind):
    """Beyond the fixtures: 200003 rows (ragged last tile, odd R) x 200
    covariates against the reference-pinned restatement."""
    R, M = 200003, 200
    x, y, th = gen.glm2_inputs(R, M, kind)
    lp, g = _glm2(ctx, kind, x, y, th, R, M)
    lpo, go = glm2_oracle(kind, x, y, th, M)
    near_rel(lp, lpo, 1e-12, what="fx")
    near_rel(g, go, RTOL, what="grad")


def _glm_cat(ctx, x, y, th, R, M, C, ldx=None):
    """Device categorical_logit_glm -> (logp, [alpha', beta'])."""
    ldx = R if ldx is None else ldx
    xf = np.zeros((ldx, M))
    xf[:R] = x
    ws = ctx.zeros(int(ctx.lib.smg_glm_categorical_ws_doubles(R, M, C)))
    out = ctx.zeros(1 + C + M * C)
    ctx.call("smg_categorical_logit_glm", ctx.put(np.ascontiguousarray(y, dtype=np.int32)), ctx.put(F(xf)), R, M,
             ldx, C, ctx.put(f64(th)), ws, out)
    o = ctx.get(out, 1 + C + M * C)
    return o[0], o[1:]


GLM_CAT_CASES = sorted(os.path.basename(p)[:-5] for p in glob.glob(os.path.join(GOLDEN, "categorical_logit_glm_R*.json")))


@pytest.mark.parametrize("name", GLM_CAT_CASES)
def test_glm_cat_golden(ctx, name):
    d = golden(name)
    R, M, C, ys = int(d["R"]), int(d["M"]), int(d["C"]), int(d["y_scalar"])
    x, y, th = gen.glm_cat_inputs(R, M, C)
    if ys:
        y = np.full(R, ys, dtype=np.int32)
    lp, g = _glm_cat(ctx, x, y, th, R, M, C)
    near_rel(lp, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, what="grad")


@pytest.mark.parametrize("R,M,C,ldx", [(200003, 256, 16, 200011), (17, 1, 2, 17), (33, 0, 7, 33), (1, 5, 16, 4),
                                       (5003, 300, 5, 5003), (4001, 20, 40, 4010), (999, 0, 17, 999)])
def test_glm_cat_vs_oracle(ctx, R, M, C, ldx):
    """Beyond the fixtures: ragged last tile, the fused path's M / C limits,
    M = 0 (intercept only), a leading dimension > R, one row; M > 256 or
    C > 16 take the GEMM path."""
    x, y, th = gen.glm_cat_inputs(R, M, C)
    lp, g = _glm_cat(ctx, x, y, th, R, M, C, ldx)
    lpo, go = glm_cat_oracle(x, y, th, M, C)
    near_rel(lp, lpo, 1e-12, what="fx")
    near_rel(g, go, RTOL, atol=1e-12 * max(1.0, np.abs(go).max()), what="grad")


@pytest.mark.parametrize("M,C", [(2, 3), (300, 20)])
def test_glm_cat_empty_and_args(ctx, M, C):
    """R = 0 -> zeros on both paths; C < 1, R < 0 or a short ldx -> SMG_ERR_ARG."""
    n = 1 + C + M * C
    out = ctx.put(np.full(n, 7.0))
    ws = ctx.zeros(max(64, int(ctx.lib.smg_glm_categorical_ws_doubles(0, M, C))))
    ab = ctx.put(np.ones(C + M * C))
    ctx.call("smg_categorical_logit_glm", 0, 0, 0, M, 0, C, ab, ws, out)
    assert np.all(ctx.get(out, n) == 0.0)
    assert ctx.lib.smg_categorical_logit_glm(ctx.ptr, 0, 0, 0, M, 0, 0, ab, ws, out) != 0
    assert ctx.lib.smg_categorical_logit_glm(ctx.ptr, 0, 0, -1, M, 0, C, ab, ws, out) != 0
    assert ctx.lib.smg_categorical_logit_glm(ctx.ptr, ws, ws, 10, M, 9, C, ab, ws, out) != 0


# ------------------------------------------ SURVEY 8(f) row 3 (spd.hip)
def _spd_device(ctx, kind, args, n, k, sym=1):
    """f = sum(W .* F(args)) and the gradient over every argument entry through
    the C-ABI (forward, then the reverse with Cadj = W)."""
    if kind == 0:
        A, B, W = args
        dA, dB, dW = ctx.put(F(A)), ctx.put(F(B)), ctx.put(F(W))
        L, aux, C = ctx.zeros(n * n), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(n)), ctx.zeros(n * k)
        ctx.call("smg_mdivide_left_spd_fwd", dA, n, dB, n, n, k, L, aux, C, n)
        gA, gB, ws = ctx.zeros(n * n), ctx.zeros(n * k), ctx.zeros(n * k)
        ctx.call("smg_mdivide_left_spd_rev", L, aux, n, k, C, n, dW, n, gA, n, gB, n, ws)
        f = float(np.sum(F(W) * ctx.get(C, n * k)))
        return f, np.concatenate([ctx.get(gA, n * n), ctx.get(gB, n * k)])
    if kind == 1:
        (A,) = args
        L, aux, out = ctx.zeros(n * n), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(n)), ctx.zeros(1)
        ctx.call("smg_log_determinant_spd_fwd", ctx.put(F(A)), n, n, L, aux, out)
        gA, ws = ctx.zeros(n * n), ctx.zeros(n * n)
        ctx.call("smg_log_determinant_spd_rev", L, aux, n, 1.0, gA, n, ws)
        return ctx.get(out, 1)[0], ctx.get(gA, n * n)
    if kind == 2:
        Lm, W = args
        dL, C, ws = ctx.put(F(Lm)), ctx.zeros(n * n), ctx.zeros(2 * n * k + n * n)
        ctx.call("smg_multiply_lower_tri_self_transpose_fwd", dL, n, n, k, C, n, ws)
        gL = ctx.zeros(n * k)
        ctx.call("smg_multiply_lower_tri_self_transpose_rev", dL, n, n, k, ctx.put(F(W)), n, gL, n, ws)
        return float(np.sum(F(W) * ctx.get(C, n * n))), ctx.get(gL, n * k)
    A, B, W = args
    dA, dB, C, ws = ctx.put(F(A)), ctx.put(F(B)), ctx.zeros(k * k), ctx.zeros(n * k + k * k)
    ctx.call("smg_quad_form_sym_fwd", dA, n, dB, n, n, k, C, k, ws)
    gA, gB = ctx.zeros(n * n), ctx.zeros(n * k)
    ctx.call("smg_quad_form_sym_rev", dA, n, dB, n, n, k, ctx.put(F(W)), k, sym, gA, n, gB, n, ws)
    return float(np.sum(F(W) * ctx.get(C, k * k))), np.concatenate([ctx.get(gA, n * n), ctx.get(gB, n * k)])


SPD_CASES = sorted(os.path.basename(p)[:-5] for pat in ("mdivide_left_spd_*", "log_determinant_spd_*",
                                                         "multiply_lower_tri_self_transpose_*", "quad_form_sym_*")
                   for p in glob.glob(os.path.join(GOLDEN, pat + ".json")))


@pytest.mark.parametrize("name", SPD_CASES)
def test_spd_golden(ctx, name):
    d = golden(name)
    kind, n, k = int(d["kind"]), int(d["n"]), int(d["k"])
    fx, g = _spd_device(ctx, kind, gen.spd_inputs(kind, n, k), n, k)
    assert ctx.status() == 0
    check_against_fixture(d, fx, g, RTOL, what=name)


@pytest.mark.parametrize("kind,n,k", [(0, 700, 33), (1, 600, 0), (2, 300, 200), (2, 200, 300),
                                      (3, 300, 150)])
def test_spd_vs_oracle_large(ctx, kind, n, k):
    """Beyond the fixtures (two-level Cholesky, multi-block TRSMs, ragged tiles)
    against the reference-pinned restatement."""
    args = gen.spd_inputs(kind, n, k)
    fx, g = _spd_device(ctx, kind, args, n, k)
    fo, go = spd_oracle(kind, args, n, k)
    near_rel(fx, fo, 1e-11, what="fx")
    near_rel(g, go, RTOL, atol=RTOL * np.abs(go).max(), what="grad")


def test_quad_form_sym_mixed_operands(ctx):
    """A data, B var: the rev vari's unsymmetrised adjoint (sym_adj = 0)."""
    n, k = 40, 12
    args = gen.spd_inputs(3, n, k)
    fx, g = _spd_device(ctx, 3, args, n, k, sym=0)
    fo, go = spd_oracle(3, args, n, k, sym=0)
    near_rel(fx, fo, 1e-12, what="fx")
    near_rel(g, go, RTOL, what="grad")


def test_spd_not_pd(ctx):
    n = 80
    A = np.eye(n)
    A[50, 50] = -2.0
    L, aux, out = ctx.zeros(n * n), ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(n)), ctx.zeros(1)
    ctx.call("smg_log_determinant_spd_fwd", ctx.put(F(A)), n, n, L, aux, out)
    assert ctx.status() & 2


def test_glm_extreme(ctx):
    d = golden("glm_extreme")
    R, M = int(d["R"]), int(d["M"])
    x = f64(d["x"]).reshape(M, R).T
    out = _glm(ctx, x, np.array(d["y"], dtype=np.int32), d["theta"], R, M)
    near_rel(out[0], d["fx"], 1e-12, what="fx")
    near_rel(out[1:], d["grad"], RTOL, what="grad")


def test_glm_wide_fallback(ctx):
    R, M = 3000, 300  # M > 256 takes the two-GEMV path
    x = gen.unif(77, R * M, -1, 1).reshape(M, R).T
    y = gen.bernoulli(78, R, 0.5)
    th = np.concatenate([[0.2], gen.unif(79, M, -0.1, 0.1)])
    ga, gb = np.zeros(1), np.zeros(M)
    lp = oracle().oracle_glm(ptr(y), ptr(F(x)), R, M, th[0], ptr(f64(th[1:])), ptr(ga), ptr(gb))
    out = _glm(ctx, x, y, th, R, M)
    near_rel(out[0], lp, 1e-12, what="fx")
    near_rel(out[1:], np.concatenate([ga, gb]), RTOL, what="grad")


# ------------------------------------------- GP composed through the C-ABI
def gp_gradient_abi(ctx, x, y, theta):
    """The GP functor of BASELINE config 3 composed from the C-ABI calls in the
    order the reverse sweep makes them (the C++ host layer does the same)."""
    n = len(x)
    a, r, s = theta
    dx, dy = ctx.put(f64(x)), ctx.put(f64(y))
    K, Kd, L = ctx.zeros(n * n), ctx.zeros(n * n), ctx.zeros(n * n)
    Dinv = ctx.zeros(ctx.lib.smg_cholesky_aux_doubles(n))
    ws, lp = ctx.zeros(2 * n), ctx.zeros(1)
    ctx.call("smg_gp_exp_quad_cov_fwd", dx, n, a, r, K, n)
    ctx.call("smg_add_diag_fwd", K, n, n, s * s, None, Kd, n)
    ctx.call("smg_check_symmetric", Kd, n, n)
    ctx.call("smg_cholesky_fwd", Kd, n, n, L, n, Dinv)
    ctx.call("smg_mvn_cholesky_fwd", dy, None, L, n, Dinv, n, ws, lp)
    fx = ctx.get(lp, 1)[0]
    La, Kda, Ka, sadj, hyp = ctx.zeros(n * n), ctx.zeros(n * n), ctx.zeros(n * n), ctx.zeros(1), ctx.zeros(2)
    ctx.call("smg_mvn_cholesky_rev", L, n, Dinv, n, ws, 1.0, 1, None, None, La, n)
    ctx.call("smg_cholesky_rev", L, n, Dinv, La, n, n, Kda, n)
    ctx.call("smg_add_diag_rev", Kda, n, n, Ka, n, sadj, 0)
    ctx.call("smg_gp_exp_quad_cov_rev", dx, n, a, r, Ka, n, hyp)
    h = ctx.get(hyp, 2)
    sa = ctx.get(sadj, 1)[0]
    return fx, np.array([h[0], h[1], sa * 2 * s])


@pytest.mark.parametrize("N", [16, 64, 256, 1024, 4096])
def test_gp_marginal_golden(ctx, N):
    d = golden(f"gp_N{N}")
    fx, g = gp_gradient_abi(ctx, d["x"], d["y"], d["theta"])
    assert ctx.status() == 0
    near_rel(fx, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, what="grad")


def gp_gradient_abi_closed_form(ctx, x, y, theta):
    """The same functor on the schedule the product takes at N % 512 == 0
    (the C++ layer's predicted closed form): the factorisation forms W = L^{-1}
    and K^{-1} progressively (smg_cholesky_fwd_checked_mark_inv, *started ==
    2), the MVN's forward runs on W (smg_mvn_cholesky_fwd_inv), and the
    reverse is one pass over K^{-1} for the three hyperparameter adjoints
    (smg_gp_inverse_adjoint) -- no Murray reverse, no add_diag / GP reverse."""
    import ctypes
    n = len(x)
    a, r, s = theta
    lib = ctx.lib
    dx, dy = ctx.put(f64(x)), ctx.put(f64(y))
    K, Kd, L = ctx.zeros(n * n), ctx.zeros(n * n), ctx.zeros(n * n)
    Dinv = ctx.zeros(lib.smg_cholesky_aux_doubles(n))
    inv_ws = ctx.zeros(lib.smg_cholesky_mvn_rev_ws_doubles(n))
    ws, lp = ctx.zeros(2 * n), ctx.zeros(1)
    ctx.call("smg_gp_exp_quad_cov_fwd", dx, n, a, r, K, n)
    ctx.call("smg_add_diag_fwd", K, n, n, s * s, None, Kd, n)
    started = ctypes.c_int(-1)
    ctx.call("smg_cholesky_fwd_checked_mark_inv", Kd, n, n, L, n, Dinv, inv_ws, ctypes.byref(started))
    assert started.value == 2
    st = ctypes.c_int(-1)
    ctx.call("smg_status_mark_wait", ctypes.byref(st))
    assert st.value == 0
    ctx.call("smg_cholesky_inverse_wait")
    ctx.call("smg_mvn_cholesky_fwd_inv", dy, None, L, n, inv_ws, n, n, ws, lp)
    fx = ctx.get(lp, 1)[0]
    dadj, hyp = ctx.zeros(1), ctx.zeros(2)
    s_vec = ws + 8 * n  # [w, s]: s = W^T w = K^{-1} y
    ctx.call("smg_cholesky_mvn_rev_v", n, s_vec, 1, 2 * n, 1.0, None, n, inv_ws, 1)  # joins K^{-1}
    ctx.call("smg_gp_inverse_adjoint", inv_ws + 8 * n * n, n, n, s_vec, 1, 2 * n, 1.0, K, n, dx, 1, a, r, dadj, hyp)
    h = ctx.get(hyp, 2)
    sa = ctx.get(dadj, 1)[0]
    return fx, np.array([h[0], h[1], sa * 2 * s])


@pytest.mark.parametrize("N", [1024, 4096])
def test_gp_marginal_golden_closed_form(ctx, N):
    """The headline's own schedule through the C-ABI against the reference's
    golden value and gradient (test_gp_marginal_golden composes Murray's
    reverse instead), twice on one context: bit-identical."""
    d = golden(f"gp_N{N}")
    m0 = ctx.mark()
    fx, g = gp_gradient_abi_closed_form(ctx, d["x"], d["y"], d["theta"])
    assert ctx.status() == 0
    near_rel(fx, d["fx"], 1e-12, what="fx")
    near_rel(g, d["grad"], RTOL, what="grad")
    ctx.rewind(m0)
    fx2, g2 = gp_gradient_abi_closed_form(ctx, d["x"], d["y"], d["theta"])
    assert fx2 == fx and np.array_equal(g2, g)


def test_handoff_stress_repeat_under_load(ctx):
    """The persistent kernels' fence-free hand-offs (smg_sync.h: sc1 payload,
    flag after every wave's vmcnt(0), sc1 loads after the poll) under uneven
    load: the GP gradient at N = 4096 and 2048 (panel kernel + persistent
    TRSVs) repeated while a second context keeps a large GEMM running on its
    own stream; every repetition must reproduce the first bit for bit (a
    stale read would not) and the first must match the reference."""
    from math_amd import hip
    other = hip.Context(0, 1 << 29)
    try:
        m = 4096
        A = other.put(np.random.default_rng(1).uniform(-1, 1, m * m // 4))
        C = other.zeros(m * m // 4)
        for N in (4096, 2048, 1024):
            d = golden(f"gp_N{N}") if N == 4096 else None
            x = gen.unif(gen.SEED + 7, N, -10.0, 10.0)
            y = np.sin(x)
            theta = (1.0, 1.5, 0.3)
            if d is not None:
                x, y, theta = d["x"], d["y"], d["theta"]
            runs = []
            for rep in range(16):
                if rep % 2 == 1:  # the other stream busy while this one runs
                    other.call("smg_gemm", 0, 1, 0, m // 2, m // 2, m // 2, 1e-3, A, m // 2, A, m // 2, 1.0, C,
                               m // 2)
                m0 = ctx.mark()
                runs.append(gp_gradient_abi(ctx, x, y, theta))
                assert ctx.status() == 0
                ctx.rewind(m0)
            fx0, g0 = runs[0]
            for fx, g in runs[1:]:
                assert fx == fx0 and np.array_equal(g, g0), (N, fx, fx0, g, g0)
            if d is not None:
                near_rel(fx0, d["fx"], 1e-12, what="fx")
                near_rel(g0, d["grad"], RTOL, what="grad")
        other.sync()
    finally:
        other.close()


@pytest.mark.parametrize("N,bad", [(70, (69, 35)), (300, (299, 150)), (1000, (999, 500)),
                                   (256, (255, 128)), (1024, (1023, 512)), (1024, (130, 129)),
                                   (512, (511, 0)), (512, (3, 2))])
def test_cholesky_fwd_checked(ctx, N, bad):
    """check_symmetric fused with the factorisation's copy: the same L and aux
    as smg_cholesky_fwd on a symmetric input; NOT_SYMMETRIC latched (and the
    upper triangle of L still zero) on an asymmetric one.  N % 64 == 0 takes
    the 16-byte form (k_check_symmetric_copy2); the perturbed entry `bad` sits
    in an off-diagonal tile or inside a diagonal tile."""
    rng = np.random.default_rng(N + 5)
    B = rng.uniform(-1, 1, (N, N))
    A = B @ B.T / N + np.eye(N)
    A = 0.5 * (A + A.T)
    na = ctx.lib.smg_cholesky_aux_doubles(N)
    dA = ctx.put(F(A))
    L1, D1 = ctx.put(np.full(N * N, 7.0)), ctx.zeros(na)
    L2, D2 = ctx.put(np.full(N * N, 7.0)), ctx.zeros(na)
    ctx.call("smg_cholesky_fwd", dA, N, N, L1, N, D1)
    ctx.call("smg_cholesky_fwd_checked", dA, N, N, L2, N, D2)
    assert ctx.status() == 0
    assert np.array_equal(ctx.get(L1, N * N), ctx.get(L2, N * N))
    assert np.array_equal(ctx.get(D1, na), ctx.get(D2, na))
    Lref = np.linalg.cholesky(A)
    assert np.allclose(ctx.get(L2, N * N).reshape(N, N, order="F"), Lref, rtol=0, atol=1e-12)
    A[bad] += 1e-6
    dA = ctx.put(F(A))
    L3 = ctx.put(np.full(N * N, 7.0))
    ctx.call("smg_cholesky_fwd_checked", dA, N, N, L3, N, ctx.zeros(na))
    assert ctx.status() & 4
    L = ctx.get(L3, N * N).reshape(N, N, order="F")
    assert np.all(np.triu(L, 1) == 0.0)


@pytest.mark.parametrize("m,n", [(2048, 512), (2048, 700), (1024, 1), (1536, 1), (4096, 1), (1024, 96), (600, 64)])
def test_mdivide_left_tri_512_blocks(ctx, m, n):
    """The large lower solve on 512-row blocks (inverses doubled up from the
    64-row level, tri.hip smg_trsm_impl) -- or, with one right-hand side, the
    persistent solve on the 256- / 512-row inverses -- against scipy's
    triangular solves:
    C = L^{-1} B, and the reverse's adjB = L^{-T} W, adjA = -tril(adjB C^T)
    (mdivide_left_tri.hpp:104-123)."""
    import scipy.linalg as sl
    rng = np.random.default_rng(m + n)
    S = rng.uniform(-1, 1, (m, m))
    S = S @ S.T / m + np.eye(m)
    L = np.linalg.cholesky(S)
    B = rng.uniform(-1, 1, (m, n))
    W = rng.uniform(-1, 1, (m, n))
    dA, dB, dC = ctx.put(F(L)), ctx.put(F(B)), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_fwd", 1, dA, m, dB, m, m, n, dC, m)
    C = ctx.get(dC, m * n).reshape(n, m).T
    Cref = sl.solve_triangular(L, B, lower=True)
    near_rel(C, Cref, 1e-10, atol=1e-11 * np.abs(Cref).max(), what="C")
    dW, dAa, dBa, ws = ctx.put(F(W)), ctx.zeros(m * m), ctx.zeros(m * n), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_rev", 1, dA, m, dC, m, dW, m, m, n, dAa, m, dBa, m, ws)
    gB = sl.solve_triangular(L, W, lower=True, trans="T")
    gA = -np.tril(gB @ Cref.T)
    near_rel(ctx.get(dBa, m * n).reshape(n, m).T, gB, 1e-10, atol=1e-11 * np.abs(gB).max(), what="gB")
    near_rel(ctx.get(dAa, m * m).reshape(m, m).T, gA, 1e-10, atol=1e-11 * np.abs(gA).max(), what="gA")


@pytest.mark.parametrize("m,n", [(1024, 1), (2048, 1), (4096, 1), (2048, 512)])
def test_mdivide_left_tri_ill_conditioned(ctx, m, n):
    """Rows scaled by a permuted grading 1e-6 .. 1 (cond(L) ~ 1e6, not a
    well-conditioned Cholesky factor): the large lower solves that multiply
    by explicit diagonal-block inverses must stay as backward stable as
    substitution (the reference's Eigen triangularView::solve).  Normwise
    backward error ||L C - B|| / (||L|| ||C|| + ||B||) within 20x scipy's
    substitution (+1e-16), both for C = L^{-1} B and for the reverse's L^{-T} W."""
    import scipy.linalg as sl
    rng = np.random.default_rng(7 * m + n)
    d = np.logspace(-6, 0, m)[rng.permutation(m)]
    S = rng.uniform(-1, 1, (m, m))
    L = d[:, None] * np.linalg.cholesky(S @ S.T / m + np.eye(m))
    B = rng.uniform(-1, 1, (m, n))
    W = rng.uniform(-1, 1, (m, n))

    def berr(A, X, R):
        return np.linalg.norm(A @ X - R) / (np.linalg.norm(A) * np.linalg.norm(X) + np.linalg.norm(R))

    dA, dB, dC = ctx.put(F(L)), ctx.put(F(B)), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_fwd", 1, dA, m, dB, m, m, n, dC, m)
    C = ctx.get(dC, m * n).reshape(n, m).T
    Cref = sl.solve_triangular(L, B, lower=True)
    assert np.all(np.isfinite(C))
    assert berr(L, C, B) <= 20 * berr(L, Cref, B) + 1e-16, (berr(L, C, B), berr(L, Cref, B))
    dW, dAa, dBa, ws = ctx.put(F(W)), ctx.zeros(m * m), ctx.zeros(m * n), ctx.zeros(m * n)
    ctx.call("smg_mdivide_left_tri_rev", 1, dA, m, dC, m, dW, m, m, n, dAa, m, dBa, m, ws)
    gB = ctx.get(dBa, m * n).reshape(n, m).T
    gref = sl.solve_triangular(L, W, lower=True, trans="T")
    assert np.all(np.isfinite(gB))
    assert berr(L.T, gB, W) <= 20 * berr(L.T, gref, W) + 1e-16, (berr(L.T, gB, W), berr(L.T, gref, W))


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("tri", [1, 2, 4, 8, 5, 6, 9, 10])
@pytest.mark.parametrize("uplo", [0, 1])
@pytest.mark.parametrize("m,n,k", [(70, 70, 45), (300, 300, 257), (1100, 1100, 700)])
def test_gemm_triangular_operands(ctx, ta, tb, tri, uplo, m, n, k):
    """smg_gemm_tri: K loops cut to the operands' triangles (stored zeros
    outside) give the dense product, for every operand orientation and output
    mode; the other output triangle is untouched."""
    rng = np.random.default_rng(m + 3 * k + 7 * tri + 11 * ta + 13 * tb + uplo)
    opA = rng.standard_normal((m, k))
    opB = rng.standard_normal((k, n))
    if tri & 1: opA = np.tril(opA)
    if tri & 2: opA = np.triu(opA)
    if tri & 4: opB = np.tril(opB)
    if tri & 8: opB = np.triu(opB)
    C = rng.standard_normal((m, n))
    ref = 0.75 * opA @ opB + 0.5 * C
    A = opA.T if ta else opA
    B = opB.T if tb else opB
    dA, dB, dC = ctx.put(F(A)), ctx.put(F(B)), ctx.put(F(C))
    ctx.call("smg_gemm_tri", ta, tb, uplo, tri, m, n, k, 0.75, dA, A.shape[0], dB, B.shape[0], 0.5, dC, m)
    out = ctx.get(dC, m * n).reshape(n, m).T
    scale = np.abs(opA).max() * np.abs(opB).max() * k + np.abs(C).max()
    mask = np.tril(np.ones((m, n), bool)) if uplo == 1 else np.ones((m, n), bool)
    assert np.abs(out[mask] - ref[mask]).max() <= 1e-13 * scale
    assert np.array_equal(out[~mask], C[~mask])


@pytest.mark.parametrize("n", [130, 1000, 2048])
def test_multiply_lower(ctx, n):
    """The tangent's L P product (both lower): C = L P with zero upper; the
    reverse accumulates tril(tril(Cadj) P^T) into Ladj and tril(L^T tril(Cadj))
    into Padj (upper triangles untouched)."""
    rng = np.random.default_rng(n)
    L = np.tril(rng.standard_normal((n, n)))
    P = np.tril(rng.standard_normal((n, n)))
    W = rng.standard_normal((n, n))
    La0, Pa0 = rng.standard_normal((n, n)), rng.standard_normal((n, n))
    dL, dP, dC = ctx.put(F(L)), ctx.put(F(P)), ctx.put(F(rng.standard_normal((n, n))))
    ctx.call("smg_multiply_lower_fwd", dL, n, dP, n, n, dC, n)
    C = ctx.get(dC, n * n).reshape(n, n).T
    ref = L @ P
    sc = np.sqrt(n) * 4
    assert np.abs(C - ref).max() <= 1e-13 * sc * n and np.all(np.triu(C, 1) == 0.0)
    dW, dLa, dPa, ws = ctx.put(F(W)), ctx.put(F(La0)), ctx.put(F(Pa0)), ctx.zeros(n * n)
    ctx.call("smg_multiply_lower_rev", dL, n, dP, n, dW, n, n, dLa, n, dPa, n, ws)
    La = ctx.get(dLa, n * n).reshape(n, n).T
    Pa = ctx.get(dPa, n * n).reshape(n, n).T
    Wl = np.tril(W)
    lo = np.tril(np.ones((n, n), bool))
    assert np.abs(La[lo] - (La0 + Wl @ P.T)[lo]).max() <= 1e-13 * sc * n
    assert np.abs(Pa[lo] - (Pa0 + L.T @ Wl)[lo]).max() <= 1e-13 * sc * n
    assert np.array_equal(La[~lo], La0[~lo]) and np.array_equal(Pa[~lo], Pa0[~lo])
