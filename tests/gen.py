"""Python mirror of oracle/gen.h (SplitMix64 + 53-bit uniforms), bit-exact.

Test infrastructure: regenerates the synthetic inputs the reference harness
(oracle/ref_harness.cpp) used for the fixtures whose inputs are not stored.
"""
import numpy as np

SEED = 20260101
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix(seed: int, n: int) -> np.ndarray:
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def u01(seed: int, n: int) -> np.ndarray:
    return (_splitmix(seed, n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def unif(seed: int, n: int, a: float, b: float) -> np.ndarray:
    return a + (b - a) * u01(seed, n)


def bernoulli(seed: int, n: int, p: float) -> np.ndarray:
    return (u01(seed, n) < p).astype(np.int32)


def mulchol_input(n: int) -> np.ndarray:
    """config 2 input A (n x n, column-major flat), ref_harness.cpp mulchol_input."""
    return unif(SEED + 2, n * n, -1.0, 1.0) * np.sqrt(3.0 / n)


def glm_inputs(R: int, M: int):
    """config 4 inputs, ref_harness.cpp glm_inputs: x (R x M col-major), y, theta."""
    x = unif(SEED + 41, R * M, -1.0, 1.0) * np.sqrt(3.0)
    y = bernoulli(SEED + 42, R, 0.5)
    b = unif(SEED + 43, M, -1.0, 1.0) * np.sqrt(3.0 / M)
    theta = np.concatenate([[0.1], b])
    return x.reshape(M, R).T.copy(order="F"), y, theta


def glm2_inputs(R: int, M: int, kind: str):
    """normal_id / poisson_log GLM inputs, ref_harness.cpp glm2_inputs: x and
    beta as glm_inputs; y uniform on [-2, 2) (normal) or floor(U[0, 6))
    counts (poisson); theta = (alpha, beta(M)[, sigma])."""
    x, _, th = glm_inputs(R, M)
    if kind == "normal":
        y = unif(SEED + 51, R, -2.0, 2.0)
        theta = np.concatenate([th, [1.3]])
    else:
        y = np.floor(unif(SEED + 52, R, 0.0, 6.0)).astype(np.int32)
        theta = np.concatenate([[th[0]], 0.5 * th[1:]])
    return x, y, theta


def glm_cat_inputs(R: int, M: int, C: int):
    """ref_harness.cpp glm_cat_inputs: x (R x M col-major) U[-1,1) sqrt 3,
    theta = (alpha U[-1,1) (C), beta U[-1,1) sqrt(3/M) (M x C col-major)),
    y = floor(U[0, C)) + 1."""
    x = unif(SEED + 81, R * M, -1.0, 1.0) * np.sqrt(3.0)
    a = unif(SEED + 82, C, -1.0, 1.0)
    b = unif(SEED + 83, M * C, -1.0, 1.0) * np.sqrt(3.0 / max(M, 1))
    y = (np.floor(unif(SEED + 84, R, 0.0, float(C))) + 1).astype(np.int32)
    return x.reshape(M, R).T.copy(order="F"), y, np.concatenate([a, b])


def maprect_inputs(J: int):
    """ref_harness.cpp maprect_inputs: x_r (J x 6, U[-2, 2)), x_i = (1 + j % 3
    outputs, fail flag 0), theta = (phi = (0.3, -0.2), theta_j = 0.1 j - 0.25)."""
    xr = unif(SEED + 91, J * 6, -2.0, 2.0).reshape(J, 6)
    xi = np.zeros((J, 2), dtype=np.int32)
    xi[:, 0] = 1 + np.arange(J) % 3
    th = np.concatenate([[0.3, -0.2], 0.1 * np.arange(J) - 0.25])
    return xr, xi, th


def spd_exact(n: int, seed: int) -> np.ndarray:
    """ref_harness.cpp spd_exact: S_ij = S_ji = u (lower source), S_ii = n + u_ii."""
    u = unif(seed, n * n, -1.0, 1.0).reshape(n, n).T  # u[i, j] = element i + j n (col-major)
    low = np.tril(u)
    S = low + np.tril(u, -1).T
    S[np.diag_indices(n)] = n + np.diag(u)
    return S


def unif_mat(r: int, c: int, seed: int) -> np.ndarray:
    return unif(seed, r * c, -1.0, 1.0).reshape(c, r).T.copy()


def spd_inputs(kind: int, n: int, k: int):
    """ref_harness.cpp fix_spd inputs: (args..., W) for kind 0 mdivide_left_spd,
    1 log_determinant_spd, 2 multiply_lower_tri_self_transpose, 3 quad_form_sym."""
    s0 = SEED + 60 + 10 * kind
    if kind in (0, 3):
        A, B = spd_exact(n, s0), unif_mat(n, k, s0 + 1)
        W = unif_mat(n if kind == 0 else k, k, s0 + 2)
        return A, B, W
    if kind == 1:
        return (spd_exact(n, s0),)
    L = unif_mat(n, k, s0 + 1)
    return L, unif_mat(n, n, s0 + 2)


def logdet_input(n: int, shift: int, flip: int) -> np.ndarray:
    """ref_harness.cpp fix_logdet input: U[-1, 1) (n x n) + shift sqrt(n) I,
    row 0 negated when flip."""
    A = unif_mat(n, n, SEED + 130 + n)
    A[np.diag_indices(n)] += shift * np.sqrt(float(n))
    if flip:
        A[0, :] *= -1.0
    return A
