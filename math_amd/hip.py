"""ctypes binding of the C-ABI in include/smg_hip.h (libsmg_hip.so).

This is the Python view of the drop-in boundary used by the parity tests and
bench.py.  It never falls back to a CPU path: if the HIP library or a GPU is
missing, every entry point raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libsmg_hip.so")

SMG_OK = 0
STATUS = {1: "hip", 2: "not_pd", 4: "not_symmetric", 8: "nonfinite", 16: "arg", 32: "oom", 64: "not_positive"}
FAMILIES = {"gemm": 0, "chol_fwd": 1, "chol_rev": 2, "gp": 3, "mvn": 4, "trsv": 5, "glm": 6, "elementwise": 7, "panel": 8, "comm": 9}

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_D = ctypes.c_double
_S = ctypes.c_size_t

_SIGS = {
    "smg_device_count": (_I, [ctypes.POINTER(_I)]),
    "smg_ctx_create": (_I, [_I, _S, ctypes.POINTER(_P)]),
    "smg_ctx_destroy": (_I, [_P]),
    "smg_ctx_device": (_I, [_P]),
    "smg_ctx_stream": (_P, [_P]),
    "smg_arena_alloc": (_P, [_P, _S]),
    "smg_arena_mark": (_S, [_P]),
    "smg_arena_rewind": (_I, [_P, _S]),
    "smg_arena_recover_all": (_I, [_P]),
    "smg_arena_used": (_S, [_P]),
    "smg_arena_reserved": (_S, [_P]),
    "smg_host_scratch": (_P, [_P, _S]),
    "smg_memcpy_h2d": (_I, [_P, _P, _P, _S]),
    "smg_memcpy_d2h": (_I, [_P, _P, _P, _S]),
    "smg_memcpy_d2d": (_I, [_P, _P, _P, _S]),
    "smg_memset": (_I, [_P, _P, _I, _S]),
    "smg_memset_async": (_I, [_P, _P, _S]),
    "smg_join_async": (_I, [_P]),
    "smg_sync": (_I, [_P]),
    "smg_sync_all": (_I, [_P]),
    "smg_status": (_I, [_P, ctypes.POINTER(_I)]),
    "smg_status_armed": (_I, [_P, ctypes.POINTER(_I)]),
    "smg_status_enqueue": (_I, [_P, _P]),
    "smg_status_inject": (_I, [_P, _I]),
    "smg_set_inv_block_mode": (_I, [_P, _I]),
    "smg_inv_block_fused": (_I, [_P, _I]),
    "smg_pinned_io": (_P, [_P, _S]),
    "smg_pinned_result": (_P, [_P, _S]),
    "smg_gather_scalars": (_I, [_P, _P, _I, _P, _P]),
    "smg_pack_tril": (_I, [_P, _I, _I, _P, _I, _P]),
    "smg_unpack_tril_add": (_I, [_P, _I, _I, _P, _P, _I]),
    "smg_publish_to_host": (_I, [_P, _P, _L, _P]),
    "smg_profile_enable": (_I, [_P, _I]),
    "smg_profile_read": (_I, [_P, _I, ctypes.POINTER(_D), ctypes.POINTER(_L)]),
    "smg_profile_flops": (_I, [_P, _I, ctypes.POINTER(_D)]),
    "smg_fill_unif": (_I, [_P, _P, _L, ctypes.c_ulonglong, _D, _D, _D]),
    "smg_fill_bernoulli": (_I, [_P, _P, _L, ctypes.c_ulonglong, _D]),
    "smg_gemm": (_I, [_P, _I, _I, _I, _I, _I, _I, _D, _P, _I, _P, _I, _D, _P, _I]),
    "smg_gemm_tri": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _D, _P, _I, _P, _I, _D, _P, _I]),
    "smg_gp_exp_quad_cov_fwd": (_I, [_P, _P, _I, _D, _D, _P, _I]),
    "smg_gp_exp_quad_cov_rev": (_I, [_P, _P, _I, _D, _D, _P, _I, _P]),
    "smg_bernoulli_logit_glm_checked": (_I, [_P, _P, _P, _L, _I, _L, _P, _P, _P]),
    "smg_bernoulli_logit_glm_io": (_I, [_P, _P, _P, _L, _I, _L, _D, _P, _P, _P, _P]),
    "smg_marker_record": (_I, [_P, _I]),
    "smg_marker_wait": (_I, [_P, _I]),
    "smg_gp_exp_quad_cov_nd_fwd": (_I, [_P, _P, _I, _I, _D, _D, _P, _I]),
    "smg_gp_exp_quad_cov_nd_rev": (_I, [_P, _P, _I, _I, _D, _D, _P, _I, _P]),
    "smg_add_diag_fwd": (_I, [_P, _P, _I, _I, _D, _P, _P, _I]),
    "smg_add_diag_rev": (_I, [_P, _P, _I, _I, _P, _I, _P, _I]),
    "smg_cholesky_block_size": (_I, [_I]),
    "smg_check_symmetric": (_I, [_P, _P, _I, _I]),
    "smg_cholesky_fwd": (_I, [_P, _P, _I, _I, _P, _I, _P]),
    "smg_cholesky_fwd_checked": (_I, [_P, _P, _I, _I, _P, _I, _P]),
    "smg_cholesky_fwd_checked_mark": (_I, [_P, _P, _I, _I, _P, _I, _P]),
    "smg_status_mark_wait": (_I, [_P, _P]),
    "smg_cholesky_rev": (_I, [_P, _P, _I, _P, _P, _I, _I, _P, _I]),
    "smg_mdivide_left_tri_fwd": (_I, [_P, _I, _P, _I, _P, _I, _I, _I, _P, _I]),
    "smg_mdivide_left_tri_rev": (_I, [_P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _P, _I, _P, _I, _P]),
    "smg_mdivide_left_tri_aux_fwd": (_I, [_P, _I, _P, _I, _P, _P, _I, _I, _I, _P, _I]),
    "smg_mdivide_left_tri_aux_rev": (_I, [_P, _I, _P, _I, _P, _P, _I, _P, _I, _I, _I, _P, _I, _P, _I, _P]),
    "smg_chol_tangent_fwd": (_I, [_P, _P, _I, _P, _P, _I, _I, _P, _P, _P, _P, _P, _I]),
    "smg_chol_tangent_fwd_w": (_I, [_P, _P, _I, _P, _P, _I, _I, _P, _P, _P, _P, _I]),
    "smg_chol_tangent_rev": (_I, [_P, _P, _I, _P, _P, _P, _P, _I, _P, _I, _I, _P, _I, _P, _I, _P]),
    "smg_multiply_lower_fwd": (_I, [_P, _P, _I, _P, _I, _I, _P, _I]),
    "smg_multiply_lower_rev": (_I, [_P, _P, _I, _P, _I, _P, _I, _I, _P, _I, _P, _I, _P]),
    "smg_multiply_fwd": (_I, [_P, _P, _I, _P, _I, _I, _I, _I, _P, _I]),
    "smg_multiply_rev": (_I, [_P, _P, _I, _P, _I, _P, _I, _I, _I, _I, _P, _I, _P, _I]),
    "smg_mvn_cholesky_fwd": (_I, [_P, _P, _P, _P, _I, _P, _I, _P, _P]),
    "smg_mvn_cholesky_rev": (_I, [_P, _P, _I, _P, _I, _P, _D, _I, _P, _P, _P, _I]),
    "smg_mvn_cholesky_fwd_inv": (_I, [_P, _P, _P, _P, _I, _P, _I, _I, _P, _P]),
    "smg_cholesky_inverse_wait": (_I, [_P]),
    "smg_cholesky_inverse_adjoint": (_I, [_P, _P, _I, _I, _P, _I, _L, _D, _P, _I]),
    "smg_cholesky_rev_inverse": (_I, [_P, _P, _I, _P, _P, _I, _P, _I, _I, _P, _I, _P]),
    "smg_gp_inverse_adjoint": (_I, [_P, _P, _I, _I, _P, _I, _L, _D, _P, _I, _P, _I, _D, _D, _P, _P]),
    "smg_cholesky_mvn_rev_ws_doubles": (ctypes.c_size_t, [_I]),
    "smg_cholesky_mvn_rev": (_I, [_P, _P, _I, _P, _I, _P, _I, _L, _D, _P, _I, _P]),
    "smg_cholesky_inv_t_async": (_I, [_P, _P, _I, _P, _I, _P, _I, _P]),
    "smg_cholesky_mvn_rev_v": (_I, [_P, _I, _P, _I, _L, _D, _P, _I, _P, _I]),
    "smg_cholesky_fwd_checked_mark_inv": (_I, [_P, _P, _I, _I, _P, _I, _P, _P, _P]),
    "smg_cholesky_fwd_checked_mark_winv": (_I, [_P, _P, _I, _I, _P, _I, _P, _P, _P]),
    "smg_trmv_inv": (_I, [_P, _I, _P, _I, _I, _P, _P]),
    "smg_rank1_lower": (_I, [_P, _I, _D, _P, _P, _P, _I]),
    "smg_cholesky_stream_panels": (_I, [_I]),
    "smg_cholesky_stream_panel_cols": (_I, [_I, _I, _P, _P]),
    "smg_sum_strict_upper": (_I, [_P, _I, _P, _I, _P]),
    "smg_cholesky_fwd_checked_mark_stream": (_I, [_P, _P, _I, _I, _P, _I, _P, _P, _P, _P, _P, _I]),
    "smg_log_sum_exp_fwd": (_I, [_P, _P, _L, _P]),
    "smg_log_sum_exp_rev": (_I, [_P, _P, _L, _D, _D, _P]),
    "smg_lgamma_fwd": (_I, [_P, _P, _L, _P]),
    "smg_lgamma_rev": (_I, [_P, _P, _L, _P, _P]),
    "smg_digamma_fwd": (_I, [_P, _P, _L, _P]),
    "smg_digamma_rev": (_I, [_P, _P, _L, _P, _P]),
    "smg_trigamma_fwd": (_I, [_P, _P, _L, _P]),
    "smg_normal_lpdf": (_I, [_P, _P, _I, _P, _I, _P, _I, _L, _I, _P, _P, _P, _P]),
    "smg_normal_lpdf_fused": (_I, [_P, _P, _P, _P, _D, _D, _D, _L, _I, _P, _P, _P, _P]),
    "smg_glm_ws_doubles": (_L, [_L, _I]),
    "smg_bernoulli_logit_glm": (_I, [_P, _P, _P, _L, _I, _L, _P, _P, _P]),
    "smg_normal_id_glm": (_I, [_P, _P, _P, _L, _I, _L, _P, _P, _P]),
    "smg_poisson_log_glm": (_I, [_P, _P, _P, _L, _I, _L, _P, _P, _P]),
    "smg_glm_categorical_ws_doubles": (_L, [_L, _I, _I]),
    "smg_categorical_logit_glm": (_I, [_P, _P, _P, _L, _I, _L, _I, _P, _P, _P]),
    "smg_mdivide_left_spd_fwd": (_I, [_P, _P, _I, _P, _I, _I, _I, _P, _P, _P, _I]),
    "smg_mdivide_left_spd_rev": (_I, [_P, _P, _P, _I, _I, _P, _I, _P, _I, _P, _I, _P, _I, _P]),
    "smg_log_determinant_spd_fwd": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "smg_log_determinant_spd_rev": (_I, [_P, _P, _P, _I, _D, _P, _I, _P]),
    "smg_log_determinant_fwd": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "smg_add_tril": (_I, [_P, _I, _I, _D, _P, _I, _P, _I]),
    "smg_copy_tril": (_I, [_P, _I, _I, _P, _I, _P, _I]),
    "smg_lse_tangent_fwd": (_I, [_P, _P, _P, _L, _P]),
    "smg_lse_tangent_rev": (_I, [_P, _P, _P, _L, _D, _D, _D, _P, _P]),
    "smg_glm_tangent_fwd": (_I, [_P, _P, _D, _P, _D, _P, _L, _P]),
    "smg_glm_tangent_rev": (_I, [_P, _P, _D, _P, _D, _P, _L, _D, _P, _P, _P]),
    "smg_log_determinant_rev": (_I, [_P, _P, _P, _I, _D, _P, _I, _P, _P]),
    "smg_multiply_lower_tri_self_transpose_fwd": (_I, [_P, _P, _I, _I, _I, _P, _I, _P]),
    "smg_multiply_lower_tri_self_transpose_rev": (_I, [_P, _P, _I, _I, _I, _P, _I, _P, _I, _P]),
    "smg_quad_form_sym_fwd": (_I, [_P, _P, _I, _P, _I, _I, _I, _P, _I, _P]),
    "smg_quad_form_sym_rev": (_I, [_P, _P, _I, _P, _I, _I, _I, _P, _I, _I, _P, _I, _P, _I, _P]),
    "smg_axpy": (_I, [_P, _L, _D, _P, _I, _P, _I]),
    "smg_axpy_dev": (_I, [_P, _L, _P, _P, _P]),
    "smg_sum": (_I, [_P, _P, _L, _P]),
    "smg_copy_matrix": (_I, [_P, _I, _I, _P, _I, _P, _I, _I, _I]),
    "smg_transpose": (_I, [_P, _I, _I, _P, _I, _P, _I, _D]),
    "smg_sym_from_lower": (_I, [_P, _I, _P, _I]),
    "smg_shift": (_I, [_P, _I, _I, _D, _P, _I, _I]),
    "smg_dot": (_I, [_P, _P, _P, _L, _P]),
    "smg_check_domain": (_I, [_P, _P, _L, _I, _P]),
    "smg_cholesky_aux_doubles": (_L, [_I]),
    "smg_gp_exp_quad_cov_tangent_fwd": (_I, [_P, _P, _I, _D, _D, _D, _D, _P, _I]),
    "smg_gp_exp_quad_cov_tangent_rev": (_I, [_P, _P, _I, _D, _D, _D, _D, _P, _I, _P]),
    "smg_phi": (_I, [_P, _I, _P, _I, _P, _I, _I]),
    "smg_diag_ratio_fwd": (_I, [_P, _I, _P, _I, _P, _I, _P]),
    "smg_diag_ratio_rev": (_I, [_P, _I, _P, _I, _P, _I, _D, _P, _I, _P, _I]),
    "smg_check_bounded_int": (_I, [_P, _P, _L, _I, _I, _P]),
    "smg_comm_unique_id": (_I, [ctypes.c_char_p]),
    "smg_comm_init": (_I, [_P, _I, _I, ctypes.c_char_p]),
    "smg_comm_allreduce_sum": (_I, [_P, _P, _L]),
    "smg_comm_allgather": (_I, [_P, _P, _L, _P]),
    "smg_comm_scatterv": (_I, [_P, _P, _P, _P, _I]),
    "smg_comm_destroy": (_I, [_P]),
}

_LIB = None


class SmgError(RuntimeError):
    pass


def lib():
    """Load libsmg_hip.so; raise loudly if it is missing (no CPU fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise SmgError(f"HIP extension not built: {LIB_PATH} (run __graft_entry__.build())")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = l
    return _LIB


def exported_symbols():
    return list(_SIGS)


def check(rc, what=""):
    if rc != SMG_OK:
        names = [v for k, v in STATUS.items() if rc & k]
        raise SmgError(f"{what}: smg status {rc} {names}")


def _np_ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


class Context:
    """One HIP stream + device bump arena (include/smg_hip.h, context section)."""

    def __init__(self, device=0, arena_bytes=1 << 30):
        self.lib = lib()
        n = _I(0)
        check(self.lib.smg_device_count(ctypes.byref(n)), "device_count")
        if n.value <= device:
            raise SmgError(f"no HIP device {device} (found {n.value})")
        p = _P()
        check(self.lib.smg_ctx_create(device, arena_bytes, ctypes.byref(p)), "ctx_create")
        self.ptr = p

    def close(self):
        if self.ptr:
            self.lib.smg_ctx_destroy(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- memory
    def alloc(self, nbytes):
        p = self.lib.smg_arena_alloc(self.ptr, max(int(nbytes), 8))
        if not p:
            raise SmgError("device arena exhausted")
        return p

    def zeros(self, n, dtype=np.float64):
        nbytes = int(n) * np.dtype(dtype).itemsize
        p = self.alloc(nbytes)
        check(self.lib.smg_memset(self.ptr, p, 0, max(nbytes, 1)), "memset")
        return p

    def put(self, a):
        a = np.ascontiguousarray(a)
        p = self.alloc(a.nbytes)
        check(self.lib.smg_memcpy_h2d(self.ptr, p, _np_ptr(a), a.nbytes), "h2d")
        self.sync()  # the numpy buffer may be freed right after
        return p

    def get(self, p, n, dtype=np.float64):
        out = np.empty(int(n), dtype=dtype)
        if out.nbytes:
            check(self.lib.smg_memcpy_d2h(self.ptr, _np_ptr(out), p, out.nbytes), "d2h")
        self.sync()
        return out

    def sync(self):
        check(self.lib.smg_sync(self.ptr), "sync")

    def status(self):
        s = _I(0)
        check(self.lib.smg_status(self.ptr, ctypes.byref(s)), "status")
        return s.value

    def mark(self):
        return self.lib.smg_arena_mark(self.ptr)

    def rewind(self, m):
        check(self.lib.smg_arena_rewind(self.ptr, m), "rewind")

    def call(self, name, *args):
        rc = getattr(self.lib, name)(self.ptr, *args)
        check(rc, name)
        return rc

    # ---- profiling
    def profile(self, on=True):
        check(self.lib.smg_profile_enable(self.ptr, 1 if on else 0), "profile")

    def profile_read(self, family):
        return profile_read(self.lib, self.ptr, family)


def profile_read(lib_, ctx_ptr, family):
    """(total ms, regions, algorithmic flops) of a kernel family on a context."""
    ms = _D(0)
    cnt = _L(0)
    fl = _D(0)
    check(lib_.smg_profile_read(ctx_ptr, FAMILIES[family], ctypes.byref(ms), ctypes.byref(cnt)), "profile_read")
    check(lib_.smg_profile_flops(ctx_ptr, FAMILIES[family], ctypes.byref(fl)), "profile_flops")
    return ms.value, cnt.value, fl.value
