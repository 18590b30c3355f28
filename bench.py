#!/usr/bin/env python3
"""bench.py — gradient evals/sec (fp64) of the BASELINE configs on MI355X.

Default workload (BASELINE.json metric, config 3): the GP-marginal
log-density at N=4096.  One step = one stan::math::gradient() of
  multi_normal_cholesky_lpdf(y | 0, cholesky_decompose(add_diag(
      gp_exp_quad_cov(x, alpha, rho), sigma^2)))
wrt (alpha, rho, sigma) through the header-only drop-in layer
(math_amd/include/stan/...) and libsmg_hip.so, inputs x, y = the reference
harness's config-3 inputs (tests/golden/gp_N4096.json), resident in HBM.
The GP does not shard (one dense factorisation): with --gpus N every rank runs
an independent replica ("replicas only"), value = total evals over
all ranks / max-over-ranks wall time.

--workload glm (config 4): bernoulli_logit_glm_lpmf gradient, R=1e7 rows x
M=256 covariates, rows partitioned over the ranks (row_partition), x and y
generated in HBM before the timed region, ONE RCCL all-reduce of the M+2
[logp, alpha', beta'] doubles per eval (strong scaling: fixed total work).

--workload mulchol (config 2): gradient of sum(cholesky_decompose(add_diag(
multiply(A, A^T), N))) wrt all N^2 entries of A, N=2048, A resident in HBM.

--workload gp_eigen: config 3 through the Eigen::Matrix<var> signatures
Stan-generated code uses (K, Kd, L materialised as host varis at every
stage and recognised again by the next functor), with the per-crossing cost.

--workload normal (config 1): gradient of normal_lpdf(theta | 0, 1), N=1024,
theta a host std::vector<var>: below the size gate (16384 elements) evaluated
on the host, as the reference keeps small calls off its device; the forced
device path (one fused launch + completion wait) is reported beside it.

--gpus N without an external launcher spawns N child processes (one per GPU,
torchrun's environment) before any GPU call; under torchrun WORLD_SIZE must
equal --gpus.

Each line carries the roofline (algorithmic flops or bytes
of one eval / the measured step time, or / the dominant kernel's HIP-event
launch time for the GLM; the GEMM family's executed flops beside it) and, on rank 0
at N=1, the reference CPU path (oracle/_ref/ref_harness: the real Stan Math
3.0.0 compiled from /root/reference) timed on one host core on a bounded sample.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6  # MI355X fp64 dense (vector = matrix), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0    # MI355X HBM3E, MI355X_MICROARCH.md
SEED = 20260101
D = ctypes.POINTER(ctypes.c_double)


def ptr(a):
    return a.ctypes.data_as(D)


def ref_bench(cfg, n, reps=1, timeout=300, threads=None):
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness" + ("_mt" if threads else ""))
    if not os.path.exists(exe):
        return None
    from math_amd import srchash
    srchash.check(exe, "ref")
    cmd = [exe, "bench", cfg, str(n), str(reps)] + ([str(threads)] if threads else [])
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=dict(os.environ, OMP_NUM_THREADS="1"))
    return json.loads(out.stdout.strip().splitlines()[-1])


def host_cores():
    """The host cores this process may use (the GPU box grants a 16-CPU share;
    os.cpu_count() shows the whole machine there)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def pmc_summary_path():
    """The newest committed PMC summary, profiles/rNN_pmc_traffic.json (highest
    round), or None."""
    import glob
    import re
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")):
        m = re.match(r"r(\d+)_pmc_traffic\.json$", os.path.basename(p))
        if m and (best is None or int(m.group(1)) > best[0]):
            best = (int(m.group(1)), p)
    return best[1] if best else None


def pmc_traffic(key):
    """HBM bytes per launch of kernel `key` (fetch + write, and the entry
    itself) from the newest committed PMC summary (tools/pmc_traffic.sh +
    tools/pmc_traffic.py: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes,
    calibrated on a known 8 B/lane stream), or (None, None, None)."""
    path = pmc_summary_path()
    try:
        with open(path) as f:
            e = json.load(f)[key]
        t = e.get("traffic_bytes_per_launch", e["fetch_bytes_per_launch"] + e["write_bytes_per_launch"])
        return t, os.path.relpath(path, ROOT), e
    except (OSError, KeyError, ValueError, TypeError):
        return None, None, None


def unif(seed, n, a, b):
    """oracle/gen.h SplitMix64 uniforms (numpy mirror, tests/gen.py)."""
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return a + (b - a) * ((z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0))


def panel_roofline(fams, steps, n):
    """The GP's dominant kernel, k_chol_panel (one persistent launch per 512
    columns): its in-panel work m b^2 - 2 b^3 / 3 per launch (m rows from the
    panel's top, b columns; SURVEY.md §8(d)'s N^3 / 3 forward, the part inside
    the panels) / its average launch time from HIP events around each launch
    (SMG_FAM_PANEL, the context stream in the profiled copy of the timed
    region), with the PMC bytes per launch and the algorithmic bytes
    16 (N - J) b per launch (read and write the panel once)."""
    pms, pn, pfl = fams["panel"]
    if pn <= 0 or pms <= 0:
        return None
    avg_ms = pms / pn
    fl = pfl / pn
    ach = fl / (avg_ms * 1e-3) / 1e12
    traffic, src, e = pmc_traffic("k_chol_panel")
    b = 512
    alg_bytes = sum(16.0 * (n - j) * min(b, n - j) for j in range(0, n, b)) / max(1, -(-n // b))
    return {"bound": "mfma", "kernel": "k_chol_panel", "achieved": ach, "peak": PEAK_FP64_TFLOPS,
            "unit": "TFLOP/s", "frac": ach / PEAK_FP64_TFLOPS, "traffic": traffic,
            "traffic_unit": "HBM bytes per k_chol_panel launch (PMC FETCH_SIZE + WRITE_SIZE)" if traffic else None,
            "traffic_source": src, "algorithmic_bytes_per_launch": alg_bytes,
            "traffic_over_algorithmic": traffic / alg_bytes if traffic else None,
            "flops_per_launch": fl, "avg_launch_us": 1e3 * avg_ms, "launches_per_step": pn / steps,
            "note": "latency-bound (the diagonal chain, DESIGN.md section 4), priced against the fp64 MFMA peak"}


def eval_roofline(wl, fams, steps, ms_per_step):
    """algorithmic flops of ONE gradient eval (the unit a step
    processes) / the measured step time / the fp64 MFMA peak.  The GEMM kernel
    family (HIP events on the context stream) is reported beside it with the
    flops its launches execute (block-inverse doubling and the symbolic
    adjoint's extra products included), named as such."""
    fl = wl.eval_flops()
    ach = fl / (ms_per_step * 1e-3) / 1e12
    gms, gn, gfl = fams["gemm"]
    return {"bound": "mfma", "kernel": "whole gradient eval (algorithmic flops / step time)",
            "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_FP64_TFLOPS,
            "algorithmic_flops_per_eval": fl, "eval_flops": wl.eval_flops_expr,
            "gemm_family": {"launches_per_step": gn / steps, "avg_launch_ms": gms / max(gn, 1),
                            "executed_flops_per_launch": gfl / max(gn, 1),
                            "executed_tflops": gfl / (gms * 1e-3) / 1e12 if gms > 0 else None,
                            "ms_per_step": gms / steps,
                            "note": "executed flops (incl. block-inverse doubling, symbolic-adjoint "
                                    "products); HIP events on the context stream"}}


class Workload:
    """init() puts the data in HBM; step() is one gradient eval; guard() checks parity."""
    unit = "gradient evals/s"

    def __init__(self, bl, args, rank, world, local, dist):
        self.bl, self.args, self.rank, self.world, self.local, self.dist = bl, args, rank, world, local, dist
        self.fx = np.zeros(1)


class GP(Workload):
    N = 4096
    metric = "gradient evals/sec (fp64), GP-marginal log-density N=4096"
    scaling = "weak"

    def init(self):
        bl = self.bl
        bl.smg_bench_gp_init.argtypes = [ctypes.c_int, ctypes.c_int, D, D]
        bl.smg_bench_gp_step.argtypes = [D, D, D]
        with open(os.path.join(ROOT, "tests", "golden", f"gp_N{self.N}.json")) as f:
            self.gold = json.load(f)
        self.x = np.array(self.gold["x"], dtype=np.float64)
        self.y = np.array(self.gold["y"], dtype=np.float64)
        self.theta = np.array(self.gold["theta"], dtype=np.float64)
        self.g = np.zeros(3)
        return bl.smg_bench_gp_init(self.local, self.N, ptr(self.x), ptr(self.y))

    def step(self):
        return self.bl.smg_bench_gp_step(ptr(self.theta), ptr(self.fx), ptr(self.g))

    def guard(self):
        want = np.array(self.gold["grad"])
        rel = np.abs(self.g - want) / np.abs(want)
        ok = rel.max() < 1e-10 and abs(self.fx[0] - self.gold["fx"]) < 1e-9 * abs(self.gold["fx"])
        return ok, f"fx={self.fx[0]!r} grad={self.g} vs {self.gold['fx']} {self.gold['grad']}"

    def units_per_step(self):
        return self.world  # one eval per replica

    def config(self):
        return {"workload": "gp_marginal_gradient", "N": self.N, "kernel": "exp_quad",
                "parallelism": f"replicas{self.world}", "path": "stan::math::gradient via header-only layer"}

    data = "synthetic (reference harness config-3 inputs: x~U(-10,10), y=sin(x)+0.3eps; theta=(1,1.5,0.3))"

    eval_flops_expr = ("N^3 (chol fwd N^3/3 + its adjoint 2N^3/3: Murray's, or under the MVN its closed form "
                       "V = L^-T N^3/3 + V V^T N^3/3), SURVEY.md §8(d)")

    def eval_flops(self):
        return float(self.N) ** 3

    def roofline(self, fams, steps, t_prof, ms_per_step):
        ev = eval_roofline(self, fams, steps, ms_per_step)
        pr = panel_roofline(fams, steps, self.N)
        if pr is None:  # (a path without panel launches)
            return ev
        pr["eval"] = ev
        return pr

    def extra(self, timed, steps):
        if type(self) is not GP:
            return {}
        # the headline functor takes x / y / mu device-resident (dev_data);
        # the reference's gp_functor passes std::vector x and Eigen y, mu:
        # the same evaluation with those argument types (uploaded per call)
        bl = self.bl
        bl.smg_bench_gp_step_reftypes.argtypes = [D, D, D]
        fx, g = np.zeros(1), np.zeros(3)
        step = lambda: bl.smg_bench_gp_step_reftypes(ptr(self.theta), ptr(fx), ptr(g))  # noqa: E731
        for _ in range(2):
            if step() != 0:
                raise SystemExit(f"reftypes step failed: {bl.smg_bench_error().decode()}")
        want = np.array(self.gold["grad"])
        if np.abs(g - want).max() > 1e-10 * np.abs(want).max():
            raise SystemExit(f"reftypes parity failure: {g} vs {want}")
        t = timed(steps, step)
        return {"reference_input_types": {
            "value": steps / t, "ms_per_step": 1e3 * t / steps,
            "note": "the same gradient with the reference harness's argument types (std::vector<double> x, "
                    "Eigen::VectorXd y and mu, uploaded each evaluation; intermediates auto = device nodes); "
                    "the headline line passes x / y / mu as dev_data"}}

    def cpu_baseline(self):
        r = ref_bench("gp", self.N, 1)
        if r is None:
            return None
        return {"value": r["evals_per_sec"], "unit": "gradient evals/s", "cores": 1, "kind": "reference",
                "sample": f"1 gradient eval of the GP marginal at N={self.N} (Stan Math 3.0.0 compiled "
                          f"from /root/reference by oracle/Makefile; {r['seconds_per_eval']:.2f} s)"}


class GPEigen(GP):
    """config 3 exactly as Stan-generated code declares it: `matrix[N,N] K`,
    Kd and L are Eigen::Matrix<var,-1,-1>, x a host std::vector, y and mu
    Eigen vectors (the reference harness's gp_functor, the CPU baseline's
    own code), so each stage crosses the Eigen boundary: every device output
    is materialised as N^2 host varis and recognised again by the next
    functor (stan/math/eigen/interop.hpp)."""
    metric = "gradient evals/sec (fp64), GP-marginal log-density N=4096, Eigen::Matrix<var> (Stan-codegen) signatures"

    def init(self):
        rc = super().init()
        self.bl.smg_bench_gp_eigen_step.argtypes = [D, D, D]
        self.bl.smg_bench_malloc_tuning.argtypes = [ctypes.c_int]
        self.bl.smg_bench_bridge_cost.argtypes = [ctypes.c_int, ctypes.c_int, D]
        self.malloc_tuning = int(os.environ.get("SMG_BENCH_MALLOC_TUNING", "1"))
        self.bl.smg_bench_malloc_tuning(self.malloc_tuning)
        return rc

    def step(self):
        return self.bl.smg_bench_gp_eigen_step(ptr(self.theta), ptr(self.fx), ptr(self.g))

    def config(self):
        c = super().config()
        c["workload"] = "gp_marginal_gradient_eigen_signatures"
        c["path"] = ("stan::math::gradient over Eigen::VectorXd theta; K, Kd, L declared Eigen::Matrix<var,-1,-1> "
                     "(3 materialisations of N^2 host varis + 3 recognitions per eval)")
        c["malloc_tuning"] = bool(self.malloc_tuning)
        return c

    def extra(self, timed, steps):
        ph = np.zeros(32)
        self.bl.smg_bench_gp_eigen_phases.argtypes = [D, D]
        best = None
        for _ in range(3):
            if self.bl.smg_bench_gp_eigen_phases(ptr(self.theta), ptr(ph)) != 0:
                raise SystemExit(f"gp_eigen phases failed: {self.bl.smg_bench_error().decode()}")
            if best is None or ph[3] < best[3]:
                best = ph.copy()
        out = np.zeros(5)
        if self.bl.smg_bench_bridge_cost(self.N, 3, ptr(out)) != 0:
            raise SystemExit(f"bridge cost failed: {self.bl.smg_bench_error().decode()}")
        # host-memory roofline of the three crossings: the bytes each writes
        # (varis + the Eigen pointer array) and reads (the staged values),
        # against a same-process probe of the same host pool's bandwidth
        bw = np.zeros(4)
        self.bl.smg_bench_host_bw.argtypes = [ctypes.c_longlong, ctypes.c_int, D]
        if self.bl.smg_bench_host_bw(1 << 29, 3, ptr(bw)) != 0:
            raise SystemExit(f"host bandwidth probe failed: {self.bl.smg_bench_error().decode()}")
        N, sv = self.N, float(bw[3])
        tri, nn = N * (N + 1) / 2, float(N) * N
        moved = {"forward_K": (tri * sv + nn * 8, tri * 8),     # K's own varis, pointers; staged values
                 "forward_Kd": (N * sv + nn * 8, 0.0),          # Kd's diagonal varis, pointers (K's shared)
                 "forward_L": (tri * sv + nn * 8, tri * 8)}     # L's varis, pointers; streamed values
        crossings = {}
        for k, (wb, rb) in moved.items():
            t = best[{"forward_K": 4, "forward_Kd": 5, "forward_L": 6}[k]]
            floor = (wb + rb) / (bw[0] * 1e9)
            crossings[k] = {"ms": t * 1e3, "bytes_written": wb, "bytes_read": rb,
                            "ms_at_probe_bandwidth": floor * 1e3, "frac_of_probe": floor / t if t > 0 else None}
        return {"eval_phases_ms": {"forward": best[0] * 1e3, "reverse_published": best[1] * 1e3,
                                   "recover": best[2] * 1e3, "gradient_call": best[3] * 1e3,
                                   "forward_K": best[4] * 1e3, "forward_Kd": best[5] * 1e3,
                                   "forward_L": best[6] * 1e3, "forward_mvn": best[7] * 1e3,
                                   "forward_L_timeline_ms": {
                                       "out_allocated": best[26] * 1e3, "candidate_found": best[27] * 1e3,
                                       "staging_ready": best[28] * 1e3, "enqueued": best[8] * 1e3,
                                       "input_verified": best[29] * 1e3, "pointers_filled": best[9] * 1e3,
                                       "panels_arrived": [round(t * 1e3, 4) for t in best[10:26:2] if t > 0],
                                       "panels_built": [round(t * 1e3, 4) for t in best[11:26:2] if t > 0],
                                       "status_read": best[31] * 1e3},
                                   "note": "one evaluation split by hand (functor forward incl. three crossings; "
                                           "a top-level grad() to a device sync, which also publishes the "
                                           "intermediate blocks' adjoints into their varis; recover_memory), best "
                                           "of 3; gradient_call: the same evaluation through stan::math::gradient "
                                           "(nothing published); forward_*: the forward's four statements"},
                "host_roofline": {"probe_write_GBps": bw[0], "probe_copy_GBps": bw[1], "pool_threads": int(bw[2]),
                                  "vari_bytes": int(bw[3]), "crossings": crossings,
                                  "note": "each crossing's bytes (written: varis + the Eigen pointer array; read: "
                                          "the staged values) at the probe's write bandwidth, over its measured "
                                          "time (forward_L overlaps the factorisation it streams from)"},
                "bridge_cost_ms": {"to_host_matrix": out[0] * 1e3, "to_dev_recognised": out[1] * 1e3,
                                   "to_dev_gathered_copy": out[2] * 1e3, "reverse_gather_touched": out[3] * 1e3,
                                   "reverse_untouched_sweep": out[4] * 1e3,
                                   "note": f"one crossing of an N={self.N} matrix, best of 3 "
                                           "(smg_bench_bridge_cost): the reverse sweeps of sum(A) + sum(B) with "
                                           "B = to_dev(to_host_matrix(A)), with / without a host node "
                                           "reading one element of the block"}}


class GLM(Workload):
    M = 256
    metric = "gradient evals/sec (fp64), bernoulli_logit_glm_lpmf 1e7 rows x 256"
    scaling = "strong"

    def init(self):
        bl = self.bl
        self.R = int(self.args.rows)
        bl.smg_bench_glm_init.argtypes = [ctypes.c_int, ctypes.c_longlong, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_char_p]
        bl.smg_bench_glm_step.argtypes = [D, D, D]
        bl.smg_bench_glm_local_rows.restype = ctypes.c_longlong
        comm_id = None
        # SMG_BENCH_GLM_RCCL1=1 at one GPU: a one-rank RCCL communicator, so the
        # step is the sharded path one rank of W runs (the per-rank proxy of
        # an 8-GPU run at --rows R/8)
        self.rccl1 = self.world == 1 and (getattr(self, "force_rccl1", False)
                                          or os.environ.get("SMG_BENCH_GLM_RCCL1") == "1")
        if self.rccl1:
            from math_amd import hip
            buf = ctypes.create_string_buffer(128)
            if hip.lib().smg_comm_unique_id(buf) != 0:
                raise SystemExit("smg_comm_unique_id failed")
            comm_id = bytes(buf.raw)
        if self.world > 1:  # RCCL unique id from rank 0, shared over the gloo group
            from math_amd import hip
            buf = ctypes.create_string_buffer(128)
            obj = [None]
            if self.rank == 0:
                if hip.lib().smg_comm_unique_id(buf) != 0:
                    raise SystemExit("smg_comm_unique_id failed")
                obj = [bytes(buf.raw)]
            self.dist.broadcast_object_list(obj, src=0)
            comm_id = obj[0]
        beta = unif(SEED + 43, self.M, -1.0, 1.0) * np.sqrt(3.0 / self.M)
        self.theta = np.concatenate([[0.1], beta])
        self.g = np.zeros(self.M + 1)
        # RCCL prints a version banner on stdout when the communicator comes
        # up: send it to stderr, so stdout carries only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            rc = bl.smg_bench_glm_init(self.local, self.R, self.M, self.rank, self.world, comm_id)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        self.rows = bl.smg_bench_glm_local_rows()
        return rc

    def step(self):
        return self.bl.smg_bench_glm_step(ptr(self.theta), ptr(self.fx), ptr(self.g))

    def guard(self):
        # deterministic (fixed-order reductions + one all-reduce): two evals bitwise equal
        fx0, g0 = self.fx.copy(), self.g.copy()
        self.step()
        ok = np.isfinite(fx0[0]) and fx0[0] == self.fx[0] and np.array_equal(g0, self.g)
        msg = f"fx {fx0[0]!r} vs {self.fx[0]!r}"
        # at config 4's size: the value and gradient of the whole job (all
        # ranks, after the all-reduce) against the CPU restatement over row
        # blocks (tests/golden/make_glm_full.py), fx 1e-12, gradient 1e-10
        path = os.path.join(ROOT, "tests", "golden", f"glm_R{self.R}_M{self.M}.json")
        if ok and os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            want = np.array(d["grad"])
            efx = abs(self.fx[0] - d["fx"]) / abs(d["fx"])
            eg = float(np.max(np.abs(self.g - want) / (np.abs(want) + np.abs(want).max())))
            ok = efx <= 1e-12 and eg <= 1e-10
            msg += f"; vs glm_R{self.R}_M{self.M}: fx rel {efx:.2e}, grad rel {eg:.2e}"
            self.reference_check = {"fixture": os.path.basename(path), "fx_rel": efx, "grad_rel": eg}
        return ok, msg

    def units_per_step(self):
        return 1  # one full-data gradient per step across all ranks

    def config(self):
        return {"workload": "bernoulli_logit_glm_gradient", "rows": self.R, "covariates": self.M,
                "rows_per_rank": int(self.rows),
                "parallelism": f"rows{self.world}+rccl_allreduce" + ("(one-rank communicator)" if self.rccl1 else ""),
                "path": "stan::math::gradient + reduce_sum_bernoulli_logit_glm via header-only layer"}

    data = "synthetic (reference harness config-4 streams: x~U(-sqrt3,sqrt3), y~Bern(0.5), generated in HBM)"

    def roofline(self, fams, steps, t_prof, ms_per_step):
        ms, n, _ = fams["glm"]
        byts = self.rows * self.M * 8 + self.rows * 4  # one read of x and y
        avg = ms / max(n, 1)
        ach = byts / (avg * 1e-3) / 1e9 if avg > 0 else None
        traffic, src, _ = pmc_traffic("glm")
        step_ms = t_prof * 1e3 / steps
        return {"bound": "hbm", "kernel": "k_glm_reg (one pass over x)", "achieved": ach,
                "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS if ach else None,
                "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC)", "traffic_source": src,
                "bytes_per_launch": byts, "avg_launch_ms": avg,
                "launches_per_step": n / steps,
                "step_minus_glm_kernels_us": (step_ms - ms / steps) * 1e3,
                "note_overhead": "profiled step time minus the GLM family's HIP-event time: host work "
                                 "(gradient() tape, one staged upload / download, one sync) + the "
                                 "partials reduction + launch gaps"}

    def cpu_baseline(self):
        # every host core, the reference's threaded map_rect
        # shape (32 row-shard jobs, their nested gradients in parallel on
        # thread-local tapes: oracle/_ref/ref_harness_mt, STAN_THREADS build)
        rs, cores = 2000000, host_cores()
        r = ref_bench("glm_mt", rs, 2, threads=cores)
        if r is None:
            return None
        per = r["seconds_per_eval"] * self.R / rs  # linear in rows (passes over x)
        return {"value": 1.0 / per, "unit": "gradient evals/s", "cores": r["threads"], "kind": "reference",
                "sample": f"2 gradient evals at {rs} rows x {self.M} as 32 map_rect-style row-shard jobs on "
                          f"{r['threads']} threads (Stan Math 3.0.0 with STAN_THREADS, "
                          f"{r['seconds_per_eval']:.3f} s each), scaled x{self.R // rs} to {self.R} rows "
                          "(linear in rows)"}


class MulChol(Workload):
    N = 2048
    metric = "gradient evals/sec (fp64), sum(cholesky(A A^T + N I)) N=2048"
    scaling = "weak"

    def init(self):
        bl = self.bl
        bl.smg_bench_mulchol_init.argtypes = [ctypes.c_int, ctypes.c_int]
        bl.smg_bench_mulchol_step.argtypes = [D, D]
        with open(os.path.join(ROOT, "tests", "golden", f"mulchol_N{self.N}.json")) as f:
            self.gold = json.load(f)
        self.sl = np.zeros(2)
        return bl.smg_bench_mulchol_init(self.local, self.N)

    def step(self, check=False):
        return self.bl.smg_bench_mulchol_step(ptr(self.fx), ptr(self.sl) if check else None)

    def guard(self):
        self.step(check=True)
        g = self.gold
        ok = (abs(self.fx[0] - g["fx"]) < 1e-11 * abs(g["fx"])
              and abs(self.sl[0] - g["grad_sum"]) < 1e-10 * g["grad_l2"] * 10
              and abs(self.sl[1] - g["grad_l2"]) < 1e-10 * g["grad_l2"])
        return ok, f"fx={self.fx[0]!r} sum={self.sl[0]!r} l2={self.sl[1]!r} vs {g['fx']} {g['grad_sum']} {g['grad_l2']}"

    def units_per_step(self):
        return self.world

    def config(self):
        return {"workload": "multiply_cholesky_gradient", "N": self.N, "parallelism": f"replicas{self.world}",
                "path": "stan::math::gradient (device-leaf) via header-only layer"}

    data = "synthetic (reference harness config-2 input: A = U(-1,1) sqrt(3/N), generated in HBM)"

    eval_flops_expr = ("7N^3 (fwd GEMM 2N^3 + rev 2 GEMM 4N^3 + chol N^3), SURVEY.md §8(d): the reference "
                       "algorithm's work; this build executes 4N^3 (the Gram product A A^T lower-only "
                       "forward, one reverse GEMM) + chol N^3")

    def eval_flops(self):
        return 7.0 * float(self.N) ** 3

    def roofline(self, fams, steps, t_prof, ms_per_step):
        r = eval_roofline(self, fams, steps, ms_per_step)
        # the same step time priced on the flops this build executes: the Gram
        # product lower-only 2N^3 -> N^3 ... (A A^T: N^3, reverse GEMM 2N^3,
        # chol fwd N^3/3 + Murray adjoint N^3)
        ex = (1.0 + 2.0 + 1.0 / 3.0 + 1.0) * float(self.N) ** 3
        ach = ex / (ms_per_step * 1e-3) / 1e12
        r["executed_flops_per_eval"] = ex
        r["executed_flops_expr"] = ("4.33N^3: forward Gram A A^T lower-only N^3 + reverse (A' = (S + S^T) A) "
                                    "2N^3 + Cholesky forward N^3/3 + Murray adjoint N^3")
        r["executed_achieved"] = ach
        r["frac_on_executed"] = ach / PEAK_FP64_TFLOPS
        return r

    def cpu_baseline(self):
        r = ref_bench("mulchol", self.N, 1)
        if r is None:
            return None
        return {"value": r["evals_per_sec"], "unit": "gradient evals/s", "cores": 1, "kind": "reference",
                "sample": f"1 gradient eval at N={self.N} (Stan Math 3.0.0, {r['seconds_per_eval']:.2f} s)"}


class HVP(GP):
    """config 5: hessian_times_vector of the GP marginal at N=4096, v = (1, -0.5, 0.25)."""
    metric = "hessian-vector products/sec (fp64), GP-marginal log-density N=4096"
    unit = "Hv products/s"

    def init(self):
        rc = super().init()
        self.bl.smg_bench_hvp_step.argtypes = [D, D, D, D]
        self.v = np.array([1.0, -0.5, 0.25])
        self.hv = np.zeros(3)
        return rc

    def step(self):
        return self.bl.smg_bench_hvp_step(ptr(self.theta), ptr(self.v), ptr(self.fx), ptr(self.hv))

    def guard(self):
        # no reference value at N=4096 (the reference's O(N^3) fvar tape is infeasible there);
        # parity is pinned at N<=256 (tests/test_cpp_functors.py); here: value = the GP's,
        # and two products bitwise equal (deterministic)
        if not np.any(self.hv):  # --warmup 0: no product has run yet
            self.step()
        h0 = self.hv.copy()
        self.step()
        ok = (abs(self.fx[0] - self.gold["fx"]) < 1e-9 * abs(self.gold["fx"])
              and np.array_equal(h0, self.hv) and np.all(np.isfinite(h0)))
        return ok, f"fx={self.fx[0]!r} Hv={h0} / {self.hv}"

    parity = ("value vs the reference golden at 1e-9; Hv at N=4096 self-consistent only (two products bitwise "
              "equal): the reference's fvar<var> tape is infeasible at N=4096; Hv pinned vs the reference at "
              "N<=256 in tests/test_cpp_functors.py")

    def config(self):
        c = super().config()
        c["workload"] = "gp_marginal_hessian_times_vector"
        c["v"] = [1.0, -0.5, 0.25]
        return c

    eval_flops_expr = "4N^3 (primal N^3 + tangent fwd N^3 + its reverse 2N^3), SURVEY.md §8(d)"

    def eval_flops(self):
        return 4.0 * float(self.N) ** 3

    def roofline(self, fams, steps, t_prof, ms_per_step):
        r = eval_roofline(self, fams, steps, ms_per_step)
        # the same step time priced on the flops the GEMM family executes per
        # product (each launch's flops, triangular K cuts counted, summed over
        # the profiled steps): measured, not a formula
        gms, gn, gfl = fams["gemm"]
        ex = gfl / steps
        ach = ex / (ms_per_step * 1e-3) / 1e12
        r["executed_flops_per_eval"] = ex
        r["executed_flops_expr"] = ("the GEMM family's executed flops per product (per-launch counts with the "
                                    "triangular K cuts, summed over the profiled steps): the value factor's forward "
                                    "and Murray adjoint, the Cholesky tangent node (W = L^-1, W A' W^T, L P and their "
                                    "reverse) and the MVN / solve products")
        r["executed_achieved"] = ach
        r["frac_on_executed"] = ach / PEAK_FP64_TFLOPS
        return r

    def cpu_baseline(self):
        # the reference's fvar<var> tape is O(N^3) scalar nodes: infeasible at N=4096 (~1.7 h);
        # the bounded sample is N=256, reported as measured (not extrapolated into `value`)
        r = ref_bench("hvp", 256, 1)
        if r is None:
            return None
        return {"value": None, "unit": "Hv products/s", "cores": 1, "kind": "reference",
                "sample": f"N=4096 infeasible on the reference; N=256 sample: {r['seconds_per_eval']:.2f} s "
                          f"per product ({r['evals_per_sec']:.3f}/s), Stan Math 3.0.0 compiled from /root/reference"}


class Normal(Workload):
    """config 1: gradient of normal_lpdf(theta | 0, 1), N=1024, theta a host
    std::vector<var> (the reference's normal_functor, prim/scal/prob/normal_lpdf.hpp:36-119)."""
    N = 1024
    metric = "gradient evals/sec (fp64), normal_lpdf N=1024"
    scaling = "weak"

    def init(self):
        bl = self.bl
        bl.smg_bench_device_init.argtypes = [ctypes.c_int]
        bl.smg_bench_normal_step.argtypes = [ctypes.c_int, D, D, D]
        bl.smg_bench_normal_gate.argtypes = [ctypes.c_longlong]
        bl.smg_bench_normal_run.argtypes = [ctypes.c_int, ctypes.c_int, D, D, D]
        with open(os.path.join(ROOT, "tests", "golden", f"normal_N{self.N}.json")) as f:
            self.gold = json.load(f)
        self.theta = np.array(self.gold["theta"], dtype=np.float64)
        self.g = np.zeros(self.N)
        # pointers and the bound entry made once: per-call ctypes conversions
        # would add several us to a ~20 us step
        self._call = bl.smg_bench_normal_step
        self._args = (self.N, ptr(self.theta), ptr(self.fx), ptr(self.g))
        return bl.smg_bench_device_init(self.local)

    def step(self):
        return self._call(*self._args)

    def run(self, k):
        """k evals in one native loop (no ctypes call per eval)"""
        return self.bl.smg_bench_normal_run(k, *self._args)

    def guard(self):
        want = np.array(self.gold["grad"])
        ok = (np.all(np.abs(self.g - want) <= 1e-10 * np.maximum(np.abs(want), 1e-10))
              and abs(self.fx[0] - self.gold["fx"]) <= 1e-12 * abs(self.gold["fx"]))
        return ok, f"fx={self.fx[0]!r} vs {self.gold['fx']}"

    def units_per_step(self):
        return self.world

    def config(self):
        return {"workload": "normal_lpdf_gradient", "N": self.N, "parallelism": f"replicas{self.world}",
                "path": "stan::math::gradient over std::vector<var> via header-only layer; N <= 16384 host "
                        "operands are evaluated on the host (size gate, as the reference gates its offload: "
                        "opencl/opencl_context.hpp:164-182)"}

    def extra(self, timed, steps):
        """the same eval forced through the fused device launch (gate 0)"""
        self.bl.smg_bench_normal_gate(0)
        for _ in range(3):
            self.step()
        ok, msg = self.guard()
        t = timed(steps)
        self.bl.smg_bench_normal_gate(16384)
        if not ok:
            raise SystemExit(f"parity failure (device path): {msg}")
        return {"device_path": {"value": steps * self.units_per_step() / t, "ms_per_step": 1e3 * t / steps,
                                "note": "one fused k_normal_fused launch + completion wait per eval "
                                        "(SMG_NORMAL_HOST_MAX=0)"}}

    data = "synthetic (reference harness config-1 input: theta ~ N(0,1), tests/golden/normal_N1024.json)"

    def roofline(self, fams, steps, t_prof, ms_per_step):
        byts = self.N * 8 * 2  # theta up, partials down (16 B per element)
        ach = byts / (ms_per_step * 1e-3) / 1e9
        return {"bound": "hbm", "kernel": "whole gradient eval (host-evaluated below the size gate: latency-bound, not HBM)",
                "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                "traffic": None, "bytes_per_eval": byts}

    def cpu_baseline(self):
        reps = 500000
        r = ref_bench("normal", self.N, reps)
        if r is None:
            return None
        return {"value": r["evals_per_sec"], "unit": "gradient evals/s", "cores": 1, "kind": "reference",
                "sample": f"{reps} gradient evals at N={self.N} (Stan Math 3.0.0, "
                          f"{r['seconds_per_eval'] * 1e6:.2f} us each)"}


WORKLOADS = {"gp": GP, "gp_eigen": GPEigen, "glm": GLM, "mulchol": MulChol, "hvp": HVP, "normal": Normal}


def _free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def spawn_ranks(n):
    """--gpus N without a launcher: start N fresh child processes, one per GPU,
    with the torchrun environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*),
    before this process touches the GPU; rank 0's stdout is the bench line."""
    import torch  # device_count() does not initialise the GPU on this image
    have = torch.cuda.device_count()
    if have < n:
        raise SystemExit(f"bench.py --gpus {n}: only {have} GPU(s) visible")
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [(r, rc) for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        raise SystemExit(f"bench.py: rank(s) failed: {bad}")
    return 0


def glm_strong(bl, args, rank, world, local, dist, timed, lib, ctx):
    """The north star's strong-scaling config in the default run: the config-4
    GLM (1e7 rows x 256, bernoulli_logit_glm_lpmf) on the same N GPUs, rows
    sharded (stan::math::row_partition), ONE ncclAllReduce of [logp, alpha',
    beta'] per gradient -- at N = 1 through a one-rank RCCL communicator, so
    every N runs the same sharded path.  The driver's 1..8-GPU runs of
    `bench.py --gpus N` thereby record the GLM's strong-scaling curve
    (value = gradient evals/s of the whole 1e7-row model) beside the GP
    replicas."""
    a = argparse.Namespace(**vars(args))
    a.rows = 1e7
    g = GLM(bl, a, rank, world, local, dist)
    g.force_rccl1 = True
    if g.init() != 0:
        raise SystemExit(f"glm_strong init failed: {bl.smg_bench_error().decode()}")
    for _ in range(3):
        if g.step() != 0:
            raise SystemExit(f"glm_strong step failed: {bl.smg_bench_error().decode()}")
    ok, msg = g.guard()
    if not ok:
        raise SystemExit(f"glm_strong parity failure: {msg}")
    steps = max(args.steps, 20)
    t = _timed_glm(g, steps, timed)
    lib.smg_profile_enable(ctx, 1)
    tp = _timed_glm(g, steps, timed)
    fams = {f: hip_profile_read(lib, ctx, f) for f in ("glm", "comm")}
    lib.smg_profile_enable(ctx, 0)
    roof = g.roofline(fams, steps, tp, 1e3 * t / steps)
    return {"metric": g.metric, "value": steps / t, "unit": g.unit, "n_gpus": world, "steps": steps,
            "ms_per_step": 1e3 * t / steps, "scaling": "strong", "rows": int(a.rows), "covariates": g.M,
            "rows_per_rank": int(g.rows), "config": g.config(),
            "roofline": {k: roof[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac",
                                              "bytes_per_launch", "avg_launch_ms", "step_minus_glm_kernels_us")},
            "per_rank": glm_rank_breakdown(fams, steps, tp, dist, world),
            "reference_check": getattr(g, "reference_check", None)}


def glm_rank_breakdown(fams, steps, t_prof, dist, world):
    """Where one rank's GLM step goes, per rank of the profiled copy of the
    timed region (HIP events on the context stream): the GLM kernels
    (k_glm_params + k_glm_reg + k_glm_io_final), the ncclAllReduce of the
    M + 2 sums, and the rest (host: the gradient() tape, the completion wait;
    launch gaps) -- with the min / max over ranks, so that an N-GPU run can
    attribute a shortfall to the kernel, the collective or the host."""
    gms, gn, _ = fams["glm"]
    cms, cn, _ = fams["comm"]
    step_ms = 1e3 * t_prof / steps
    mine = [gms / steps, 1e3 * cms / max(cn, 1), step_ms - gms / steps - cms / steps]
    rows = [mine]
    if dist is not None and world > 1:
        import torch
        out = [torch.zeros(3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(out, torch.tensor(mine, dtype=torch.float64))
        rows = [o.tolist() for o in out]
    keys = ("glm_kernel_ms", "allreduce_us", "host_and_gaps_us")
    scale = (1.0, 1.0, 1e3)

    def col(i):
        return [r[i] * scale[i] for r in rows]
    return {"ranks": len(rows), "allreduces_per_step": cn / steps,
            **{k: {"min": min(col(i)), "max": max(col(i)), "per_rank": col(i)} for i, k in enumerate(keys)},
            "note": "glm_kernel_ms per step; allreduce_us per ncclAllReduce (HIP events around the call on the "
                    "context stream: includes waiting for the other ranks); host_and_gaps_us per step = profiled "
                    "step time - both"}


def _timed_glm(g, steps, timed):
    """timed() over the GLM's step (the GP workload's timed() calls its own step)."""
    return timed(steps, g.step)


def hip_profile_read(lib, ctx, fam):
    from math_amd import hip
    return hip.profile_read(lib, ctx, fam)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="gp")
    ap.add_argument("--rows", type=float, default=1e7, help="GLM rows (config 4)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-glm-strong", action="store_true",
                    help="gp workload: skip the config-4 GLM strong-scaling line (glm_strong)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    dist = None
    if world > 1:
        import torch.distributed as dist  # CPU-side barrier / max / id exchange (gloo)
        dist.init_process_group("gloo")

    from math_amd import hip
    from math_amd import srchash
    bl_path = os.path.join(ROOT, "math_amd", "lib", "libsmg_bench.so")
    srchash.check(bl_path, "bench")  # (the GPU box cannot rebuild it: refuse a stale one)
    bl = ctypes.CDLL(bl_path)
    bl.smg_bench_ctx.restype = ctypes.c_void_p
    bl.smg_bench_error.restype = ctypes.c_char_p
    lib = hip.lib()
    wl = WORKLOADS[args.workload](bl, args, rank, world, local, dist)
    if wl.init() != 0:
        raise SystemExit(f"init failed: {bl.smg_bench_error().decode()}")
    ctx = ctypes.c_void_p(bl.smg_bench_ctx())

    def step():
        if wl.step() != 0:
            raise SystemExit(f"step failed: {bl.smg_bench_error().decode()}")

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(k, fn=None):
        barrier()
        lib.smg_sync(ctx)
        t0 = time.perf_counter()
        if fn is not None:
            for _ in range(k):
                if fn() != 0:
                    raise SystemExit(f"step failed: {bl.smg_bench_error().decode()}")
        elif hasattr(wl, "run"):
            if wl.run(k) != 0:
                raise SystemExit(f"step failed: {bl.smg_bench_error().decode()}")
        else:
            for _ in range(k):
                step()
        lib.smg_sync(ctx)
        t = time.perf_counter() - t0
        barrier()
        if dist is not None:
            import torch
            tt = torch.tensor([t], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            t = float(tt.item())
        return t

    for _ in range(args.warmup):
        step()
    ok, msg = wl.guard()  # parity guard on the measured configuration
    if not ok:
        raise SystemExit(f"parity failure: {msg}")

    t = timed(args.steps)
    value = args.steps * wl.units_per_step() / t
    ms_per_step = 1e3 * t / args.steps
    ok, msg = wl.guard()  # and on the last timed step
    if not ok:
        raise SystemExit(f"parity failure after the timed steps: {msg}")

    # profiled copy of the timed region: HIP events on the context stream
    lib.smg_profile_enable(ctx, 1)
    tp = timed(args.steps)
    fams = {f: hip.profile_read(lib, ctx, f) for f in hip.FAMILIES}
    lib.smg_profile_enable(ctx, 0)

    line = {
        "metric": wl.metric,
        "value": value,
        "unit": wl.unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": wl.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": wl.data,
        "config": wl.config(),
        "roofline": wl.roofline(fams, args.steps, tp, ms_per_step),
    }
    if hasattr(wl, "extra"):
        line.update(wl.extra(timed, args.steps))
    if getattr(wl, "parity", None):
        line["parity"] = wl.parity
    if getattr(wl, "reference_check", None):
        line["reference_check"] = wl.reference_check
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = wl.cpu_baseline()
        except Exception as e:  # noqa: BLE001
            line["cpu_baseline"] = {"value": None, "error": str(e)[:200]}
    strong = args.workload == "gp" and not args.no_glm_strong
    if strong:
        line["glm_strong"] = glm_strong(bl, args, rank, world, local, dist, timed, lib, ctx)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if (world > 1 and args.workload == "glm") or strong:
        lib.smg_comm_destroy(ctx)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
