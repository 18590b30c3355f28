#!/usr/bin/env python3
"""bench.py — gradient evals/sec (fp64) of the GP-marginal log-density, N=4096.

BASELINE.json metric: "gradient evals/sec (fp64), GP-marginal log-density
N=4096, 1->8 MI355X".  One step = one stan::math::gradient() of
  multi_normal_cholesky_lpdf(y | 0, cholesky_decompose(add_diag(
      gp_exp_quad_cov(x, alpha, rho), sigma^2)))
wrt (alpha, rho, sigma) through the header-only drop-in layer
(math_amd/include/stan/...) and libsmg_hip.so, inputs x, y = the reference
harness's config-3 inputs (tests/golden/gp_N4096.json), resident in HBM.

The GP does not shard (one dense factorisation): with --gpus N every rank runs
an independent replica on its own GPU ("replicas only"); value =
total evals over all ranks / max-over-ranks wall time.

Also reports, for the dominant kernel family (the fp64 MFMA GEMM), its
algorithmic flops / HIP-event time over a profiled copy of the timed region,
and the reference CPU path (oracle/_ref/ref_harness, the real Stan Math
3.0.0 compiled from /root/reference) timed on one host core.
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

PEAK_FP64_TFLOPS = 78.6  # MI355X fp64 (vector = matrix), MI355X_MICROARCH.md / BASELINE.md §3
N_GP = 4096


def load_inputs():
    with open(os.path.join(ROOT, "tests", "golden", f"gp_N{N_GP}.json")) as f:
        d = json.load(f)
    return (np.array(d["x"], dtype=np.float64), np.array(d["y"], dtype=np.float64),
            np.array(d["theta"], dtype=np.float64), d)


def cpu_baseline(timeout=300):
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    try:
        out = subprocess.run([exe, "bench", "gp", str(N_GP), "1"], capture_output=True, text=True,
                             timeout=timeout, env=dict(os.environ, OMP_NUM_THREADS="1"))
        r = json.loads(out.stdout.strip().splitlines()[-1])
        return {"value": r["evals_per_sec"], "unit": "gradient evals/s", "cores": 1, "kind": "reference",
                "sample": f"1 gradient eval of the GP marginal at N={N_GP} (Stan Math 3.0.0 compiled from "
                          f"/root/reference by oracle/Makefile; {r['seconds_per_eval']:.2f} s)"}
    except Exception as e:  # noqa: BLE001
        return {"value": None, "error": str(e)[:200]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # CPU-side barrier/max only (gloo); no data-path collective
        dist.init_process_group("gloo")

    from math_amd import hip
    bl = ctypes.CDLL(os.path.join(ROOT, "math_amd", "lib", "libsmg_bench.so"))
    bl.smg_bench_ctx.restype = ctypes.c_void_p
    bl.smg_bench_error.restype = ctypes.c_char_p
    D = ctypes.POINTER(ctypes.c_double)
    bl.smg_bench_gp_init.argtypes = [ctypes.c_int, ctypes.c_int, D, D]
    bl.smg_bench_gp_step.argtypes = [D, D, D]
    lib = hip.lib()

    x, y, theta, gold = load_inputs()
    p = lambda a: a.ctypes.data_as(D)  # noqa: E731
    if bl.smg_bench_gp_init(local, N_GP, p(x), p(y)) != 0:
        raise SystemExit(f"init failed: {bl.smg_bench_error().decode()}")
    ctx = ctypes.c_void_p(bl.smg_bench_ctx())
    fx = np.zeros(1)
    g = np.zeros(3)

    def step():
        if bl.smg_bench_gp_step(p(theta), p(fx), p(g)) != 0:
            raise SystemExit(f"step failed: {bl.smg_bench_error().decode()}")

    def barrier():
        if dist is not None:
            dist.barrier()

    def timed(k):
        barrier()
        lib.smg_sync(ctx)
        t0 = time.perf_counter()
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
    # parity guard on the measured configuration (reference golden values)
    rel = np.abs(g - np.array(gold["grad"])) / np.abs(np.array(gold["grad"]))
    if not (rel.max() < 1e-10 and abs(fx[0] - gold["fx"]) < 1e-9 * abs(gold["fx"])):
        raise SystemExit(f"parity failure: fx={fx[0]!r} grad={g} vs {gold['fx']} {gold['grad']}")

    t = timed(args.steps)
    evals = args.steps * world
    value = evals / t
    ms_per_step = 1e3 * t / args.steps

    # profiled copy of the timed region: HIP events on the context stream
    lib.smg_profile_enable(ctx, 1)
    tp = timed(args.steps)
    fams = {f: hip.profile_read(lib, ctx, f) for f in hip.FAMILIES}
    lib.smg_profile_enable(ctx, 0)
    gemm_ms, gemm_n, gemm_fl = fams["gemm"]
    achieved = gemm_fl / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else None

    line = {
        "metric": "gradient evals/sec (fp64), GP-marginal log-density N=4096",
        "value": value,
        "unit": "gradient evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (reference harness config-3 inputs: x~U(-10,10), y=sin(x)+0.3eps; theta=(1,1.5,0.3))",
        "config": {"workload": "gp_marginal_gradient", "N": N_GP, "kernel": "exp_quad",
                   "parallelism": f"replicas{world}", "path": "stan::math::gradient via header-only layer"},
        "roofline": {
            "bound": "mfma",
            "kernel": "k_gemm (fp64 MFMA, all launches of the family)",
            "achieved": achieved,
            "peak": PEAK_FP64_TFLOPS,
            "unit": "TFLOP/s",
            "frac": (achieved / PEAK_FP64_TFLOPS) if achieved else None,
            "traffic": None,
            "launches_per_step": gemm_n / args.steps,
            "flops_per_launch": gemm_fl / max(gemm_n, 1),
            "avg_launch_ms": gemm_ms / max(gemm_n, 1),
            "eval_achieved": (N_GP ** 3) / (tp / args.steps) / 1e12,
            "eval_frac": (N_GP ** 3) / (tp / args.steps) / 1e12 / PEAK_FP64_TFLOPS,
            "eval_flops": "N^3 (chol fwd N^3/3 + Murray adjoint 2N^3/3), SURVEY.md §8(d)",
        },
        "families_ms_per_step": {f: v[0] / args.steps for f, v in fams.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
