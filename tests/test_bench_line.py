"""bench.py's contract on the GPU: the default (GP) line also carries the
north star's strong-scaling config, the config-4 GLM at the same number of
GPUs (glm_strong: 1e7 rows x 256 sharded over the ranks, one ncclAllReduce
per gradient; at one GPU through a one-rank RCCL communicator, the path
every rank of an 8-GPU run takes)."""
import json
import os
import subprocess
import sys

import pytest

from _util import ROOT


@pytest.mark.gpu
def test_bench_default_line_carries_glm_strong():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3",
                        "--warmup", "1", "--no-cpu-baseline"], capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["config"]["workload"] == "gp_marginal_gradient"
    g = d["glm_strong"]
    assert g["n_gpus"] == 1 and g["rows"] == 10_000_000 and g["rows_per_rank"] == 10_000_000
    assert g["scaling"] == "strong" and g["value"] > 0 and g["ms_per_step"] > 0
    assert "one-rank communicator" in g["config"]["parallelism"]
    r = g["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] < 1.0
    assert abs(r["bytes_per_launch"] - (1e7 * 256 * 8 + 1e7 * 4)) < 1
    # per-rank attribution of the GLM step (kernel / all-reduce / host), min / max over ranks
    pr = g["per_rank"]
    assert pr["ranks"] == 1 and abs(pr["allreduces_per_step"] - 1.0) < 1e-9
    for k in ("glm_kernel_ms", "allreduce_us", "host_and_gaps_us"):
        assert pr[k]["min"] <= pr[k]["max"] and len(pr[k]["per_rank"]) == 1
    assert 0 < pr["glm_kernel_ms"]["min"] < g["ms_per_step"] * 1.5
    assert pr["allreduce_us"]["min"] > 0
    # the whole job's value and gradient against the full-size fixture (guard passed, so within tolerance)
    rc = g["reference_check"]
    assert rc["fixture"] == "glm_R10000000_M256.json" and rc["fx_rel"] <= 1e-12 and rc["grad_rel"] <= 1e-10
    # the GP line's roofline: the dominant kernel (k_chol_panel) from HIP events,
    # its PMC bytes from the newest committed summary, the whole eval beside it
    gr = d["roofline"]
    assert gr["kernel"] == "k_chol_panel" and gr["bound"] == "mfma" and 0 < gr["frac"] < 1.0
    assert gr["avg_launch_us"] > 0 and abs(gr["launches_per_step"] - 8) < 1e-9
    assert gr["algorithmic_bytes_per_launch"] == 18874368.0
    import glob
    import re
    newest = max(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")),
                 key=lambda p: int(re.match(r"r(\d+)_", os.path.basename(p)).group(1)))
    assert gr["traffic_source"] == os.path.relpath(newest, ROOT)
    assert 0 < gr["eval"]["frac"] < 1.0
