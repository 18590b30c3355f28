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
