"""Dev timing: GP N gradient composed through the C-ABI (no C++ tape)."""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import numpy as np
from math_amd import hip
from test_gpu_kernels import gp_gradient_abi
from _util import golden
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
d = golden(f"gp_N{N}")
ctx = hip.Context(0, 4 << 30)
ctx.profile(True)
for r in range(reps):
    m = ctx.mark()
    t = time.perf_counter()
    fx, g = gp_gradient_abi(ctx, d["x"], d["y"], d["theta"])
    ctx.sync()
    dt = time.perf_counter() - t
    ctx.rewind(m)
    print(f"rep {r}: {dt*1e3:.2f} ms fx={fx:.12g} g={g} ref={d['grad']}", flush=True)
for f in hip.FAMILIES:
    ms, c, fl = ctx.profile_read(f)
    print(f"{f:12s} {ms:9.3f} ms total  {c} regions")
