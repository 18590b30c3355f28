"""The header-only C++ stan::math layer (math_amd/include) driven end to end.

CPU part: the C++ test programs build and the C-ABI library exports every
symbol include/smg_hip.h declares.  GPU part: the programs run the GP
gradient through stan::math::gradient (device tape) and are compared with the
reference's golden values at 1e-10 relative (expect_near_rel semantics).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from _util import ROOT, golden, near_rel

BIN = os.path.join(ROOT, "tests", "cpp", "_bin")
LIB = os.path.join(ROOT, "math_amd", "lib", "libsmg_hip.so")


def _declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "smg_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(smg_[a-z0-9_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "build() must produce math_amd/lib/libsmg_hip.so"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (smg_[a-z0-9_]+)", out))
    missing = [s for s in _declared_symbols() if s not in exported]
    assert not missing, f"declared but not exported: {missing}"


def test_python_binding_covers_header():
    from math_amd import hip
    missing = [s for s in _declared_symbols() if s not in hip.exported_symbols()]
    assert not missing, missing


def test_cpp_programs_built():
    for name in ("test_gp_tape", "test_functors"):
        assert os.path.exists(os.path.join(BIN, name)), f"{name} not built (run __graft_entry__.build())"


def _run(name, stdin):
    p = subprocess.run([os.path.join(BIN, name)], input=stdin, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("N", [16, 256, 4096])
def test_gp_gradient_through_tape(N):
    d = golden(f"gp_N{N}")
    stdin = f"{N} " + " ".join(repr(float(v)) for v in d["theta"]) + "\n"
    stdin += " ".join(repr(float(v)) for v in d["x"]) + "\n" + " ".join(repr(float(v)) for v in d["y"]) + "\n"
    lines = [l.split() for l in _run("test_gp_tape", stdin).strip().splitlines()]
    for row in lines[:3]:  # std::vector twice (re-use of recovered arenas) + Eigen::VectorXd
        vals = np.array([float(v) for v in row])
        near_rel(vals[0], d["fx"], 1e-12, what="fx")
        near_rel(vals[1:], d["grad"], 1e-10, what="grad")
    assert lines[3] == ["stack", "0", "0"]  # nested tape fully recovered
