"""The C ABI from plain C programs: tests/native/capi_smoke.c (appnp_propagate) and
tests/native/dist_smoke.c (the row-partitioned engine, two ranks as two threads on one GPU),
compiled with gcc against include/ppnp_amd.h and the HIP runtime here (CPU), executed on the
GPU box (-m gpu)."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
EXE = os.path.join(NATIVE, "capi_smoke")
DIST_EXE = os.path.join(NATIVE, "dist_smoke")


def build(name="capi_smoke"):
    exe = os.path.join(NATIVE, name)
    cmd = ["gcc", "-O2", "-std=c11", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT}/include",
           "-I/opt/rocm/include", os.path.join(NATIVE, name + ".c"), "-o", exe,
           f"-L{ROOT}/ppnp_amd", "-lppnp_amd", "-L/opt/rocm/lib", "-lamdhip64", "-lm",
           "-pthread", f"-Wl,-rpath,{ROOT}/ppnp_amd", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return exe


def test_capi_compiles_from_c():
    assert os.path.exists(build())
    assert os.path.exists(build("dist_smoke"))


@pytest.mark.gpu
def test_capi_runs_from_c():
    exe = EXE if os.path.exists(EXE) else build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "capi_smoke ok" in r.stdout


@pytest.mark.gpu
def test_dist_engine_runs_from_c():
    exe = DIST_EXE if os.path.exists(DIST_EXE) else build("dist_smoke")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "dist_smoke ok" in r.stdout
