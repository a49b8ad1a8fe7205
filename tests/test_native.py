"""The C ABI from a plain C program (tests/native/capi_smoke.c): compiled with gcc against
include/ppnp_amd.h and the HIP runtime here (CPU), executed on the GPU box (-m gpu)."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "capi_smoke.c")
EXE = os.path.join(ROOT, "tests", "native", "capi_smoke")


def build():
    cmd = ["gcc", "-O2", "-std=c11", "-D__HIP_PLATFORM_AMD__", f"-I{ROOT}/include",
           "-I/opt/rocm/include", SRC, "-o", EXE, f"-L{ROOT}/ppnp_amd", "-lppnp_amd",
           "-L/opt/rocm/lib", "-lamdhip64", "-lm", f"-Wl,-rpath,{ROOT}/ppnp_amd",
           "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return EXE


def test_capi_compiles_from_c():
    assert os.path.exists(build())


@pytest.mark.gpu
def test_capi_runs_from_c():
    exe = EXE if os.path.exists(EXE) else build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "capi_smoke ok" in r.stdout
