"""A plain C program calling the drop-in boundary (tests/c_abi/abi_smoke.c):
the reference's v1 kernel names, the v2 status-returning entry points, and the
C shim + centralized op at one rank, every byte checked against the C oracle.
This is the caller a Rust / cgo / C host would be."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "c_abi", "build", "abi_smoke")


def test_c_program_links_against_the_c_abi():
    """CPU: the C test program is built (`__graft_entry__.build()` / `make -C tests/c_abi`)
    and resolves every library it needs."""
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c_abi")], check=True)
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True, check=True).stdout
    assert "not found" not in out, out
    assert "libbagua_core.so" in out and "libbagua_kernels.so" in out


@pytest.mark.gpu
def test_c_program_against_oracle():
    assert os.path.exists(BIN), "build tests/c_abi first (make -C tests/c_abi)"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "c abi smoke ok" in r.stdout
