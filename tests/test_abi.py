"""CPU tests of the drop-in boundary: the in-tree C-ABI libraries load and
export every function include/*.h declares, unmangled, including every
symbol the reference's Rust FFI binds (bagua-core-internal/src/kernels/mod.rs:3-137)
and the C shim (bagua-core-c/src/lib.rs:9-69).  No compute calls (no GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "bagua-core_amd", "lib")

# every extern "C" function of bagua-core-internal/src/kernels/mod.rs:3-137
REFERENCE_KERNEL_FFI = [
    "divide_inplace_f32_host", "divide_inplace_f16_host", "average_inplace_f32_host", "average_inplace_f16_host",
    "substract_inplace_f32_host", "substract_inplace_f16_host", "add_inplace_f32_host", "add_inplace_f16_host",
    "addmul_inplace_f32_host", "addmul_inplace_f16_host", "reduce_mean_f32_inplace_host",
    "reduce_mean_f16_inplace_host", "reduce_sum_f32_inplace_host", "reduce_sum_f16_inplace_host",
    "compress_f32_to_uint8_host", "decompress_uint8_to_f32_host", "compress_f16_to_uint8_host",
    "decompress_uint8_to_f16_host", "array_min_max_size_f32_host", "array_min_max_size_f16_host",
    "async_model_average_host",
]
# bagua-core-c/src/lib.rs:9-69 (exported unmangled here)
REFERENCE_C_SHIM = ["bagua_single_communicator_c_create", "bagua_single_communicator_c_destroy",
                    "bagua_single_communicator_c_nranks"]


def declared(header: str) -> list[str]:
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src)
    skip = {"if", "for", "while", "return", "sizeof", "void"}  # "void (*callback)(...)" is a field
    return sorted({n for n in names if n not in skip})


def exported(so: str) -> set[str]:
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "bagua-core_amd")], check=True)
    return True


def test_kernels_header_fully_exported(built):
    syms = exported(os.path.join(LIB, "libbagua_kernels.so"))
    missing = [n for n in declared("bagua_kernels.h") if n not in syms]
    assert not missing, missing


def test_core_header_fully_exported(built):
    syms = exported(os.path.join(LIB, "libbagua_core.so"))
    missing = [n for n in declared("bagua_core.h") if n not in syms]
    assert not missing, missing


def test_reference_ffi_names_present(built):
    k = exported(os.path.join(LIB, "libbagua_kernels.so"))
    c = exported(os.path.join(LIB, "libbagua_core.so"))
    assert not [n for n in REFERENCE_KERNEL_FFI if n not in k]
    assert not [n for n in REFERENCE_C_SHIM if n not in c]


def test_python_binding_loads_and_declares_everything(built):
    import bagua_core
    from bagua_core import _native as N
    assert set(N.KERNEL_SIGNATURES) <= exported(N.KERNELS_PATH)
    assert set(N.CORE_SIGNATURES) <= exported(N.CORE_PATH)
    for name in ("BaguaTensorPy", "BaguaBucketPy", "BaguaCommBackendPy", "BaguaSingleCommunicatorPy"):
        assert hasattr(bagua_core, name)
    # pure host-side queries (no device work)
    assert N.K.bagua_minmax_u8_compressed_bytes(0, 1 << 26, 1) == 67108896
    assert N.K.bagua_minmax_u8_compressed_bytes(1, 1 << 20, 1) == (1 << 20) + 32
    assert N.K.bagua_onebit_compressed_bytes(1 << 26, 1) == 32 + (1 << 23)
    assert N.C.bagua_compressed_size(1, 0, 8, 1 << 25) == 268435712
    assert N.K.bagua_status_string(2) == b"workspace too small"
    assert N.C.bagua_dtype_bytes(N.DTYPE_BF16) == 2


def test_c_shim_null_safety(built):
    from bagua_core import _native as N
    h = ctypes.c_void_p(0)
    N.C.bagua_single_communicator_c_destroy(ctypes.byref(h))  # lib.rs:32-38: null is a no-op
    n = ctypes.c_size_t(7)
    assert N.C.bagua_single_communicator_c_nranks(ctypes.byref(h), ctypes.byref(n)) == -1  # lib.rs:58-62


def test_python_surface_rejects_cpu_and_bad_dtypes(built):
    import torch
    import bagua_core
    with pytest.raises(RuntimeError):
        bagua_core.BaguaTensorPy(torch.zeros(4, dtype=torch.float64, device="cpu"), "x")
    with pytest.raises(RuntimeError):
        bagua_core.BaguaTensorPy(torch.zeros(4), "cpu tensor")  # datatypes/mod.rs:629-633


def test_piece_ranges_cover_chunk(built):
    """bagua_minmax_u8_piece_range (host-only): pieces tile [0, cs) in order, 512-element aligned."""
    lib = ctypes.CDLL(os.path.join(LIB, "libbagua_kernels.so"))
    f = lib.bagua_minmax_u8_piece_range
    f.restype = ctypes.c_int
    b, e = ctypes.c_int(), ctypes.c_int()
    for cs, pieces in [(0, 1), (1, 4), (1536, 4), (40000, 3), (1 << 25, 4), (12345, 7)]:
        pos = 0
        for q in range(pieces):
            assert f(cs, pieces, q, ctypes.byref(b), ctypes.byref(e)) == 0
            assert b.value == pos and e.value >= b.value
            assert b.value % 512 == 0 or b.value == cs
            pos = e.value
        assert pos == cs
    assert f(10, 0, 0, ctypes.byref(b), ctypes.byref(e)) != 0
    assert f(10, 2, 2, ctypes.byref(b), ctypes.byref(e)) != 0
    assert f(10, 2 | (1 << 21), 0, ctypes.byref(b), ctypes.byref(e)) != 0  # unknown schedule bit


def test_tapered_piece_schedule(built):
    """BAGUA_PIECES_TAPERED in the schedule argument (no environment read): from 3 pieces on
    the first and the last piece are about half the others, edges 512-aligned, [0, cs) tiled."""
    from bagua_core import _native as N
    lib = ctypes.CDLL(os.path.join(LIB, "libbagua_kernels.so"))
    f = lib.bagua_minmax_u8_piece_range
    f.restype = ctypes.c_int
    ws = lib.bagua_minmax_u8_pipeline_workspace_bytes
    ws.restype = ctypes.c_size_t
    b, e = ctypes.c_int(), ctypes.c_int()
    for cs, pieces in [(1 << 25, 4), (1 << 25, 8), (40000, 5), (1536, 3), (0, 4)]:
        lens, pos = [], 0
        for q in range(pieces):
            assert f(cs, pieces | N.PIECES_TAPERED, q, ctypes.byref(b), ctypes.byref(e)) == 0
            assert b.value == pos and e.value >= b.value and (b.value % 512 == 0 or b.value == cs)
            lens.append(e.value - b.value)
            pos = e.value
        assert pos == cs
        if cs >= 512 * 8 * pieces:
            mid = lens[1]
            assert abs(lens[0] - mid / 2) <= 512 and abs(lens[-1] - mid / 2) <= 512, lens
        # plain and tapered schedules differ, and the workspace follows the schedule
        assert ws(cs, pieces | N.PIECES_TAPERED) > 0
    assert f(1 << 20, 2 | N.PIECES_TAPERED, 0, ctypes.byref(b), ctypes.byref(e)) == 0
    assert e.value == 1 << 19  # fewer than 3 pieces: tapering does not apply


def test_time_next_kernel_argument_check(built):
    """bagua_time_next_kernel needs both events or neither (host-only check)."""
    lib = ctypes.CDLL(os.path.join(LIB, "libbagua_kernels.so"))
    f = lib.bagua_time_next_kernel
    f.restype, f.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]
    assert f(None, None) == 0
    assert f(ctypes.c_void_p(16), None) == 1
    assert f(None, ctypes.c_void_p(16)) == 1
