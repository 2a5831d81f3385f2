"""ctypes binding of the C ABI (include/bagua_kernels.h, include/bagua_core.h).

The product path always runs through the in-tree HIP libraries
`bagua-core_amd/lib/libbagua_kernels.so` and `libbagua_core.so`.  There is
no CPU or PyTorch fallback: if the libraries are missing the import fails
loudly (build them with `make -C bagua-core_amd` or
`python -c "import __graft_entry__ as g; g.build()"`).
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first: our libs bind to the same libamdhip64.so.7)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(_PKG_ROOT, "lib")
KERNELS_PATH = os.path.join(LIB_DIR, "libbagua_kernels.so")
CORE_PATH = os.path.join(LIB_DIR, "libbagua_core.so")

for _p in (KERNELS_PATH, CORE_PATH):
    if not os.path.exists(_p):
        raise ImportError(
            f"bagua_core: native library {_p} is missing; build it with `make -C {_PKG_ROOT}` "
            "(no CPU fallback exists by design)")

kernels = ctypes.CDLL(KERNELS_PATH, mode=ctypes.RTLD_GLOBAL)
core = ctypes.CDLL(CORE_PATH, mode=ctypes.RTLD_GLOBAL)
try:  # the per-tensor scheduler calls without ctypes (csrc/pyext/fastpath.c, links libbagua_core.so)
    from . import _fastpath as FAST
except ImportError as _e:
    raise ImportError(f"bagua_core: the fast-path extension is missing; build it with `make -C {_PKG_ROOT}`") from _e

# dtype / method / op codes (bagua_kernels.h, bagua_core.h)
DTYPE_F32, DTYPE_F16, DTYPE_BF16, DTYPE_U8, DTYPE_I64, DTYPE_U64 = 0, 1, 2, 3, 4, 5
COMPRESSION_NONE, COMPRESSION_MINMAX_UINT8, COMPRESSION_ONEBIT = 0, 1, 2
# piece schedules (bagua_kernels.h): a count, optionally OR-ed with PIECES_TAPERED
PIECES_COUNT_MASK, PIECES_TAPERED, PIECES_MULTIPATH, PIECES_FOLDED, PIECES_TABLES = (0xFFFF, 0x10000, 0x20000, 0x40000,
                                                                                   0x80000)
OP_SUM, OP_PROD, OP_MIN, OP_MAX, OP_AVG = 0, 1, 2, 3, 10

STATUS = {0: "ok", 1: "invalid argument", 2: "workspace too small", 3: "HIP launch failed",
          4: "unsupported dtype or layout", 16: "RCCL error", 17: "out of device memory", 18: "communicator aborted"}


class bagua_tensor_t(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_uint64), ("num_elem", ctypes.c_uint64), ("num_elem_allocated", ctypes.c_uint64),
                ("dtype", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class bagua_bucket_op_t(ctypes.Structure):
    """include/bagua_core.h bagua_bucket_op_t"""
    _fields_ = [("kind", ctypes.c_int32), ("average", ctypes.c_int32), ("compression", ctypes.c_int32),
                ("fused", ctypes.c_int32), ("comm", ctypes.c_void_p), ("weight", bagua_tensor_t),
                ("left_peer_weight", bagua_tensor_t), ("right_peer_weight", bagua_tensor_t),
                ("callback", ctypes.c_void_p), ("user", ctypes.c_void_p), ("intranode", ctypes.c_void_p)]


BUCKET_OP_CENTRALIZED_LOW_PRECISION, BUCKET_OP_CENTRALIZED_FULL_PRECISION = 1, 2
BUCKET_OP_DECENTRALIZED_LOW_PRECISION, BUCKET_OP_CALLBACK = 3, 4
STATUS_INVALID_ARG = 1

_T = ctypes.POINTER(bagua_tensor_t)
_vp, _sz, _i32, _u64, _f32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64, ctypes.c_float
_C = ctypes.c_void_p  # BaguaSingleCommunicatorC*


def _sig(lib, name, restype, argtypes):
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


# ---- libbagua_kernels (C ABI v2 + v1) ---------------------------------------
KERNEL_SIGNATURES = {
    "bagua_status_string": (ctypes.c_char_p, [_i32]),
    "bagua_last_hip_error": (_i32, []),
    "bagua_time_next_kernel": (_i32, [_vp, _vp]),
    "bagua_time_next_kernels": (_i32, [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _i32]),
    "bagua_timed_kernels": (_i32, []),
    "bagua_timed_kernel_name": (_i32, [_i32, ctypes.c_char_p, ctypes.c_size_t]),
    "bagua_minmax_u8_compressed_bytes": (_sz, [_i32, _i32, _i32]),
    "bagua_minmax_u8_workspace_bytes": (_sz, [_i32, _i32]),
    "bagua_minmax_u8_compress": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]),
    "bagua_minmax_u8_decompress": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _vp]),
    "bagua_minmax_u8_compress_stage": (_i32, [_i32, _i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]),
    "bagua_minmax_u8_resident_path": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _i32, _vp]),
    "bagua_minmax_u8_resident_trace": (_i32, [_vp]),
    "bagua_minmax_u8_release_stream": (_i32, [_vp]),
    "bagua_minmax_u8_set_stream_resident": (_i32, [_vp, _i32]),
    "bagua_minmax_u8_centralized_one_rank": (_i32, [_i32, _vp, _i32, _i32, _vp, _sz, _vp]),
    "bagua_onebit_one_rank_workspace_bytes": (_sz, [_i32]),
    "bagua_onebit_centralized_one_rank": (_i32, [_i32, _vp, _i32, _i32, _vp, _sz, _vp]),
    "bagua_minmax_u8_resident_slots_in_use": (_i32, [_i32]),
    "bagua_minmax_u8_resident_give_ups": (_i32, [_vp, ctypes.POINTER(_u64)]),
    "bagua_minmax_u8_decompress_reduce": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _vp]),
    "bagua_minmax_u8_reduce_requantize": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _vp, _sz, _i32, _vp, _sz,
                                                 _vp]),
    "bagua_minmax_u8_reduce_requantize_final": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _vp, _sz, _i32, _vp,
                                                       _sz, _vp]),
    "bagua_minmax_u8_piece_range": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "bagua_minmax_u8_pipeline_workspace_bytes": (_sz, [_i32, _i32]),
    "bagua_minmax_u8_quantize_range": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _i32, _i32,
                                              _vp]),
    "bagua_minmax_u8_decompress_range": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _i32, _vp]),
    "bagua_minmax_u8_reduce_piece": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _i32, _i32, _i32, _vp, _sz, _vp]),
    "bagua_minmax_u8_requantize_pieces": (_i32, [_i32, _vp, _i32, _i32, _vp, _sz, _i32, _i32, _vp, _sz, _vp]),
    "bagua_minmax_u8_requantize_piece": (_i32, [_i32, _vp, _i32, _i32, _vp, _sz, _i32, _i32, _i32, _vp, _sz, _vp]),
    "bagua_minmax_u8_reduce_requantize_piece": (_i32, [_i32, _vp, _sz, _i32, _i32, _i32, _vp, _sz, _i32, _i32, _i32,
                                                        _vp, _sz, _vp]),
    "bagua_minmax_u8_fold_piece_partials": (_i32, [_i32, _i32, _i32, _vp, _sz, _vp]),
    "bagua_ring_mix_minmax": (_i32, [_i32, _vp, _vp, _vp, _vp, _i32, _vp, _sz, _vp]),
    "bagua_ring_apply_minmax": (_i32, [_i32, _vp, _vp, _vp, _sz, _i32, _vp, _vp, _vp, _vp, _vp]),
    "bagua_ring_apply_minmax_range": (_i32, [_i32, _vp, _vp, _vp, _sz, _i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp]),
    "bagua_ring_one_rank_minmax": (_i32, [_i32, _vp, _vp, _vp, _vp, _i32, _vp, _sz, _vp]),
    "bagua_onebit_compressed_bytes": (_sz, [_i32, _i32]),
    "bagua_onebit_workspace_bytes": (_sz, [_i32, _i32]),
    "bagua_onebit_compress": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]),
    "bagua_onebit_decompress": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _vp]),
    "bagua_onebit_reduce_requantize": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _vp, _sz, _i32, _vp, _sz,
                                              _vp]),
    "bagua_onebit_piece_range": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "bagua_onebit_encode_range": (_i32, [_i32, _vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _i32, _vp]),
    "bagua_onebit_finalize": (_i32, [_vp, _sz, _i32, _i32, _i32, _vp, _sz, _vp]),
    "bagua_onebit_decompress_range": (_i32, [_i32, _vp, _sz, _i32, _i32, _vp, _i32, _i32, _vp]),
    "bagua_reduce_chunks": (_i32, [_i32, _vp, _i32, _i32, _i32, _i32, _vp]),
    "bagua_add_inplace": (_i32, [_i32, _vp, _vp, _i32, _vp]),
    "bagua_addmul_inplace": (_i32, [_i32, _vp, _vp, _i32, _f32, _vp]),
    "bagua_substract_inplace": (_i32, [_i32, _vp, _vp, _i32, _vp]),
    "bagua_average_inplace": (_i32, [_i32, _vp, _vp, _i32, _vp]),
    "bagua_divide_inplace": (_i32, [_i32, _vp, _f32, _i32, _vp]),
    # v1 names (bagua_kernels.cu:573-691), declared for the export check and direct use
    "compress_f32_to_uint8_host": (None, [_vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]),
    "decompress_uint8_to_f32_host": (None, [_vp, _sz, _i32, _i32, _vp, _vp]),
    "compress_f16_to_uint8_host": (None, [_vp, _i32, _i32, _i32, _vp, _sz, _vp, _sz, _i32, _vp]),
    "decompress_uint8_to_f16_host": (None, [_vp, _sz, _i32, _i32, _vp, _vp]),
    "array_min_max_size_f32_host": (_sz, [_vp, _i32, _vp, _vp]),
    "array_min_max_size_f16_host": (_sz, [_vp, _i32, _vp, _vp]),
    "reduce_mean_f32_inplace_host": (None, [_vp, _i32, _i32, _i32, _vp]),
    "reduce_mean_f16_inplace_host": (None, [_vp, _i32, _i32, _i32, _vp]),
    "reduce_sum_f32_inplace_host": (None, [_vp, _i32, _i32, _i32, _vp]),
    "reduce_sum_f16_inplace_host": (None, [_vp, _i32, _i32, _i32, _vp]),
    "add_inplace_f32_host": (None, [_vp, _vp, _i32, _vp]),
    "add_inplace_f16_host": (None, [_vp, _vp, _i32, _vp]),
    "addmul_inplace_f32_host": (None, [_vp, _vp, _i32, _f32, _vp]),
    "addmul_inplace_f16_host": (None, [_vp, _vp, _i32, _f32, _vp]),
    "substract_inplace_f32_host": (None, [_vp, _vp, _i32, _vp]),
    "substract_inplace_f16_host": (None, [_vp, _vp, _i32, _vp]),
    "average_inplace_f32_host": (None, [_vp, _vp, _i32, _vp]),
    "average_inplace_f16_host": (None, [_vp, _vp, _i32, _vp]),
    "divide_inplace_f32_host": (None, [_vp, _f32, _i32, _vp]),
    "divide_inplace_f16_host": (None, [_vp, _f32, _i32, _vp]),
    "async_model_average_host": (None, [_vp, _vp, _vp, _f32, _i32, _vp]),
}

CORE_SIGNATURES = {
    "bagua_dtype_bytes": (_sz, [_i32]),
    "bagua_memcpy_device_to_host_sync": (_i32, [_vp, _u64, _sz]),
    "bagua_stream_wait_event": (_i32, [_u64, _u64]),
    "bagua_pool_alloc": (_i32, [_i32, _sz, ctypes.POINTER(ctypes.c_uint64)]),
    "bagua_pool_free": (_i32, [_u64]),
    "bagua_pool_free_after": (_i32, [_u64, ctypes.POINTER(ctypes.c_uint64), _i32]),
    "bagua_pool_trim": (_i32, [_i32]),
    "bagua_pool_bytes_pending": (_sz, [_i32]),
    "bagua_pool_capture_begin": (_vp, []),
    "bagua_pool_capture_end": (_i32, [_vp]),
    "bagua_pool_capture_release": (_i32, [_vp]),
    "bagua_release_stream_resources": (_i32, [_i32, _u64]),
    "bagua_stream_workspace_count": (_sz, []),
    "bagua_pool_bytes_in_use": (_sz, [_i32]),
    "bagua_pool_bytes_cached": (_sz, [_i32]),
    "bagua_compressed_size": (_sz, [_i32, _i32, _sz, _sz]),
    "bagua_tensor_compress": (_i32, [_T, _i32, _i32, _u64, _i32, _T]),
    "bagua_tensor_compress_into": (_i32, [_T, _i32, _i32, _u64, _i32, _T]),
    "bagua_tensor_decompress_from": (_i32, [_T, _i32, _i32, _T, _u64]),
    "bagua_tensor_reduce_inplace": (_i32, [_T, _i32, _i32, _i32, _u64]),
    "bagua_tensor_add_inplace": (_i32, [_T, _T, _u64]),
    "bagua_tensor_addmul_inplace": (_i32, [_T, _T, _f32, _u64]),
    "bagua_tensor_clone_from": (_i32, [_T, _T, _u64]),
    "bagua_single_communicator_c_create": (_C, [_sz, _sz, _sz, _u64, ctypes.c_char_p]),
    "bagua_single_communicator_c_destroy": (None, [ctypes.POINTER(_C)]),
    "bagua_single_communicator_c_nranks": (ctypes.c_int32, [ctypes.POINTER(_C), ctypes.POINTER(_sz)]),
    "bagua_single_communicator_c_rank": (ctypes.c_int32, [ctypes.POINTER(_C), ctypes.POINTER(_sz)]),
    "bagua_single_communicator_c_stream": (_u64, [_C]),
    "bagua_generate_nccl_unique_id_str": (_i32, [ctypes.c_char_p, _sz]),
    "bagua_comm_abort": (_i32, [_C]),
    "bagua_comm_check_abort": (_i32, [_C]),
    "bagua_comm_allreduce_inplace": (_i32, [_C, _T, _i32]),
    "bagua_comm_allreduce": (_i32, [_C, _T, _T, _i32]),
    "bagua_comm_broadcast": (_i32, [_C, _T, _i32]),
    "bagua_comm_reduce_inplace": (_i32, [_C, _T, _i32, _i32]),
    "bagua_comm_reduce": (_i32, [_C, _T, _T, _i32, _i32]),
    "bagua_centralized_low_precision_hierarchical": (_i32, [_C, _C, _T, _i32, _i32]),
    "bagua_centralized_full_precision_hierarchical": (_i32, [_C, _C, _T, _i32]),
    "bagua_decentralized_low_precision_hierarchical": (_i32, [_C, _C, _T, _T, _T, _T, _i32]),
    "bagua_comm_alltoall": (_i32, [_C, _T, _T]),
    "bagua_comm_alltoall_inplace": (_i32, [_C, _T]),
    "bagua_comm_allgather_inplace": (_i32, [_C, _T]),
    "bagua_comm_allgather": (_i32, [_C, _T, _T]),
    "bagua_comm_send": (_i32, [_C, _T, _i32]),
    "bagua_comm_recv": (_i32, [_C, _T, _i32]),
    "bagua_comm_group_start": (_i32, []),
    "bagua_comm_group_end": (_i32, []),
    "bagua_comm_barrier": (_i32, [_C]),
    "bagua_comm_synchronize": (_i32, [_C]),
    "bagua_comm_set_async": (_i32, [_C, _i32]),
    "bagua_loopback_group_create": (_vp, [_i32, _i32]),
    "bagua_loopback_group_destroy": (None, [_vp]),
    "bagua_loopback_communicator_create": (_C, [_vp, _sz, _u64]),
    "bagua_centralized_low_precision_synchronous": (_i32, [_C, _T, _i32, _i32]),
    "bagua_centralized_low_precision_synchronous_unfused": (_i32, [_C, _T, _i32, _i32]),
    "bagua_centralized_low_precision_pipelined": (_i32, [_C, _T, _i32, _i32, _i32]),
    "bagua_centralized_full_precision_synchronous": (_i32, [_C, _T, _i32]),
    "bagua_decentralized_low_precision_synchronous": (_i32, [_C, _T, _T, _T, _T, _i32]),
    "bagua_decentralized_low_precision_synchronous_unfused": (_i32, [_C, _T, _T, _T, _T, _i32]),
    "bagua_decentralized_low_precision_pipelined": (_i32, [_C, _T, _T, _T, _T, _i32, _i32]),
    "bagua_ring_exchange_plan": (_i32, [_i32, _i32, _i32, _i32, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_sz)]),
    "bagua_bucket_create": (_vp, [ctypes.c_char_p, _T, ctypes.POINTER(ctypes.c_char_p), _i32, ctypes.POINTER(_i32)]),
    "bagua_bucket_destroy": (None, [_vp]),
    "bagua_bucket_append_op": (_i32, [_vp, ctypes.POINTER(bagua_bucket_op_t)]),
    "bagua_bucket_clear_ops": (_i32, [_vp]),
    "bagua_bucket_num_ops": (_i32, [_vp]),
    "bagua_bucket_mark_tensor_ready": (_i32, [_vp, ctypes.c_char_p, _u64]),
    "bagua_bucket_mark_tensor_ready_desc": (_i32, [_vp, ctypes.c_char_p, _u64, _T]),
    "bagua_bucket_refresh_tensor": (_i32, [_vp, ctypes.c_char_p, _T]),
    "bagua_bucket_ready_for_comm": (_i32, [_vp]),
    "bagua_bucket_reset_comm_ready": (_i32, [_vp]),
    "bagua_bucket_execute": (_i32, [_vp, _u64]),
    "bagua_comm_backend_create": (_vp, [_sz, _i32]),
    "bagua_comm_backend_destroy": (None, [_vp]),
    "bagua_comm_backend_register_ordered_buckets": (_i32, [_vp, ctypes.POINTER(_vp), _i32]),
    "bagua_comm_backend_mark_communication_ready": (_i32, [_vp, ctypes.c_char_p, _u64]),
    "bagua_comm_backend_mark_communication_ready_desc": (_i32, [_vp, ctypes.c_char_p, _u64, _T]),
    "bagua_comm_backend_wait_pending_comm_ops": (_i32, [_vp, ctypes.POINTER(_i32)]),
    "bagua_comm_backend_failures": (_i32, [_vp]),
    "bagua_comm_backend_stuck": (_i32, [_vp]),
    "bagua_comm_schedule_config": (_i32, [_vp, ctypes.POINTER(ctypes.c_int32), _i32]),
    "bagua_comm_backend_failure_message": (_i32, [_vp, _i32, ctypes.c_char_p, _sz]),
    "bagua_comm_backend_set_op_timeout_ms": (_i32, [_vp, ctypes.c_int64]),
    "bagua_comm_backend_set_lanes": (_i32, [_vp, _i32]),
    "bagua_comm_backend_lanes": (_i32, [_vp]),
    "bagua_ring_exchange_ops": (_i32, [_i32, _i32, _i32, _i32, _i32, _i32, _vp, _i32]),
}

K = type("K", (), {})()
C = type("C", (), {})()
for _n, (_r, _a) in KERNEL_SIGNATURES.items():
    setattr(K, _n, _sig(kernels, _n, _r, _a))
for _n, (_r, _a) in CORE_SIGNATURES.items():
    setattr(C, _n, _sig(core, _n, _r, _a))


class BaguaNativeError(RuntimeError):
    pass


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = STATUS.get(rc, f"status {rc}")
        if rc == 3:
            msg += f" (hipError {K.bagua_last_hip_error()})"
        raise BaguaNativeError(f"{what} failed: {msg}")


def time_next_kernels(events) -> None:
    """arm the kernel library's timing hook for len(events) launches on this thread:
    events = [(start, stop), ...] of torch.cuda.Event(enable_timing=True), already recorded once"""
    n = len(events)
    st = (_vp * max(1, n))(*[a.cuda_event for a, _ in events])
    sp = (_vp * max(1, n))(*[b.cuda_event for _, b in events])
    check(K.bagua_time_next_kernels(st, sp, n), "time_next_kernels")


def timed_kernel_names() -> list:
    """names of the kernels the last time_next_kernels arming timed, in launch order"""
    out = []
    buf = ctypes.create_string_buffer(128)
    for i in range(K.bagua_timed_kernels()):
        check(K.bagua_timed_kernel_name(i, buf, 128), "timed_kernel_name")
        out.append(buf.value.decode())
    return out
