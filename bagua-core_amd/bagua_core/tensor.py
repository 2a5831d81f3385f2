"""BaguaTensorPy — the tensor surface of bagua-core's Python module.

Mirrors `BaguaTensorPy` (bagua-core-py/src/lib.rs:196-299): construction from
a torch tensor and a name, `compress(method, n_chunks, target_chunk)`,
`decompress_from(method, n_chunks, compressed)`, `to_numpy_f32/u8`, and the
accessors.  Every codec call goes through the C ABI into the gfx950 kernels
(libbagua_core.so -> libbagua_kernels.so); nothing is computed in Python.

Extensions over the reference: torch.bfloat16 tensors (the reference rejects
them, lib.rs:211-221) and the "OneBitSignScale" method.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as N

_DTYPES = {
    torch.float32: (N.DTYPE_F32, "F32"),
    torch.float16: (N.DTYPE_F16, "F16"),
    torch.bfloat16: (N.DTYPE_BF16, "BF16"),
    torch.uint8: (N.DTYPE_U8, "U8"),
    torch.int64: (N.DTYPE_I64, "I64"),
}
_DTYPE_NAMES = {code: name for code, name in _DTYPES.values()}
_DTYPE_NAMES[N.DTYPE_U64] = "U64"

METHODS = {"MinMaxUInt8": N.COMPRESSION_MINMAX_UINT8, "OneBitSignScale": N.COMPRESSION_ONEBIT}


def compression_code(method: str) -> int:
    try:
        return METHODS[method]
    except KeyError:
        # datatypes/mod.rs:837-839 `unimplemented!()` for any other method
        raise NotImplementedError(f"unsupported compression method {method!r}") from None


def current_stream_ptr(device_id: int) -> int:
    return int(torch.cuda.current_stream(device_id).cuda_stream)


class BaguaTensorPy:
    """A named device tensor: either a view of a torch tensor or a pool buffer."""

    def __init__(self, torch_tensor: torch.Tensor, name: str):
        spec = _DTYPES.get(torch_tensor.dtype)
        if spec is None:
            raise RuntimeError(f"unsupported tensor dtype {torch_tensor.dtype}")
        if torch_tensor.device.type != "cuda":
            # datatypes/mod.rs:629-633
            raise RuntimeError("currently only cuda tensors are supported in Bagua")
        if not torch_tensor.is_contiguous():
            raise RuntimeError("BaguaTensorPy requires a contiguous tensor")
        self._torch = torch_tensor
        self._name = name
        self._name_b = name.encode()
        self._pool_ptr = 0
        self._raw = None
        self._streams: set[int] = set()
        # cached descriptor of the torch-backed tensor (the device is fixed; pointer,
        # size and dtype are re-read from the torch tensor on every use: a `.data` swap)
        self._desc = N.bagua_tensor_t()
        self._desc.dtype = spec[0]
        self._desc.device_id = torch_tensor.device.index if torch_tensor.device.index is not None \
            else torch.cuda.current_device()
        # the storage the scheduler's last mark saw and its device (_mark_device)
        self._mark_ptr, self._mark_dev = -1, self._desc.device_id

    # ---- construction from a pool buffer (compress output) ------------------
    @classmethod
    def _from_raw(cls, raw: N.bagua_tensor_t, name: str, owned: bool) -> "BaguaTensorPy":
        obj = cls.__new__(cls)
        obj._torch = None
        obj._name = name
        obj._name_b = name.encode()
        obj._raw = raw
        obj._pool_ptr = raw.ptr if owned else 0
        obj._streams = set()
        return obj

    def _used_on(self, stream: int) -> None:
        """Record a stream that queued work reading or writing this buffer."""
        if self._pool_ptr:
            self._streams.add(int(stream))

    def __del__(self):
        ptr = getattr(self, "_pool_ptr", 0)
        if ptr:
            # stream-ordered release: the block is reused only after the work
            # already queued on every stream that touched it has completed
            streams = sorted(getattr(self, "_streams", ()))
            arr = (ctypes.c_uint64 * max(1, len(streams)))(*streams)
            N.C.bagua_pool_free_after(ptr, arr, len(streams))
            self._pool_ptr = 0

    def raw(self) -> N.bagua_tensor_t:
        """A fresh descriptor of the tensor's current storage."""
        if self._torch is None:
            return self._raw
        t = self._torch
        n = t.numel()
        dev = t.device.index if t.device.type == "cuda" else -1
        return N.bagua_tensor_t(t.data_ptr(), n, n, _DTYPES[t.dtype][0],
                                self._desc.device_id if dev is None else dev)

    def _current(self) -> N.bagua_tensor_t:
        """The cached descriptor refreshed in place from the torch tensor: the
        scheduler's per-mark path allocates no ctypes object (the reference reads
        data_ptr / numel at run time, datatypes/mod.rs:775-791)."""
        if self._torch is None:
            return self._raw
        t = self._torch
        d = self._desc
        ptr = t.data_ptr()
        if ptr != d.ptr:
            # new storage (a .data / set_ swap): re-read what may have changed with it --
            # the bucket's native check (dtype and device may not change,
            # datatypes/mod.rs:1079-1118) must see the device the storage is on now
            dv = t.device
            d.device_id = -1 if dv.type != "cuda" else (dv.index if dv.index is not None else d.device_id)
            d.ptr = ptr
        spec = _DTYPES.get(t.dtype)
        d.dtype = spec[0] if spec else -1
        n = t.numel()
        d.num_elem = n
        d.num_elem_allocated = n
        return d

    def _mark_device(self, ptr: int) -> int:
        """The device of the torch tensor's storage, re-read when a mark sees new storage
        (`ptr`, a .data / set_ swap) and cached for the next marks."""
        dv = self._torch.device
        self._mark_dev = -1 if dv.type != "cuda" else (dv.index if dv.index is not None else self._desc.device_id)
        self._mark_ptr = ptr
        return self._mark_dev

    # ---- accessors (lib.rs:280-298) -----------------------------------------
    def name(self) -> str:
        return self._name

    def data_ptr(self) -> int:
        return int(self.raw().ptr)

    def device_id(self) -> int:
        return int(self.raw().device_id)

    def num_elements(self) -> int:
        return int(self.raw().num_elem)

    def num_elements_allocated(self) -> int:
        return int(self.raw().num_elem_allocated)

    def dtype(self) -> str:
        return _DTYPE_NAMES[self.raw().dtype]

    def torch_tensor(self) -> torch.Tensor | None:
        return self._torch

    # ---- codec (lib.rs:235-239, 275-278; datatypes/mod.rs:815-889) -----------
    def compress(self, method: str, n_chunks: int, target_chunk: int) -> "BaguaTensorPy":
        code = compression_code(method)
        src = self.raw()
        if n_chunks <= 0 or src.num_elem_allocated % n_chunks != 0:
            raise RuntimeError("compression tensor size % n_chunks must be 0")
        out = N.bagua_tensor_t()
        rc = N.C.bagua_tensor_compress(ctypes.byref(src), code, n_chunks, current_stream_ptr(src.device_id),
                                       target_chunk, ctypes.byref(out))
        N.check(rc, f"compress({method}, n_chunks={n_chunks}, target_chunk={target_chunk})")
        res = BaguaTensorPy._from_raw(out, "compressed_tensor", owned=True)
        res._used_on(current_stream_ptr(src.device_id))
        return res

    def decompress_from(self, method: str, n_chunks: int, compressed_buffer: "BaguaTensorPy") -> None:
        code = compression_code(method)
        dst = self.raw()
        if n_chunks <= 0 or dst.num_elem_allocated % n_chunks != 0:
            raise RuntimeError("compression tensor size % n_chunks must be 0")
        comp = compressed_buffer.raw()
        stream = current_stream_ptr(dst.device_id)
        rc = N.C.bagua_tensor_decompress_from(ctypes.byref(dst), code, n_chunks, ctypes.byref(comp), stream)
        N.check(rc, f"decompress_from({method}, n_chunks={n_chunks})")
        compressed_buffer._used_on(stream)

    # helpers of RawBaguaTensor used by the comm ops (datatypes/mod.rs:203-522)
    def reduce_mean_inplace(self, n_chunks: int, target_chunk: int) -> None:
        r = self.raw()
        N.check(N.C.bagua_tensor_reduce_inplace(ctypes.byref(r), n_chunks, target_chunk, 1,
                                                current_stream_ptr(r.device_id)), "reduce_mean_inplace")

    def reduce_sum_inplace(self, n_chunks: int, target_chunk: int) -> None:
        r = self.raw()
        N.check(N.C.bagua_tensor_reduce_inplace(ctypes.byref(r), n_chunks, target_chunk, 0,
                                                current_stream_ptr(r.device_id)), "reduce_sum_inplace")

    def add_inplace(self, other: "BaguaTensorPy") -> None:
        r, o = self.raw(), other.raw()
        N.check(N.C.bagua_tensor_add_inplace(ctypes.byref(r), ctypes.byref(o), current_stream_ptr(r.device_id)),
                "add_inplace")

    def addmul_inplace(self, other: "BaguaTensorPy", factor: float) -> None:
        r, o = self.raw(), other.raw()
        N.check(N.C.bagua_tensor_addmul_inplace(ctypes.byref(r), ctypes.byref(o), factor,
                                                current_stream_ptr(r.device_id)), "addmul_inplace")

    # ---- read-back (lib.rs:241-273, cuda_utils.rs:1-6) -------------------------
    def _to_numpy(self, np_dtype, expect: int) -> np.ndarray:
        r = self.raw()
        if r.dtype != expect:
            raise AssertionError(f"expected dtype {_DTYPE_NAMES[expect]}, tensor is {_DTYPE_NAMES[r.dtype]}")
        torch.cuda.current_stream(r.device_id).synchronize()
        out = np.empty(int(r.num_elem), dtype=np_dtype)
        rc = N.C.bagua_memcpy_device_to_host_sync(out.ctypes.data, r.ptr, out.nbytes)
        N.check(rc, "device-to-host copy")
        return out

    def to_numpy_f32(self) -> np.ndarray:
        return self._to_numpy(np.float32, N.DTYPE_F32)

    def to_numpy_u8(self) -> np.ndarray:
        return self._to_numpy(np.uint8, N.DTYPE_U8)

    def __repr__(self) -> str:
        r = self.raw()
        return (f"BaguaTensorPy(name={self._name!r}, dtype={_DTYPE_NAMES[r.dtype]}, num_elements={r.num_elem}, "
                f"device_id={r.device_id})")
