"""salz_amd - MI355X-native SA-LZ codec (drop-in for akiutoslahti/salz's compression path).

Python mirror of the reference C API over libsalz.so (ctypes, plain pointers and sizes):

    encoded_len_max(n)            lib/salz.h:25-28
    encode_safe(src) -> bytes     salz_encode_safe, lib/salz.h:42-43 (raises SalzError on -1)
    decode_safe(src, n) -> bytes  salz_decode_safe, lib/salz.h:57-58

plus the GPU extensions of include/salz_gpu.h (contexts, device-resident encode, batched
multi-GPU container encode, stage dumps and statistics).

The product path is the HIP library only: importing this package fails loudly when
libsalz.so is missing, and encoding fails (SalzError) when no gfx950 device is usable.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# SALZ_LIB_PATH: load another build of the library (A/B timing in tools/ab.sh)
LIB_PATH = os.environ.get("SALZ_LIB_PATH") or os.path.join(_HERE, "libsalz.so")


class SalzError(RuntimeError):
    """A libsalz call returned -1 (same failure conditions as the reference)."""


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C salz_amd`")
    return ctypes.CDLL(LIB_PATH)


lib = _load()

_u8p = ctypes.c_void_p
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)

lib.salz_encode_safe.argtypes = [_u8p, _sz, _u8p, _szp]
lib.salz_encode_safe.restype = ctypes.c_int
lib.salz_decode_safe.argtypes = [_u8p, _sz, _u8p, _szp]
lib.salz_decode_safe.restype = ctypes.c_int
lib.salz_decode_frame.argtypes = [_u8p, _sz, _u8p, _szp]
lib.salz_decode_frame.restype = ctypes.c_int
lib.encode_vnibble_le.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64)]
lib.encode_vnibble_le.restype = _sz
lib.vnibble_size.argtypes = [ctypes.c_uint32]
lib.vnibble_size.restype = _sz
lib.salz_gpu_device_count.argtypes = []
lib.salz_gpu_device_count.restype = ctypes.c_int
lib.salz_gpu_parse_chunk_log.argtypes = [_sz]
lib.salz_gpu_parse_chunk_log.restype = ctypes.c_uint32
lib.salz_gpu_last_error.argtypes = []
lib.salz_gpu_last_error.restype = ctypes.c_char_p
lib.salz_gpu_malloc.argtypes = [ctypes.c_int, _sz]
lib.salz_gpu_malloc.restype = ctypes.c_void_p
lib.salz_gpu_free.argtypes = [ctypes.c_int, ctypes.c_void_p]
lib.salz_gpu_free.restype = None
lib.salz_gpu_memcpy_h2d.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, _sz]
lib.salz_gpu_memcpy_h2d.restype = ctypes.c_int
lib.salz_gpu_memcpy_d2h.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, _sz]
lib.salz_gpu_memcpy_d2h.restype = ctypes.c_int
lib.salz_gpu_synchronize.argtypes = [ctypes.c_int]
lib.salz_gpu_synchronize.restype = ctypes.c_int
lib.salz_gpu_ctx_create.argtypes = [ctypes.c_int, _sz]
lib.salz_gpu_ctx_create.restype = ctypes.c_void_p
lib.salz_gpu_ctx_destroy.argtypes = [ctypes.c_void_p]
lib.salz_gpu_ctx_destroy.restype = None
lib.salz_gpu_encode_device.argtypes = [ctypes.c_void_p, _u8p, _sz, _u8p, _sz, _szp, ctypes.c_void_p]
lib.salz_gpu_encode_device.restype = ctypes.c_int
lib.salz_gpu_encode_host.argtypes = [ctypes.c_void_p, _u8p, _sz, _u8p, _szp]
lib.salz_gpu_encode_host.restype = ctypes.c_int
lib.salz_gpu_pool_config.argtypes = [ctypes.c_int, _sz, ctypes.c_int]
lib.salz_gpu_pool_config.restype = None
lib.salz_gpu_pool_bytes.argtypes = [ctypes.c_int]
lib.salz_gpu_pool_bytes.restype = _sz
if hasattr(lib, "salz_gpu_workspace_allocs"):  # (absent from round-4 builds loaded for A/B timing)
    lib.salz_gpu_workspace_allocs.argtypes = []
    lib.salz_gpu_workspace_allocs.restype = _sz
lib.salz_gpu_set_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
lib.salz_gpu_set_timing.restype = None
lib.salz_gpu_encode_batch.argtypes = [ctypes.c_void_p, _u8p, _sz, _sz, _u8p, _szp]
lib.salz_gpu_encode_batch.restype = ctypes.c_int
lib.salz_gpu_encode_batch_device.argtypes = [ctypes.c_void_p, _u8p, _sz, _sz, _u8p, _sz, _szp, ctypes.c_void_p]
lib.salz_gpu_encode_batch_device.restype = ctypes.c_int
lib.salz_debug_init_order.argtypes = [_sz, _sz, ctypes.c_void_p]
lib.salz_debug_init_order.restype = ctypes.c_int
lib.salz_debug_radix_selftest.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                          ctypes.c_int]
lib.salz_debug_radix_selftest.restype = ctypes.c_long
if hasattr(lib, "salz_debug_xchg_offsets"):  # (absent from older builds loaded for A/B runs)
    lib.salz_debug_xchg_offsets.argtypes = [ctypes.c_int] + [ctypes.POINTER(ctypes.c_uint64)] * 4
    lib.salz_debug_xchg_offsets.restype = ctypes.c_int
lib.salz_encode_blocks.argtypes = [_u8p, _sz, _sz, _u8p, _szp, ctypes.c_int]
lib.salz_encode_blocks.restype = ctypes.c_int
lib.salz_blocks_len_max.argtypes = [_sz, _sz]
lib.salz_blocks_len_max.restype = _sz
lib.salz_decode_blocks.argtypes = [_u8p, _sz, _u8p, _szp, ctypes.c_int]
lib.salz_decode_blocks.restype = ctypes.c_int


# split suffix sort (include/salz_gpu.h salz_dist_ops): collectives supplied by the caller
DIST_ALLTOALL = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(ctypes.c_uint64))
DIST_ALLREDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64))


class DistOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("alltoall", DIST_ALLTOALL), ("allreduce_sum", DIST_ALLREDUCE)]


lib.salz_gpu_dist_suffix_array.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(DistOps), ctypes.c_void_p, ctypes.c_void_p, _sz,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                           ctypes.POINTER(ctypes.c_int)]
lib.salz_gpu_dist_suffix_array.restype = ctypes.c_int
lib.salz_gpu_dist_comm_id.argtypes = [ctypes.c_void_p]
lib.salz_gpu_dist_comm_id.restype = ctypes.c_int
lib.salz_gpu_dist_comm_create.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.salz_gpu_dist_comm_create.restype = ctypes.c_void_p
lib.salz_gpu_dist_comm_destroy.argtypes = [ctypes.c_void_p]
lib.salz_gpu_dist_comm_destroy.restype = None
lib.salz_gpu_dist_suffix_array_comm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p,
                                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64),
                                                ctypes.POINTER(ctypes.c_int)]
lib.salz_gpu_dist_suffix_array_comm.restype = ctypes.c_int
lib.salz_gpu_encode_from_sa.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _sz, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.POINTER(ctypes.c_uint64), _sz, ctypes.c_void_p, _sz, _szp]
lib.salz_gpu_encode_from_sa.restype = ctypes.c_int


class _Dump(ctypes.Structure):
    _fields_ = [(name, ctypes.c_void_p) for name in
                ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff", "cost")]


lib.salz_gpu_encode_dump.argtypes = [ctypes.c_void_p, _u8p, _sz, _u8p, _szp, ctypes.POINTER(_Dump)]
lib.salz_gpu_encode_dump.restype = ctypes.c_int
lib.salz_debug_encode_batch_dump.argtypes = [ctypes.c_void_p, _u8p, _sz, _sz, _u8p, _szp, ctypes.POINTER(_Dump)]
lib.salz_debug_encode_batch_dump.restype = ctypes.c_int


class Stats(ctypes.Structure):
    _fields_ = [("ms_upload", ctypes.c_double), ("ms_sa", ctypes.c_double),
                ("ms_lcp", ctypes.c_double), ("ms_ansv", ctypes.c_double),
                ("ms_parse", ctypes.c_double), ("ms_emit", ctypes.c_double),
                ("ms_total", ctypes.c_double), ("sa_rounds", ctypes.c_int32),
                ("parse_iters", ctypes.c_int32), ("sa_sorted_elems", ctypes.c_uint64),
                ("lcp_long_bytes", ctypes.c_uint64), ("emit_bits", ctypes.c_uint64),
                ("emit_bytes", ctypes.c_uint64), ("exit_nodes", ctypes.c_uint32),
                ("radix_scatter_launches", ctypes.c_uint32), ("ms_radix_scatter", ctypes.c_double),
                ("radix_scatter_elems", ctypes.c_uint64), ("sa_dc3_levels", ctypes.c_int32),
                ("radix_scatter_bytes", ctypes.c_uint64)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


lib.salz_gpu_get_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(Stats)]
lib.salz_gpu_get_stats.restype = ctypes.c_int


def _buf(data) -> np.ndarray:
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return np.ascontiguousarray(a.reshape(-1).view(np.uint8))


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def last_error() -> str:
    return lib.salz_gpu_last_error().decode(errors="replace")


def xchg_offsets(send_counts, recv_counts):
    """Test hook (host only): where each peer's run starts in the send and receive buffers of one
    exchange of the split suffix sort's in-library RCCL path (dsa.hip xchg_offsets)."""
    n = len(send_counts)
    U = ctypes.c_uint64 * n
    so, ro = U(), U()
    if lib.salz_debug_xchg_offsets(n, U(*send_counts), U(*recv_counts), so, ro) != 0:
        raise SalzError("xchg_offsets: invalid arguments")
    return list(so), list(ro)


def radix_selftest(m: int, bits: int, iters: int = 2, seed: int = 1, device: int = 0, nine: bool = False) -> int:
    """Test hook: the suffix sorter's LSD radix sort on m random (key, index) pairs of `bits` key
    bits, on the device, with 8-bit digits or (nine) 9-bit digits wherever they save a pass (the
    rank rounds' plan); returns the number of runs whose output was out of order, unstable or
    not a permutation of the input (-1: allocation failed)."""
    return lib.salz_debug_radix_selftest(device, m, bits, iters, seed, 1 if nine else 0)


def encoded_len_max(plain_len: int) -> int:
    """lib/salz.h:25-28: 4 + n + roundup(n, 64) / 8."""
    return 4 + plain_len + ((plain_len + 63) // 64 * 64) // 8


def device_count() -> int:
    return lib.salz_gpu_device_count()


def encode_safe(src, dst_capacity: Optional[int] = None) -> bytes:
    """salz_encode_safe: encode one block (> 8 bytes) on the GPU. Raises SalzError on -1."""
    s = _buf(src)
    cap = encoded_len_max(len(s)) if dst_capacity is None else dst_capacity
    out = np.empty(max(cap, 1), np.uint8)
    n = ctypes.c_size_t(cap)
    if lib.salz_encode_safe(_ptr(s) if len(s) else None, len(s), _ptr(out), ctypes.byref(n)) != 0:
        raise SalzError(f"salz_encode_safe failed: {last_error()}")
    return out[: n.value].tobytes()


def decode_safe(src, plain_capacity: int, frame: bool = False) -> bytes:
    """salz_decode_safe (or salz_decode_frame when frame=True). Raises SalzError on -1."""
    s = _buf(src)
    out = np.empty(max(plain_capacity, 1), np.uint8)
    n = ctypes.c_size_t(plain_capacity)
    fn = lib.salz_decode_frame if frame else lib.salz_decode_safe
    if fn(_ptr(s), len(s), _ptr(out), ctypes.byref(n)) != 0:
        raise SalzError("salz_decode_safe failed")
    return out[: n.value].tobytes()


def encode_blocks(src, block_size: int, n_devices: int = 0) -> bytes:
    """Reference CLI container of src in blocks of block_size, encoded across GPUs."""
    s = _buf(src)
    cap = lib.salz_blocks_len_max(len(s), block_size)
    out = np.empty(cap, np.uint8)
    n = ctypes.c_size_t(cap)
    if lib.salz_encode_blocks(_ptr(s), len(s), block_size, _ptr(out), ctypes.byref(n), n_devices) != 0:
        raise SalzError(f"salz_encode_blocks failed: {last_error()}")
    return out[: n.value].tobytes()


def decode_blocks(src, plain_capacity: int, threads: int = 0) -> bytes:
    s = _buf(src)
    out = np.empty(max(plain_capacity, 1), np.uint8)
    n = ctypes.c_size_t(plain_capacity)
    if lib.salz_decode_blocks(_ptr(s), len(s), _ptr(out), ctypes.byref(n), threads) != 0:
        raise SalzError("salz_decode_blocks failed")
    return out[: n.value].tobytes()


class DeviceBuffer:
    """HBM allocation made through libsalz's own HIP runtime."""

    def __init__(self, nbytes: int, device: int = 0):
        self.device, self.nbytes = device, nbytes
        self.ptr = lib.salz_gpu_malloc(device, nbytes)
        if not self.ptr:
            raise SalzError(f"device allocation failed: {last_error()}")

    def upload(self, data) -> "DeviceBuffer":
        a = _buf(data)
        assert len(a) <= self.nbytes
        if lib.salz_gpu_memcpy_h2d(self.device, self.ptr, _ptr(a), len(a)) != 0:
            raise SalzError(last_error())
        return self

    def download(self, nbytes: int) -> bytes:
        out = np.empty(max(nbytes, 1), np.uint8)
        if lib.salz_gpu_memcpy_d2h(self.device, _ptr(out), self.ptr, nbytes) != 0:
            raise SalzError(last_error())
        return out[:nbytes].tobytes()

    def free(self):
        if self.ptr:
            lib.salz_gpu_free(self.device, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def synchronize(device: int = 0) -> None:
    if lib.salz_gpu_synchronize(device) != 0:
        raise SalzError(last_error())


class Context:
    """A device context (salz_gpu_ctx) with workspace for blocks up to max_block bytes."""

    def __init__(self, device: int = 0, max_block: int = 1 << 20):
        self.handle = lib.salz_gpu_ctx_create(device, max_block)
        if not self.handle:
            raise SalzError(f"salz_gpu_ctx_create failed: {last_error()}")
        self.device = device
        self.max_block = max_block

    def close(self):
        if self.handle:
            lib.salz_gpu_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timing(self, on: bool = True):
        lib.salz_gpu_set_timing(self.handle, 1 if on else 0)

    def stats(self) -> dict:
        s = Stats()
        lib.salz_gpu_get_stats(self.handle, ctypes.byref(s))
        return s.as_dict()

    def encode(self, src, dst_capacity: Optional[int] = None) -> bytes:
        s = _buf(src)
        cap = encoded_len_max(len(s)) if dst_capacity is None else dst_capacity
        out = np.empty(max(cap, 1), np.uint8)
        n = ctypes.c_size_t(cap)
        if lib.salz_gpu_encode_host(self.handle, _ptr(s), len(s), _ptr(out), ctypes.byref(n)) != 0:
            raise SalzError(f"encode failed: {last_error()}")
        return out[: n.value].tobytes()

    def encode_into(self, src, out: np.ndarray) -> int:
        """salz_gpu_encode_host into a caller-owned buffer (reused across calls, as the reference
        CLI reuses its block buffers, programs/salzcli.c); returns the stream length."""
        s = _buf(src)
        n = ctypes.c_size_t(len(out))
        if lib.salz_gpu_encode_host(self.handle, _ptr(s), len(s), _ptr(out), ctypes.byref(n)) != 0:
            raise SalzError(f"encode failed: {last_error()}")
        return n.value

    def encode_batch(self, src, block_size: int) -> list[bytes]:
        """salz_gpu_encode_batch: every block of src in one pipeline pass; the streams."""
        s = _buf(src)
        nb = max(1, -(-len(s) // block_size))
        cap = nb * (encoded_len_max(min(block_size, len(s))) + 8)
        out = np.empty(max(cap, 1), np.uint8)
        n = ctypes.c_size_t(cap)
        if lib.salz_gpu_encode_batch(self.handle, _ptr(s), len(s), block_size, _ptr(out), ctypes.byref(n)) != 0:
            raise SalzError(f"encode_batch failed: {last_error()}")
        data, pos, streams = out[: n.value].tobytes(), 0, []
        while pos < len(data):
            L = int.from_bytes(data[pos:pos + 4], "little")
            streams.append(data[pos + 4:pos + 4 + L])
            pos += 4 + L
        return streams

    def encode_batch_device(self, d_src: int, src_len: int, block_size: int, d_dst: int, dst_cap: int,
                            stream: Optional[int] = None) -> int:
        """salz_gpu_encode_batch_device: packed frames of every block into HBM; their bytes."""
        n = ctypes.c_size_t(0)
        rc = lib.salz_gpu_encode_batch_device(self.handle, d_src, src_len, block_size, d_dst, dst_cap,
                                              ctypes.byref(n), stream)
        if rc != 0:
            raise SalzError(f"encode_batch_device failed: {last_error()}")
        return n.value

    def encode_batch_dump(self, src, block_size: int) -> tuple[list[bytes], dict]:
        """encode_batch plus the batch's stage arrays (test hook): sa holds global text
        positions; psv/nsv/lp/ln/dlen/doff/cost are indexed by global position."""
        s = _buf(src)
        npos = len(s) - 8
        arrs = {k: np.zeros(npos + (1 if k == "cost" else 0), np.int32)
                for k in ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff", "cost")}
        d = _Dump(**{k: v.ctypes.data for k, v in arrs.items()})
        nb = max(1, -(-len(s) // block_size))
        cap = nb * (encoded_len_max(min(block_size, len(s))) + 8)
        out = np.empty(max(cap, 1), np.uint8)
        n = ctypes.c_size_t(cap)
        if lib.salz_debug_encode_batch_dump(self.handle, _ptr(s), len(s), block_size, _ptr(out),
                                            ctypes.byref(n), ctypes.byref(d)) != 0:
            raise SalzError(f"encode_batch_dump failed: {last_error()}")
        data, pos, streams = out[: n.value].tobytes(), 0, []
        while pos < len(data):
            L = int.from_bytes(data[pos:pos + 4], "little")
            streams.append(data[pos + 4:pos + 4 + L])
            pos += 4 + L
        return streams, arrs

    def encode_device(self, d_src: int, src_len: int, d_dst: int, dst_cap: int,
                      stream: Optional[int] = None) -> int:
        """Encode a block resident in HBM (raw device pointers); returns the stream length."""
        n = ctypes.c_size_t(0)
        rc = lib.salz_gpu_encode_device(self.handle, d_src, src_len, d_dst, dst_cap,
                                        ctypes.byref(n), stream)
        if rc != 0:
            raise SalzError(f"encode_device failed: {last_error()}")
        return n.value

    def encode_dump(self, src) -> tuple[bytes, dict]:
        """Encode and return the intermediate arrays (sa, psv, nsv, lp, ln, dlen, doff, cost)."""
        s = _buf(src)
        n = len(s) - 8
        arrs = {k: np.zeros(n + (1 if k == "cost" else 0), np.int32)
                for k in ("sa", "psv", "nsv", "lp", "ln", "dlen", "doff", "cost")}
        d = _Dump(**{k: v.ctypes.data for k, v in arrs.items()})
        cap = encoded_len_max(len(s))
        out = np.empty(cap, np.uint8)
        m = ctypes.c_size_t(cap)
        if lib.salz_gpu_encode_dump(self.handle, _ptr(s), len(s), _ptr(out), ctypes.byref(m),
                                    ctypes.byref(d)) != 0:
            raise SalzError(f"encode_dump failed: {last_error()}")
        return out[: m.value].tobytes(), arrs
