"""Host-side mirror of ``bmqp::Crc32c`` (reference:
/root/reference/src/groups/bmq/bmqp/bmqp_crc32c.h:225-257) plus the batched
MI355X entry point.

    Crc32c.calculate(data, crc=Crc32c.k_NULL_CRC32C)      -> int   (CPU, like the reference)
    Crc32c.calculate_blob(blob, crc=...)                    -> int   (CPU, bmqp_crc32c.cpp:47-67)
    Crc32c.calculate_batch(arena, offsets, lengths, seeds)  -> out   (GPU only)

``calculate_batch`` accepts torch tensors resident on an MI355X (no copies;
enqueued on torch's current stream) or host buffers (numpy / bytes), which the
library stages through HBM.  It never computes on the CPU: without a usable
GPU it raises ``BmqCrcError`` (BMQCRC_ENODEV).
"""
import ctypes

import numpy as np

from . import _native
from ._native import BmqCrcError  # noqa: F401  (re-export)


class Blob:
    """Minimal stand-in for ``bdlbb::Blob``: an ordered list of data buffers.

    Mirrors the members bmqp::Crc32c uses: ``num_data_buffers()``,
    ``buffer(i)``, ``last_data_buffer_length()``.
    """

    def __init__(self, buffers=()):
        self._buffers = [bytes(b) for b in buffers]
        self._last_len = len(self._buffers[-1]) if self._buffers else 0

    def append_data_buffer(self, buf):
        self._buffers.append(bytes(buf))
        self._last_len = len(self._buffers[-1])

    def set_last_data_buffer_length(self, n):
        self._last_len = n

    def num_data_buffers(self):
        return len(self._buffers)

    def buffer(self, i):
        return self._buffers[i]

    def last_data_buffer_length(self):
        return self._last_len


def _as_bytes_ptr(data):
    if data is None:
        return None, 0, None
    if isinstance(data, (bytes, bytearray, memoryview)):
        buf = (ctypes.c_char * len(data)).from_buffer_copy(bytes(data))
        return ctypes.cast(buf, ctypes.c_void_p), len(data), buf
    arr = np.ascontiguousarray(data).view(np.uint8).reshape(-1)
    return ctypes.c_void_p(arr.ctypes.data), arr.size, arr


class Crc32c:
    """``bmqp::Crc32c`` (bmqp_crc32c.h:225-257)."""

    k_NULL_CRC32C = 0

    @staticmethod
    def calculate(data, crc=0, length=None):
        """CRC32-C of ``data`` (bytes-like / numpy), continuing from ``crc``.

        ``data=None`` requires ``length`` 0 (bmqp_crc32c.h:242-243).
        """
        ptr, n, keep = _as_bytes_ptr(data)
        if length is not None:
            if length > n:
                raise ValueError("length exceeds buffer")
            n = length
        if ptr is None and n:
            raise ValueError("null data with non-zero length")
        r = _native.lib.bmqcrc_crc32c(ptr, n, crc & 0xFFFFFFFF)
        del keep
        return r

    @staticmethod
    def calculate_blob(blob, crc=0):
        """CRC32-C over the data buffers of ``blob`` (bmqp_crc32c.cpp:47-67)."""
        nb = blob.num_data_buffers()
        if nb == 0:
            return crc & 0xFFFFFFFF
        keeps, ptrs, lens = [], (ctypes.c_void_p * nb)(), (ctypes.c_uint32 * nb)()
        for i in range(nb):
            b = blob.buffer(i)
            n = len(b) if i < nb - 1 else blob.last_data_buffer_length()
            p, _, k = _as_bytes_ptr(b)
            keeps.append(k)
            ptrs[i] = p
            lens[i] = n
        return _native.lib.bmqcrc_crc32c_blob(ptrs, lens, nb, crc & 0xFFFFFFFF)

    @staticmethod
    def combine(crc_a, crc_b, len_b):
        return _native.lib.bmqcrc_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)

    @staticmethod
    def verify_batch(arena, offsets, lengths, expected, bad_cap=1 << 20, seg_bytes=0,
                     devices=None):
        """Batched recovery check (bmqcrc_crc32c_verify): (n_bad, bad indices)."""
        return verify_batch(arena, offsets, lengths, expected, bad_cap, seg_bytes,
                            devices=devices)

    @staticmethod
    def calculate_blobs(blobs, seeds=None, seg_bytes=0, gather=True):
        """Batched Blob overload (bmqcrc_crc32c_gather / bmqcrc_crc32c_blobs) on the GPU."""
        return calculate_blobs(blobs, seeds, seg_bytes, gather=gather)

    @staticmethod
    def calculate_batch(arena, offsets, lengths, seeds=None, out=None, *, seg_bytes=0,
                        device=None, stream=None, sync=True, time_kernel=False,
                        whole_messages=False, devices=None, plan=False, max_len=0, min_len=0):
        """Batched CRC32-C of messages ``arena[offsets[i] : offsets[i]+lengths[i]]``.

        torch CUDA tensors: ``arena`` uint8, ``offsets`` int64, ``lengths`` /
        ``seeds`` / ``out`` int32 (read as u32) on one device; the call is
        enqueued on ``stream`` (default: torch's current stream) and
        ``out`` (int32 tensor) is returned.  Host arrays: numpy in, numpy
        ``uint32`` out.  ``whole_messages`` (BMQCRC_F_WHOLE_MESSAGES): one
        lane per message, no planner launches -- for batches of small messages.
        ``devices`` (host arrays only): split the batch over several GPUs.
        ``plan`` (BMQCRC_F_PLAN, device tensors): run the planner for this
        batch instead of predicting its shape from the previous batch.
        ``max_len`` (bmqcrc_opts.max_len, device tensors): the caller's bound
        on every length; when it fits one segment the batch is one launch
        whatever the previous batch was (a longer message stays exact);
        with ``min_len`` too, a range whose lengths all have the same u
        segments (u dividing 64) gets the uniform single launch.
        """
        try:
            import torch
        except ImportError:  # pragma: no cover
            torch = None
        if torch is not None and isinstance(arena, torch.Tensor) and arena.is_cuda:
            return _batch_torch(torch, arena, offsets, lengths, seeds, out, seg_bytes, stream,
                                sync, time_kernel, whole_messages, plan, max_len, min_len)
        return _batch_host(arena, offsets, lengths, seeds, out, seg_bytes, device,
                           whole_messages, devices)


def _batch_torch(torch, arena, offsets, lengths, seeds, out, seg_bytes, stream, sync,
                 time_kernel=False, whole_messages=False, plan=False, max_len=0, min_len=0):
    dev = arena.device
    n = offsets.numel()
    for name, t, dt in (("offsets", offsets, torch.int64), ("lengths", lengths, torch.int32)):
        if not (isinstance(t, torch.Tensor) and t.device == dev and t.dtype == dt
                and t.is_contiguous()):
            raise TypeError("%s must be a contiguous %s tensor on %s" % (name, dt, dev))
    if lengths.numel() != n:
        raise ValueError("offsets/lengths size mismatch")
    if seeds is not None and not _is_vec(torch, seeds, dev, torch.int32, n):
        raise TypeError("seeds must be a contiguous int32 tensor of %d elements on %s" % (n, dev))
    if arena.dtype != torch.uint8 or not arena.is_contiguous():
        raise TypeError("arena must be a contiguous uint8 tensor")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=dev)
    elif not _is_vec(torch, out, dev, torch.int32, n):
        raise TypeError("out must be a contiguous int32 tensor of %d elements on %s" % (n, dev))
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    flags = _native.BMQCRC_F_DEVICE_PTRS | (0 if sync else _native.BMQCRC_F_ASYNC)
    if time_kernel:
        flags |= _native.BMQCRC_F_TIME_KERNEL
    if whole_messages:
        flags |= _native.BMQCRC_F_WHOLE_MESSAGES
    if plan:
        flags |= _native.BMQCRC_F_PLAN
    o = _native.make_opts(device=dev.index if dev.index is not None else -1,
                          stream=stream.cuda_stream, flags=flags, seg_bytes=seg_bytes,
                          max_len=max_len, min_len=min_len)
    _native.check(_native.lib.bmqcrc_crc32c_batch(
        arena.data_ptr(), arena.numel(), offsets.data_ptr(), lengths.data_ptr(),
        seeds.data_ptr() if seeds is not None else None, out.data_ptr(), n, ctypes.byref(o)))
    return out


def _is_vec(torch, t, dev, dtype, n):
    """A contiguous 1-D-sized tensor of n elements of dtype on dev."""
    return (isinstance(t, torch.Tensor) and t.device == dev and t.dtype == dtype
            and t.is_contiguous() and t.numel() == n)


def _check_host_out(out, n):
    if not (isinstance(out, np.ndarray) and out.dtype == np.uint32 and out.size == n
            and out.flags.c_contiguous and out.flags.writeable):
        raise TypeError("out must be a writeable C-contiguous uint32 ndarray of %d elements" % n)
    return out


def _batch_host(arena, offsets, lengths, seeds, out, seg_bytes, device, whole_messages=False,
                devices=None):
    a = np.frombuffer(bytes(arena), dtype=np.uint8) if isinstance(
        arena, (bytes, bytearray, memoryview)) else np.ascontiguousarray(arena).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    if off.shape != ln.shape:
        raise ValueError("offsets/lengths size mismatch")
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    if sd is not None and sd.shape != off.shape:
        raise ValueError("seeds must have one entry per message")
    res = np.empty(off.size, dtype=np.uint32) if out is None else _check_host_out(out, off.size)
    o = _native.make_opts(device=-1 if device is None else device, seg_bytes=seg_bytes,
                          flags=_native.BMQCRC_F_WHOLE_MESSAGES if whole_messages else 0,
                          devices=devices)
    _native.check(_native.lib.bmqcrc_crc32c_batch(
        a.ctypes.data if a.size else None, a.size, off.ctypes.data, ln.ctypes.data,
        sd.ctypes.data if sd is not None else None, res.ctypes.data, off.size, ctypes.byref(o)))
    return res


def _u8_host(arena):
    if isinstance(arena, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(arena), dtype=np.uint8)
    return np.ascontiguousarray(arena).view(np.uint8).reshape(-1)


def verify_batch(arena, offsets, lengths, expected, bad_cap=1 << 20, seg_bytes=0, device=None,
                 devices=None):
    """GPU batch CRC of every message compared on the device with `expected`.

    Returns (n_bad, bad_index ndarray[uint64], ascending, at most bad_cap)."""
    a = _u8_host(arena)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    ex = np.ascontiguousarray(expected, dtype=np.uint32)
    if not (off.shape == ln.shape == ex.shape):
        raise ValueError("offsets/lengths/expected size mismatch")
    nbad = ctypes.c_uint64()
    idx = np.zeros(max(int(bad_cap), 1), dtype=np.uint64)
    o = _native.make_opts(device=-1 if device is None else device, seg_bytes=seg_bytes,
                          devices=devices)
    _native.check(_native.lib.bmqcrc_crc32c_verify(
        a.ctypes.data if a.size else None, a.size, off.ctypes.data, ln.ctypes.data,
        ex.ctypes.data, off.size, ctypes.byref(nbad), idx.ctypes.data, int(bad_cap),
        ctypes.byref(o)))
    return int(nbad.value), idx[:min(int(nbad.value), int(bad_cap))].copy()


def calculate_blobs(blobs, seeds=None, seg_bytes=0, device=None, gather=True):
    """``bmqp::Crc32c::calculate(blob, seed)`` for a list of Blob on the GPU
    (``Crc32c::calculateBatch(const Blob*)``).  Returns ndarray[uint32].

    gather=True (the C++ overload's path, bmqcrc_crc32c_gather): the blobs'
    buffers stay where they are and the library copies them once, through a
    pinned staging ring, into HBM.  gather=False: the buffers are first laid
    out in one host arena and bmqcrc_crc32c_blobs CRCs each buffer and chains
    them on the device."""
    bufs, lens, first = [], [], [0]
    for b in blobs:
        nb = b.num_data_buffers()
        for i in range(nb):
            data = b.buffer(i)
            n = len(data) if i < nb - 1 else b.last_data_buffer_length()
            bufs.append(data)
            lens.append(n)
        first.append(len(lens))
    ln = np.asarray(lens, dtype=np.uint32)
    fb = np.asarray(first, dtype=np.uint64)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    if sd is not None and sd.size != len(blobs):
        raise ValueError("seeds must have one entry per blob")
    out = np.empty(len(blobs), dtype=np.uint32)
    o = _native.make_opts(device=-1 if device is None else device, seg_bytes=seg_bytes)
    if gather:
        keep = [_as_bytes_ptr(bytes(d) if isinstance(d, (bytes, bytearray, memoryview)) else d)
                for d in bufs]
        ptrs = (ctypes.c_void_p * max(len(keep), 1))(*[k[0] for k in keep])
        for k, n in zip(keep, lens):
            if n > k[1]:
                raise ValueError("buffer shorter than its data length")
        _native.check(_native.lib.bmqcrc_crc32c_gather(
            ptrs, ln.ctypes.data if ln.size else None, ln.size, fb.ctypes.data,
            sd.ctypes.data if sd is not None else None, out.ctypes.data, len(blobs),
            ctypes.byref(o)))
        del keep
        return out
    arena = np.frombuffer(b"".join(bytes(d[:n]) for d, n in zip(bufs, lens)) + b"\0",
                          dtype=np.uint8)
    offs = np.zeros(len(lens), dtype=np.uint64)
    if len(lens) > 1:
        offs[1:] = np.cumsum(np.asarray(lens[:-1], dtype=np.uint64))
    _native.check(_native.lib.bmqcrc_crc32c_blobs(
        arena.ctypes.data, arena.size, offs.ctypes.data if ln.size else None,
        ln.ctypes.data if ln.size else None, ln.size, fb.ctypes.data,
        sd.ctypes.data if sd is not None else None, out.ctypes.data, len(blobs),
        ctypes.byref(o)))
    return out


def calculate_batch_multi(arena, offsets, lengths, seeds=None, devices=None, seg_bytes=0):
    """Host-buffer batch sharded byte-balanced over several GPUs of this process."""
    a = np.ascontiguousarray(arena).view(np.uint8)
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    ln = np.ascontiguousarray(lengths, dtype=np.uint32)
    sd = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
    res = np.empty(off.size, dtype=np.uint32)
    if devices is None:
        devices = list(range(device_count()))
    dv = (ctypes.c_int * len(devices))(*devices)
    _native.check(_native.lib.bmqcrc_crc32c_batch_multi(
        a.ctypes.data, a.size, off.ctypes.data, ln.ctypes.data,
        sd.ctypes.data if sd is not None else None, res.ctypes.data, off.size, dv, len(devices),
        seg_bytes))
    return res


def fill_synthetic(tensor, seed, stream=None, begin=0):
    """Fill a CUDA uint8 tensor with bytes [begin, begin+numel) of synthetic stream ``seed``."""
    import torch
    if stream is None:
        stream = torch.cuda.current_stream(tensor.device)
    o = _native.make_opts(device=tensor.device.index, stream=stream.cuda_stream,
                          flags=_native.BMQCRC_F_ASYNC)
    _native.check(_native.lib.bmqcrc_fill_synthetic(tensor.data_ptr(), tensor.numel(), seed,
                                                    begin, ctypes.byref(o)))
    return tensor


def kernel_timing(device, stream):
    """(total_ms, count) of fold kernels timed with time_kernel=True since the last query."""
    tot, cnt = ctypes.c_double(), ctypes.c_uint32()
    _native.check(_native.lib.bmqcrc_kernel_timing(device, stream.cuda_stream, ctypes.byref(tot),
                                                  ctypes.byref(cnt)))
    return tot.value, cnt.value


def last_launch(device, stream):
    """Launch plan of the previous batch on (device, stream)
    (bmqcrc_last_launch, bmqcrc_last_plan): dict(kernels, spec, seg_bytes,
    map) -- kernels launched
    (1 = the fold alone), segments per message a single launch assumed (0 =
    planned), segment size, whether the planner built the size-class map."""
    k, u, sb = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
    _native.check(_native.lib.bmqcrc_last_launch(device, stream.cuda_stream, ctypes.byref(k),
                                                ctypes.byref(u), ctypes.byref(sb)))
    m = ctypes.c_uint32()
    _native.check(_native.lib.bmqcrc_last_plan(device, stream.cuda_stream, ctypes.byref(m)))
    return {"kernels": k.value, "spec": u.value, "seg_bytes": sb.value, "map": m.value}


def forget_shape(device, stream):
    """Drop the batch-shape prediction of (device, stream)
    (bmqcrc_forget_shape): the next batch there is planned."""
    _native.check(_native.lib.bmqcrc_forget_shape(device, stream.cuda_stream))


def plan_wait(device, stream, wait_us=100):
    """Longest wait (microseconds) of the single-pass planner's blocks for
    each other on (device, stream) before a ragged batch's size-class map is
    given up (bmqcrc_plan_wait, default 100; results stay exact, the fold then
    searches the per-message segment offsets instead of the size-class map).
    Returns how many planned batches there gave up their map so far."""
    n = ctypes.c_uint64()
    _native.check(_native.lib.bmqcrc_plan_wait(device, stream.cuda_stream, int(wait_us),
                                              ctypes.byref(n)))
    return n.value


def reserve(device, stream, n_msgs, arena_bytes, seg_bytes=0):
    """Pre-size the workspace of (device, stream) for batches of up to n_msgs
    messages over arena_bytes (bmqcrc_reserve): afterwards a device-pointer
    batch of that size allocates nothing, so it can be captured in a graph."""
    _native.check(_native.lib.bmqcrc_reserve(device, stream.cuda_stream, n_msgs, arena_bytes,
                                             seg_bytes))


class HostRegistration:
    """Zero-copy view of a host array for the GPU (bmqcrc_host_register):
    ``dev_ptr`` is the device-side address of ``array``'s first byte.  The
    array must stay alive (and unmoved) until ``close()``."""

    def __init__(self, array, device=-1):
        self.array = np.ascontiguousarray(array).view(np.uint8).reshape(-1)
        self.nbytes = self.array.size
        p = ctypes.c_void_p()
        _native.check(_native.lib.bmqcrc_host_register(self.array.ctypes.data, self.nbytes,
                                                       device, ctypes.byref(p)))
        self.dev_ptr = p.value
        self._open = True

    def close(self):
        if self._open:
            self._open = False
            _native.check(_native.lib.bmqcrc_host_unregister(self.array.ctypes.data))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def calculate_batch_ptr(arena_ptr, arena_bytes, offsets, lengths, seeds=None, out=None, *,
                        seg_bytes=0, stream=None, sync=True):
    """Batch over a device-visible arena given by address (a device allocation
    or a ``HostRegistration.dev_ptr``); offsets/lengths/seeds/out as in
    ``Crc32c.calculate_batch``'s torch form."""
    import torch
    dev = offsets.device
    n = offsets.numel()
    if not _is_vec(torch, offsets, dev, torch.int64, n) or \
            not _is_vec(torch, lengths, dev, torch.int32, n):
        raise TypeError("offsets/lengths must be contiguous int64/int32 tensors of n elements")
    if seeds is not None and not _is_vec(torch, seeds, dev, torch.int32, n):
        raise TypeError("seeds must be a contiguous int32 tensor of %d elements on %s" % (n, dev))
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=dev)
    elif not _is_vec(torch, out, dev, torch.int32, n):
        raise TypeError("out must be a contiguous int32 tensor of %d elements on %s" % (n, dev))
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    flags = _native.BMQCRC_F_DEVICE_PTRS | (0 if sync else _native.BMQCRC_F_ASYNC)
    o = _native.make_opts(device=dev.index if dev.index is not None else -1,
                          stream=stream.cuda_stream, flags=flags, seg_bytes=seg_bytes)
    _native.check(_native.lib.bmqcrc_crc32c_batch(
        arena_ptr, arena_bytes, offsets.data_ptr(), lengths.data_ptr(),
        seeds.data_ptr() if seeds is not None else None, out.data_ptr(), n, ctypes.byref(o)))
    return out


def device_count():
    return _native.lib.bmqcrc_device_count()
