"""ctypes binding to the in-tree C-ABI library ``lib/libbmqcrc.so``.

There is no pure-Python or CPU substitute for the batch path: if the library
is missing this module raises at import, and the batch entry point returns
BMQCRC_ENODEV (raised as ``BmqCrcError``) when no MI355X is usable.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libbmqcrc.so")

BMQCRC_OK = 0
BMQCRC_EIO = -5
BMQCRC_ENOMEM = -12
BMQCRC_ENODEV = -19
BMQCRC_EINVAL = -22
BMQCRC_F_DEVICE_PTRS = 0x1
BMQCRC_F_ASYNC = 0x2
BMQCRC_F_TIME_KERNEL = 0x4
BMQCRC_F_WHOLE_MESSAGES = 0x8
BMQCRC_F_PLAN = 0x10


class BmqCrcError(RuntimeError):
    def __init__(self, rc, msg):
        super().__init__("bmqcrc error %d: %s" % (rc, msg))
        self.rc = rc


class Opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("device", ctypes.c_int32),
                ("stream", ctypes.c_void_p), ("flags", ctypes.c_uint32),
                ("seg_bytes", ctypes.c_uint32), ("ndevices", ctypes.c_uint32),
                ("devices", ctypes.c_void_p), ("max_len", ctypes.c_uint32),
                ("min_len", ctypes.c_uint32)]


# One HIP runtime per process: when PyTorch-ROCm is present it ships its own
# libamdhip64.so (soname libamdhip64.so.7).  Loading torch first lets this
# library's DT_NEEDED libamdhip64.so.7 bind to that same runtime instead of
# pulling a second copy from /opt/rocm (two runtimes cannot share a device).
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is optional for the C ABI itself
    torch = None

if not os.path.exists(LIB_PATH):
    raise ImportError("libbmqcrc.so not built (%s); run `python -c \"import __graft_entry__ as g; "
                      "g.build()\"` first" % LIB_PATH)

lib = ctypes.CDLL(LIB_PATH)
_u32, _u64, _vp, _int = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int

lib.bmqcrc_crc32c.restype = _u32
lib.bmqcrc_crc32c.argtypes = [_vp, _u32, _u32]
lib.bmqcrc_crc32c_blob.restype = _u32
lib.bmqcrc_crc32c_blob.argtypes = [ctypes.POINTER(_vp), ctypes.POINTER(_u32), _u32, _u32]
lib.bmqcrc_combine.restype = _u32
lib.bmqcrc_combine.argtypes = [_u32, _u32, _u64]
lib.bmqcrc_crc32c_batch.restype = _int
lib.bmqcrc_crc32c_batch.argtypes = [_vp, _u64, _vp, _vp, _vp, _vp, _u64, ctypes.POINTER(Opts)]
lib.bmqcrc_crc32c_verify.restype = _int
lib.bmqcrc_crc32c_verify.argtypes = [_vp, _u64, _vp, _vp, _vp, _u64, ctypes.POINTER(_u64), _vp,
                                     _u64, ctypes.POINTER(Opts)]
lib.bmqcrc_crc32c_blobs.restype = _int
lib.bmqcrc_crc32c_blobs.argtypes = [_vp, _u64, _vp, _vp, _u64, _vp, _vp, _vp, _u64,
                                    ctypes.POINTER(Opts)]
lib.bmqcrc_crc32c_batch_multi.restype = _int
lib.bmqcrc_crc32c_gather.restype = _int
lib.bmqcrc_crc32c_gather.argtypes = [ctypes.POINTER(_vp), _vp, _u64, _vp, _vp, _vp, _u64,
                                     ctypes.POINTER(Opts)]
lib.bmqcrc_crc32c_batch_multi.argtypes = [_vp, _u64, _vp, _vp, _vp, _vp, _u64, _vp, _int, _u32]
lib.bmqcrc_reserve.restype = _int
lib.bmqcrc_reserve.argtypes = [_int, _vp, _u64, _u64, _u32]
lib.bmqcrc_fill_synthetic.restype = _int
lib.bmqcrc_fill_synthetic.argtypes = [_vp, _u64, _u64, _u64, ctypes.POINTER(Opts)]
lib.bmqcrc_kernel_timing.restype = _int
lib.bmqcrc_kernel_timing.argtypes = [_int, _vp, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(_u32)]
lib.bmqcrc_last_plan.restype = _int
lib.bmqcrc_last_plan.argtypes = [_int, _vp, ctypes.POINTER(_u32)]
lib.bmqcrc_last_launch.restype = _int
lib.bmqcrc_last_launch.argtypes = [_int, _vp, ctypes.POINTER(_u32), ctypes.POINTER(_u32),
                                   ctypes.POINTER(_u32)]
lib.bmqcrc_forget_shape.restype = _int
lib.bmqcrc_forget_shape.argtypes = [_int, _vp]
if hasattr(lib, "bmqcrc_plan_wait"):  # ABI 2.3 (an older build loads for same-box A/B)
    lib.bmqcrc_plan_wait.restype = _int
    lib.bmqcrc_plan_wait.argtypes = [_int, _vp, _u64, ctypes.POINTER(_u64)]
lib.bmqcrc_host_register.restype = _int
lib.bmqcrc_host_register.argtypes = [_vp, _u64, _int, ctypes.POINTER(_vp)]
lib.bmqcrc_host_unregister.restype = _int
lib.bmqcrc_host_unregister.argtypes = [_vp]
lib.bmqcrc_device_count.restype = _int
lib.bmqcrc_device_count.argtypes = []
lib.bmqcrc_last_error.restype = ctypes.c_char_p
lib.bmqcrc_last_error.argtypes = []
lib.bmqcrc_version.restype = _u32
lib.bmqcrc_version.argtypes = []

# include/bmqcrc_protocol.h
_i64, _pu64, _pint, _popts = ctypes.c_int64, ctypes.POINTER(_u64), ctypes.POINTER(_int), \
    ctypes.POINTER(Opts)
lib.bmqcrc_put_event_scan.restype = _i64
lib.bmqcrc_put_event_scan.argtypes = [_vp, _u64, _vp, _vp, _vp, _u64]
lib.bmqcrc_put_event_fill_crcs.restype = _i64
lib.bmqcrc_put_event_fill_crcs.argtypes = [_vp, _u64, _popts]
lib.bmqcrc_put_event_verify.restype = _int
lib.bmqcrc_put_event_verify.argtypes = [_vp, _u64, _pu64, _pu64, _vp, _u64, _popts]
lib.bmqcrc_journal_scan.restype = _i64
lib.bmqcrc_journal_scan.argtypes = [_vp, _u64, _vp, _u64, _vp, _pint, _pu64, _vp, _vp, _vp, _vp,
                                    _u64]
lib.bmqcrc_journal_bounds.restype = _int
lib.bmqcrc_journal_bounds.argtypes = [_vp, _u64, _pu64, _pu64]
lib.bmqcrc_recover_verify.restype = _int
lib.bmqcrc_recover_verify.argtypes = [_vp, _u64, _vp, _u64, _vp, _pint, _pu64, _pu64, _pu64, _vp,
                                      _u64, _popts]
lib.bmqcrc_csl_scan.restype = _i64
lib.bmqcrc_csl_scan.argtypes = [_vp, _u64, _vp, _vp, _vp, _vp, _u64, _pint, _pu64]
lib.bmqcrc_csl_validate.restype = _int
lib.bmqcrc_csl_validate.argtypes = [_vp, _u64, _vp, _pint, _pu64, _pu64, _popts]


def check(rc):
    if rc != BMQCRC_OK:
        raise BmqCrcError(rc, lib.bmqcrc_last_error().decode(errors="replace"))
    return rc


def check_count(n):
    """Scans return a count (>= 0) or a negative BMQCRC_E* code."""
    if n < 0:
        raise BmqCrcError(n, lib.bmqcrc_last_error().decode(errors="replace"))
    return n


def make_opts(device=-1, stream=None, flags=0, seg_bytes=0, devices=None, max_len=0,
              min_len=0):
    """bmqcrc_opts; `devices` (a sequence of ordinals, repeats allowed) spreads
    the format-walk entry points over several devices (ABI 2.1); `max_len`
    and `min_len` declare bounds on a device-resident batch's lengths (ABI 2.4)."""
    o = Opts()
    o.struct_size = ctypes.sizeof(Opts)
    o.device = device
    o.stream = stream
    o.flags = flags
    o.seg_bytes = seg_bytes
    o.max_len = max_len
    o.min_len = min_len
    if devices is not None and len(devices) > 1:
        arr = (ctypes.c_int32 * len(devices))(*devices)
        o._devices_keep = arr  # the array lives as long as the opts
        o.ndevices = len(devices)
        o.devices = ctypes.cast(arr, ctypes.c_void_p)
    return o
