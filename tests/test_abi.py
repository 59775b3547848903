"""The C-ABI library loads and exports every entry point include/bmqcrc.h and
include/bmqcrc_protocol.h declare, and nothing else under the bmqcrc_ prefix
(no compute on a GPU here)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "blazingmq_amd", "lib", "libbmqcrc.so")


HEADERS = ("bmqcrc.h", "bmqcrc_protocol.h")


def declared():
    src = ""
    for h in HEADERS:
        with open(os.path.join(ROOT, "include", h)) as f:
            src += f.read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(bmqcrc_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_api():
    names = declared()
    for n in ("bmqcrc_crc32c", "bmqcrc_crc32c_blob", "bmqcrc_combine", "bmqcrc_crc32c_batch",
              "bmqcrc_crc32c_batch_multi", "bmqcrc_reserve", "bmqcrc_fill_synthetic",
              "bmqcrc_kernel_timing", "bmqcrc_device_count", "bmqcrc_last_error",
              "bmqcrc_version", "bmqcrc_crc32c_verify", "bmqcrc_crc32c_blobs",
              "bmqcrc_put_event_scan", "bmqcrc_put_event_fill_crcs", "bmqcrc_put_event_verify",
              "bmqcrc_journal_scan", "bmqcrc_journal_bounds", "bmqcrc_recover_verify", "bmqcrc_csl_scan",
              "bmqcrc_csl_validate", "bmqcrc_host_register", "bmqcrc_host_unregister"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    for n in declared():
        assert hasattr(lib, n), n
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    assert set(declared()) <= exported
    # internal launchers and error hooks stay hidden
    assert set(n for n in exported if n.startswith("bmqcrc_")) == set(declared())


def test_library_contains_gfx950_code_object(tmp_path):
    # --offloading extracts the bundles next to its input: run it on a copy
    import shutil
    lib = shutil.copy(LIB, tmp_path / "libbmqcrc.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True)
    assert "gfx950" in (out.stdout + out.stderr)


def test_version_and_error_string():
    lib = ctypes.CDLL(LIB)
    lib.bmqcrc_version.restype = ctypes.c_uint32
    assert lib.bmqcrc_version() >> 16 == 2 and lib.bmqcrc_version() & 0xffff >= 7
    lib.bmqcrc_last_error.restype = ctypes.c_char_p
    assert isinstance(lib.bmqcrc_last_error(), bytes)


def test_zero_struct_size_reads_only_the_abi20_fields():
    # struct_size 0 is an ABI 2.0 caller, whose struct ends at ndevices (24
    # bytes): the library must not read past it.  Put the 2.0 fields at the
    # front of a larger buffer whose later bytes are garbage that would be an
    # invalid ndevices / max_len / min_len, and check the call is not
    # refused for them: ENODEV without a GPU, a computed CRC with one.
    from blazingmq_amd import _native as N
    assert N.Opts.ndevices.offset == 24
    payload = (ctypes.c_uint8 * 64)(*range(64))
    offs = (ctypes.c_uint64 * 1)(0)
    lens = (ctypes.c_uint32 * 1)(8)
    out = (ctypes.c_uint32 * 1)()
    raw = (ctypes.c_uint8 * ctypes.sizeof(N.Opts))()
    ctypes.memset(raw, 0xA5, ctypes.sizeof(raw))
    v20 = N.make_opts()
    v20.struct_size = 0
    ctypes.memmove(raw, ctypes.byref(v20), 24)
    rc = N.lib.bmqcrc_crc32c_batch(payload, 64, offs, lens, None, out, 1,
                                   ctypes.cast(raw, ctypes.POINTER(N.Opts)))
    assert rc in (0, N.BMQCRC_ENODEV), (rc, N.lib.bmqcrc_last_error())
    if rc == 0:
        assert out[0] == N.lib.bmqcrc_crc32c(payload, 8, 0)


def test_opts_layout_matches_the_header(tmp_path):
    # bmqcrc_opts as the C compiler lays it out (ABI 2.4 appends max_len, 2.5 min_len) and
    # as the ctypes binding does: same size, same field offsets
    from blazingmq_amd import _native as N
    src = tmp_path / "opts.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "bmqcrc.h"\n'
                   'int main(void) { printf("%zu %zu %zu %zu %zu\\n", sizeof(bmqcrc_opts), '
                   'offsetof(bmqcrc_opts, ndevices), offsetof(bmqcrc_opts, devices), '
                   'offsetof(bmqcrc_opts, max_len), offsetof(bmqcrc_opts, min_len)); return 0; }\n')
    exe = tmp_path / "opts"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    assert got == [ctypes.sizeof(N.Opts), N.Opts.ndevices.offset, N.Opts.devices.offset,
                   N.Opts.max_len.offset, N.Opts.min_len.offset]
