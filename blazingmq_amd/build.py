"""Build the in-tree native artefacts.

* ``blazingmq_amd/lib/libbmqcrc.so`` -- the product: HIP kernels for gfx950
  (hipcc --offload-arch=gfx950) + the C-ABI host code (include/bmqcrc.h).
* ``oracle/lib/liboracle_crc32c.so`` -- the CPU checker (test infrastructure).
* ``tests/cpp/bin/bmqp_selftest`` -- the C++ drop-in (bmqp::Crc32c) test
  driver (test infrastructure), linked against libbmqcrc.so.

hipcc cross-compiles gfx950 code objects without a GPU present.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib")
ORACLE = os.path.join(ROOT, "oracle")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

PRODUCT_SOURCES = ["crc32c_kernels.hip", "bmqcrc_host.cpp", "crc32c_cpu.cpp", "bmqp_crc32c.cpp",
                   "bmqcrc_protocol.cpp"]
PRODUCT_DEPS = ["bmqcrc_internal.h", "crc32c_consts.h"]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def _stale(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def build_consts():
    gen = os.path.join(ROOT, "tools", "gen_crc_consts.py")
    out = os.path.join(CSRC, "crc32c_consts.h")
    if _stale(out, [gen]):
        _run([sys.executable, gen, out])


def build_product(force=False, defines=(), target_name="libbmqcrc.so"):
    """defines: extra -D flags for same-box A/B variants (tools/build_variant.sh)."""
    os.makedirs(LIB, exist_ok=True)
    build_consts()
    target = os.path.join(LIB, target_name)
    srcs = [os.path.join(CSRC, s) for s in PRODUCT_SOURCES]
    deps = srcs + [os.path.join(CSRC, d) for d in PRODUCT_DEPS] + [
        os.path.join(ROOT, "include", "bmqcrc.h"), os.path.join(ROOT, "include", "bmqp_crc32c.h"),
        os.path.join(ROOT, "include", "bmqcrc_protocol.h")]
    if force or _stale(target, deps):
        objs = []
        for s in srcs:
            o = os.path.join(LIB, os.path.basename(s) + ".o")
            cmd = [HIPCC, "-O3", "-fPIC", "-std=c++17", "-Wall", "-I" + os.path.join(ROOT, "include"),
                   *defines, "-c", s, "-o", o]
            if s.endswith(".hip"):
                cmd[1:1] = ["-x", "hip", "--offload-arch=" + ARCH, "-munsafe-fp-atomics"]
            _run(cmd)
            objs.append(o)
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, *objs, "-o", target,
              "-lpthread"])
        for o in objs:
            os.remove(o)
        for leftover in os.listdir(LIB):  # hipcc offload-bundling intermediates
            if leftover.startswith(target_name + "."):
                os.remove(os.path.join(LIB, leftover))
    selftest = os.path.join(ROOT, "tests", "cpp", "bin", "bmqp_selftest")
    st_src = os.path.join(ROOT, "tests", "cpp", "bmqp_crc32c_selftest.cpp")
    if target_name != "libbmqcrc.so":
        return target
    if os.path.exists(st_src) and (force or _stale(selftest, [st_src, target])):
        os.makedirs(os.path.dirname(selftest), exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), st_src,
              "-o", selftest, "-L" + LIB, "-lbmqcrc", "-pthread",
              "-Wl,-rpath,$ORIGIN/../../../blazingmq_amd/lib"])
    build_scalar_ladder(target, force)
    return target


def build_scalar_ladder(target, force=False):
    """bench.py --scalar's harness (tools/scalar_ladder.cpp): a measurement
    tool, so a failure to build it is reported and never fails the product."""
    ladder = os.path.join(ROOT, "tools", "bin", "scalar_ladder")
    ld_src = os.path.join(ROOT, "tools", "scalar_ladder.cpp")
    if os.path.exists(ld_src) and (force or _stale(ladder, [ld_src, target])):
        os.makedirs(os.path.dirname(ladder), exist_ok=True)
        try:
            _run(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"), ld_src,
                  "-o", ladder, "-L" + LIB, "-lbmqcrc",
                  "-Wl,-rpath,$ORIGIN/../../blazingmq_amd/lib"])
        except (OSError, subprocess.CalledProcessError) as e:
            print("warning: tools/scalar_ladder not built (%s); bench.py --scalar is "
                  "unavailable" % e, file=sys.stderr)
    return ladder


def build_oracle(force=False):
    out_dir = os.path.join(ORACLE, "lib")
    os.makedirs(out_dir, exist_ok=True)
    src = os.path.join(ORACLE, "crc32c_oracle.c")
    target = os.path.join(out_dir, "liboracle_crc32c.so")
    if force or _stale(target, [src]):
        _run(["gcc", "-O3", "-fPIC", "-shared", "-pthread", "-Wall", "-Wextra", src, "-o", target])
    return target


def build_all(force=False):
    build_oracle(force)
    return build_product(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
