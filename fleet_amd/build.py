"""Build the native libraries of fleet_amd in-tree (they travel to the GPU box).

  fleet_amd/libfleetcodec.so   HIP kernels (gfx950) + the C-ABI of include/fleet_codec.h
  fleet_amd/libfleet_native.so JNI shim re-exporting the reference's Java_* symbols
                               (built against the test JNI header when no JDK is present)

Flags: -ffp-contract=off keeps every fp32/fp64 operation a single IEEE rounding
(the codec must match the reference's x86-64 SSE arithmetic bit for bit);
no fast-math; f32 denormals are kept (hipcc's gfx950 default).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libfleetcodec.so")
JNI_LIB = os.path.join(PKG, "libfleet_native.so")
ARCH = os.environ.get("FLEET_OFFLOAD_ARCH", "gfx950")

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
COMMON = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-fno-slp-vectorize", f"-I{INCLUDE}", f"-I{CSRC}"]

SOURCES = [("kernels.hip", True), ("stream_kernels.hip", True), ("model_codec.hip", True), ("fleet_codec.cpp", True),
           ("model_state.cpp", True), ("teacher.hip", True), ("sampler_state.cpp", True)]


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError("build failed: " + " ".join(cmd))
    return r


def build_codec(force: bool = False, out: str = LIB, defines=()) -> str:
    """Build libfleetcodec.so; `out` / `defines` (-D flags) build an experiment
    variant elsewhere (e.g. ab/ for gpu_ab_workloads.sh (r04 tree)) from the same sources."""
    srcs = [os.path.join(CSRC, s) for s, _ in SOURCES]
    deps = srcs + [os.path.join(CSRC, h) for h in ("codec_device.h", "codec_math.h", "decimal6.h", "kernels.h", "model_codec.h",
                                                   "teacher_math.h")] + [
        os.path.join(INCLUDE, "fleet_codec.h")]
    if not force and not defines and not _newer(out, deps):
        return out
    objdir = os.path.join(PKG, "build") if out == LIB else out + ".objs"
    os.makedirs(objdir, exist_ok=True)

    def compile_one(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        lang = ["-x", "hip", f"--offload-arch={ARCH}"]
        # the stream kernels are VALU-issue bound at 5-6 waves per SIMD: the ILP-first
        # machine scheduler beats the default there and loses on the tiles, hence their
        # own unit (FLEET_STREAM_SCHED=default builds it with the default scheduler)
        sched = os.environ.get("FLEET_STREAM_SCHED", "max-ilp")
        extra = ["-mllvm", f"-amdgpu-sched-strategy={sched}"] if (
            src.endswith("stream_kernels.hip") and sched != "default") else []
        main_sched = os.environ.get("FLEET_MAIN_SCHED", "")  # experiments: the main unit's scheduler
        if main_sched and src.endswith("/kernels.hip"):
            extra = ["-mllvm", f"-amdgpu-sched-strategy={main_sched}"]
        _run([HIPCC, *lang, *COMMON, *extra, *[f"-D{d}" for d in defines], "-c", src, "-o", obj])
        return obj

    with ThreadPoolExecutor(max_workers=len(srcs)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out + ".tmp"
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp])
    os.replace(tmp, out)
    return out


def build_jni(force: bool = False) -> str:
    """JNI shim. With JAVA_HOME set it builds against the real <jni.h>; otherwise
    against the minimal test header (tests/native/jni) so tests can drive it."""
    src = os.path.join(CSRC, "jni_shim.cpp")
    if not os.path.exists(src):
        return ""
    jh = os.environ.get("JAVA_HOME")
    if jh and os.path.exists(os.path.join(jh, "include", "jni.h")):
        inc = [f"-I{jh}/include", f"-I{jh}/include/linux"]
    else:
        inc = [f"-I{os.path.join(ROOT, 'tests', 'native', 'jni')}"]
    if not force and not _newer(JNI_LIB, [src, LIB, os.path.join(INCLUDE, "fleet_codec.h")]):
        return JNI_LIB
    tmp = JNI_LIB + ".tmp"
    _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", *inc, f"-I{INCLUDE}", src, "-o", tmp,
          f"-L{PKG}", "-lfleetcodec", "-Wl,-rpath,$ORIGIN"])
    os.replace(tmp, JNI_LIB)
    return JNI_LIB


def build_all(force: bool = False) -> None:
    build_codec(force)
    build_jni(force)


if __name__ == "__main__":
    # python -m fleet_amd.build [--force] | --variant OUT.so NAME=VALUE ...
    if "--variant" in sys.argv:
        i = sys.argv.index("--variant")
        print(build_codec(True, os.path.abspath(sys.argv[i + 1]), tuple(sys.argv[i + 2:])))
    else:
        build_all(force="--force" in sys.argv)
        print(LIB)
