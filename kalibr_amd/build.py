"""In-tree builds: libkalibr_hip.so (HIP kernels + C-ABI, gfx950, explicit hipcc, no JIT cache) and
libkalibr_backend.so (the C++ host layer over the C-ABI, host/kalibr_backend.*, plain g++)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "kb_capi.hip")
SRC_SPLINE = os.path.join(HERE, "csrc", "kb_spline.hip")
OUT = os.path.join(HERE, "libkalibr_hip.so")
DEPS = ["kb_capi.hip", "kb_kernels.hip", "kb_pcg.hip", "kb_device.h", "kb_math.h", "kb_spline.hip", "kb_build_tu.hip"]
SRC_BUILD_TU = os.path.join(HERE, "csrc", "kb_build_tu.hip")
N_BUILD_TU = 9  # camera-model sets, one translation unit each (kb_build_tu.hip -DKB_TU_ID=i)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result", "-Wno-unused-value"]


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(HERE, "csrc", f) for f in DEPS] + [os.path.join(HERE, "..", "include", "kalibr_hip.h")]
    return any(os.path.getmtime(p) > t for p in deps)


def _compile_link(out, extra=()):
    """The translation units (kb_capi.hip, kb_spline.hip and the nine per-model-set build-kernel units of
    kb_build_tu.hip) compiled in parallel (hipcc -c, no relocatable device code: each TU owns its kernels), then
    linked into one shared library."""
    jobs = [(out + ".capi.o", SRC, []), (out + ".spline.o", SRC_SPLINE, [])]
    jobs += [(out + ".b%d.o" % i, SRC_BUILD_TU, ["-DKB_TU_ID=%d" % i]) for i in range(N_BUILD_TU)]
    cflags = [f for f in FLAGS if f != "-shared"] + list(extra)
    width = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    pending, running, rcs = list(jobs), [], []
    while pending or running:
        while pending and len(running) < width:
            o, s, d = pending.pop(0)
            running.append(subprocess.Popen([HIPCC] + cflags + d + ["-c", "-o", o, s]))
        running[0].wait()
        rcs.append(running.pop(0).returncode)
    if any(rcs):
        raise subprocess.CalledProcessError(max(rcs), "hipcc -c")
    objs = [o for o, _, _ in jobs]
    subprocess.run([HIPCC] + FLAGS + list(extra) + ["-o", out + ".tmp"] + objs + ["-lrccl"], check=True)
    os.replace(out + ".tmp", out)
    for o in objs:
        os.remove(o)


def build(force=False):
    if force or needs_build():
        _compile_link(OUT)
    return OUT


HOST_SRC = os.path.join(HERE, "host", "kalibr_backend.cpp")
HOST_IO_SRC = os.path.join(HERE, "host", "calibration_io.cpp")
HOST_TOOLS_SRC = os.path.join(HERE, "host", "calibration_tools.cpp")
HOST_OUT = os.path.join(HERE, "libkalibr_backend.so")
INCLUDE = os.path.join(HERE, "..", "include")
CXX = os.environ.get("CXX", "g++")


def build_host(force=False):
    """C++ host layer (LinearSystemSolver / TrustRegionPolicy / Optimizer2 mirror, observation packing and YAML
    export) linked to libkalibr_hip.so."""
    deps = [HOST_SRC, HOST_IO_SRC, HOST_TOOLS_SRC, os.path.join(HERE, "host", "kalibr_backend.hpp"),
            os.path.join(HERE, "host", "calibration_io.hpp"), os.path.join(HERE, "host", "calibration_tools.hpp"), OUT]
    if force or not os.path.exists(HOST_OUT) or any(os.path.getmtime(p) > os.path.getmtime(HOST_OUT) for p in deps):
        cmd = [CXX, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I", INCLUDE, "-o", HOST_OUT + ".tmp", HOST_SRC, HOST_IO_SRC, HOST_TOOLS_SRC,
               "-L", HERE, "-lkalibr_hip", "-Wl,-rpath,$ORIGIN"]
        subprocess.run(cmd, check=True)
        os.replace(HOST_OUT + ".tmp", HOST_OUT)
    return HOST_OUT


def build_variant(name, defines):
    """A measurement variant of the library (kernel alternatives behind -D switches) as libkalibr_hip_<name>.so,
    selected by KB_VARIANT_LIB=<name> (tools and A/B runs only; the product loads libkalibr_hip.so)."""
    out = os.path.join(HERE, "libkalibr_hip_%s.so" % name)
    _compile_link(out, ["-D" + x for x in defines])
    return out


def build_stamps():
    """Diagnostic variant with per-phase s_memrealtime stamps (tools/diag_stamps.py only)."""
    out = os.path.join(HERE, "libkalibr_hip_stamps.so")
    _compile_link(out, ["-DKB_STAMPS"])
    return out


if __name__ == "__main__":
    print(build(force=True))
    print(build_host(force=True))
