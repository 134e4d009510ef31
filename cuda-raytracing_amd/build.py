"""Build the native pieces of this repository.

librt_hip.so   cuda-raytracing_amd/csrc  -> the product: HIP kernels for gfx950 + the C-ABI shim
               + the C++ host scene/BVH mirror (one shared library, include/rt_abi.h).
liboracle.so   oracle/rt_oracle.c        -> the CPU restatement used only by tests, smoke() and
               bench.py's cpu_baseline leg (gcc, OpenMP, -ffp-contract=off).

Both are built in-tree so the built .so files travel to the GPU box with the repo snapshot.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-raytracing_amd")
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "build")
LIB = os.path.join(PKG, "librt_hip.so")
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")

# Numerics flags shared by every translation unit of the product: no FMA contraction, IEEE
# fp32 division and square root (bit-exact agreement between host code, kernels and oracle).
FP_FLAGS = ["-ffp-contract=off", "-fno-fast-math"]
# Device code generation: branches on wave-uniform conditions stay scalar branches instead of being
# structurized like divergent ones (config 2: 15.65 vs 15.93 ms per frame, three interleaved runs
# on one box, tools/build_variant.sh + tools/gpu_variants.sh; config 4 unchanged).
HIP_CODEGEN_FLAGS = ["-mllvm", "-structurizecfg-skip-uniform-regions=1"]
# ... except for the 6-wave kernels: each render family below is compiled twice, once with the option
# and its 6-wave kernels sent to a second unit (RT_W6_SPLIT), once without the option holding only those
# (RT_W6_ONLY) -- the 6-wave leaf-tree kernel was miscompiled under the option (rt_fast_body.h)
W6_SPLIT = {"rt_fast_prod.hip", "rt_fast_timing.hip", "rt_fast_ab.hip", "rt_fast_ab2.hip", "rt_fast_refill.hip",
            "rt_fast_screen.hip"}
HOST_SOURCES = ["scene.cpp", "objload.cpp", "mirror.cpp", "leaftree.cpp", "xorwow.cpp", "image.cpp", "shard.cpp"]
# the render kernel families compile as separate translation units, in parallel (rt_render.h)
HIP_SOURCES = ["rt_fast_prod.hip", "rt_fast_timing.hip", "rt_fast_stats.hip", "rt_ref.hip", "rt_kernel.hip", "image.hip",
               "bvh_build.hip", "comm.hip"]
# librt_hip_exp.so: the exact alternatives kept for A/B measurement and their parity tests (A/B kernel
# variants, refill, the lone-pixel kernel, the wavefront tracer); loading it registers them with
# librt_hip.so (rt_render.h ExperimentalKernels, rt.load_experimental())
EXP_SOURCES = ["rt_fast_ab.hip", "rt_fast_ab2.hip", "rt_fast_refill.hip", "rt_fast_screen.hip", "rt_lone.hip", "rt_wavefront.hip",
               "rt_exp.hip"]
EXP_LIB = os.path.join(PKG, "librt_hip_exp.so")


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _newer(target, deps):
    if not os.path.exists(target):
        return False
    t = os.path.getmtime(target)
    return all(os.path.getmtime(d) <= t for d in deps)


def _deps(dirpath, exts):
    return [os.path.join(dirpath, f) for f in os.listdir(dirpath) if f.endswith(exts)]


def _hip_job(src, w6=None):
    """w6: None (a plain unit), "split" (RT_W6_SPLIT) or "only" (RT_W6_ONLY, without the codegen option)."""
    obj = os.path.join(BUILD, src + (".w6.o" if w6 == "only" else ".o"))
    extra = {None: HIP_CODEGEN_FLAGS, "split": HIP_CODEGEN_FLAGS + ["-DRT_W6_SPLIT"], "only": ["-DRT_W6_ONLY"]}[w6]
    return obj, [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *FP_FLAGS,
                 "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics", "-fno-slp-vectorize", *extra,
                 "-I", INC, "-I", CSRC, "-c", os.path.join(CSRC, src), "-o", obj]


def _hip_jobs(src):
    return [_hip_job(src, "split"), _hip_job(src, "only")] if src in W6_SPLIT else [_hip_job(src)]


def _compile(jobs, force):
    """Compile (object, command) jobs in parallel.  An object is rebuilt when its source or any header
    changed, or when its command line did (the command is recorded next to the object), so flag A/Bs
    never link a stale object."""
    headers = _deps(CSRC, (".h",)) + _deps(INC, (".h",))

    def stale(j):
        obj, cmd = j
        rec = obj + ".cmd"
        same_cmd = os.path.exists(rec) and open(rec).read() == " ".join(cmd)
        return force or not same_cmd or not _newer(obj, [cmd[cmd.index("-c") + 1]] + headers)

    def run(j):
        _run(j[1])
        with open(j[0] + ".cmd", "w") as fh:
            fh.write(" ".join(j[1]))

    from concurrent.futures import ThreadPoolExecutor
    workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 8))
    todo = [j for j in jobs if stale(j)]
    with ThreadPoolExecutor(max_workers=workers) as ex:
        list(ex.map(run, todo))
    return bool(todo)


def build_product(force=False):
    """librt_hip.so and the experimental plugin librt_hip_exp.so (linked against it)."""
    os.makedirs(BUILD, exist_ok=True)
    jobs = [j for src in HIP_SOURCES for j in _hip_jobs(src)]
    for src in HOST_SOURCES:
        obj = os.path.join(BUILD, src + ".o")
        jobs.append((obj, ["g++", "-O2", "-std=c++17", "-fPIC", *FP_FLAGS, "-I", INC, "-I", CSRC,
                           "-c", os.path.join(CSRC, src), "-o", obj]))
    exp_jobs = [j for src in EXP_SOURCES for j in _hip_jobs(src)]
    changed = _compile(jobs + exp_jobs, force)
    objs = [o for o, _ in jobs]
    if changed or not _newer(LIB, objs):
        tmp = LIB + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-L/opt/rocm/lib", "-lrccl", "-o", tmp])
        os.replace(tmp, LIB)
    eobjs = [o for o, _ in exp_jobs]
    if changed or not _newer(EXP_LIB, eobjs + [LIB]):
        tmp = EXP_LIB + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *eobjs, "-L", PKG, "-l:librt_hip.so",
              "-Wl,-rpath,$ORIGIN", "-Wl,--no-undefined", "-o", tmp])
        os.replace(tmp, EXP_LIB)
    return LIB


HOST_DRIVER_SRC = os.path.join(ROOT, "tests", "cpp", "host_driver.cpp")
HOST_DRIVER = os.path.join(ROOT, "tests", "cpp", "host_driver")


def build_host_driver(force=False):
    """The C++ host of tests/test_cpp_host.py: drives librt_hip.so through include/rt_abi.h."""
    deps = [HOST_DRIVER_SRC, LIB, os.path.join(INC, "rt_abi.h")]
    if not os.path.exists(HOST_DRIVER_SRC) or (not force and _newer(HOST_DRIVER, deps)):
        return HOST_DRIVER
    tmp = HOST_DRIVER + ".tmp"
    _run(["g++", "-O2", "-std=c++17", "-I", INC, HOST_DRIVER_SRC, "-L", PKG, "-lrt_hip",
          "-Wl,-rpath,$ORIGIN/../../cuda-raytracing_amd", "-o", tmp])
    os.replace(tmp, HOST_DRIVER)
    return HOST_DRIVER


def build_oracle(force=False):
    src = os.path.join(ORACLE_DIR, "rt_oracle.c")
    deps = [src, os.path.abspath(__file__)] + _deps(ORACLE_DIR, (".h",))
    if not force and _newer(ORACLE_LIB, deps):
        return ORACLE_LIB
    tmp = ORACLE_LIB + ".tmp"
    _run(["gcc", "-O2", "-std=c11", "-fPIC", "-shared", "-fopenmp", *FP_FLAGS, src, "-o", tmp, "-lm"])
    os.replace(tmp, ORACLE_LIB)
    return ORACLE_LIB


def build_reference_parts(force=False):
    """oracle/_ref: the parts of the reference that compile from their own sources here (the
    vendored glm behind oracle/ref_glm.cpp), when /root/reference is present -- a checker for
    the oracle, test infrastructure only (oracle/build_ref.sh)."""
    out = os.path.join(ORACLE_DIR, "_ref", "libref_glm.so")
    deps = [os.path.join(ORACLE_DIR, "ref_glm.cpp"), os.path.join(ORACLE_DIR, "build_ref.sh")]
    if not os.path.isdir("/root/reference/include/glm") or (not force and _newer(out, deps)):
        return out if os.path.exists(out) else None
    _run(["bash", os.path.join(ORACLE_DIR, "build_ref.sh")])
    return out


def build_all(force=False):
    build_product(force)
    build_oracle(force)
    build_reference_parts(force)
    build_host_driver(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
