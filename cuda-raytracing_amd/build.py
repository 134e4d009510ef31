"""Build the native pieces of this repository.

librt_hip.so   cuda-raytracing_amd/csrc  -> the product: HIP kernels for gfx950 + the C-ABI shim
               + the C++ host scene/BVH mirror (one shared library, include/rt_abi.h).
liboracle.so   oracle/rt_oracle.c        -> the CPU restatement used only by tests, smoke() and
               bench.py's cpu_baseline leg (gcc, OpenMP, -ffp-contract=off).

Both are built in-tree so the built .so files travel to the GPU box with the repo snapshot.
"""
import os
import re
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
# on one box, tools/build_variant.sh + tools/gpu_variants.sh; config 4 unchanged) -- with LLVM's
# redundant-END_CF removal off: that removal lowers an inner divergent if whose join is its parent's
# as `s_and_b64 exec, exec, cond` (no saved mask), and the register allocator, which runs after it, may
# put live-range copies into the flow block behind it, which the lanes turned off then skip.  Together
# with the first option it corrupted the 6-wave leaf-tree kernel (rt_fast_body.h);
# check_exec_narrowing below guards every object against that pattern.
HIP_CODEGEN_FLAGS = ["-mllvm", "-structurizecfg-skip-uniform-regions=1", "-mllvm", "-amdgpu-remove-redundant-endcf=0"]
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


def _hip_job(src):
    obj = os.path.join(BUILD, src + ".o")
    return obj, [HIPCC, "-x", "hip", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", *FP_FLAGS,
                 "-fhip-fp32-correctly-rounded-divide-sqrt", "-munsafe-fp-atomics", "-fno-slp-vectorize",
                 *HIP_CODEGEN_FLAGS, "-I", INC, "-I", CSRC, "-c", os.path.join(CSRC, src), "-o", obj]


LLVM_BIN = "/opt/rocm/lib/llvm/bin"
_VECTOR_OP = re.compile(r"\s*(v_|global_|scratch_|buffer_|ds_|flat_)")
_LANE_OP = re.compile(r"\s*v_(readlane|readfirstlane|writelane)_")  # ignore exec (not a hazard here)


def disassemble(obj):
    """The gfx950 code object inside a HIP object file (.hip_fatbin bundle), disassembled."""
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        fat, co = os.path.join(td, "fat.bin"), os.path.join(td, "dev.co")
        secs = subprocess.run([f"{LLVM_BIN}/llvm-readelf", "-S", obj], check=True, capture_output=True, text=True).stdout
        if ".hip_fatbin" not in secs:
            return ""  # no device code in this unit
        subprocess.run([f"{LLVM_BIN}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(td, "x.o")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM_BIN}/clang-offload-bundler", "--type=o", f"--targets=hipv4-amdgcn-amd-amdhsa--{ARCH}",
                        f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([f"{LLVM_BIN}/llvm-objdump", "-d", f"--mcpu={ARCH}", co], check=True,
                              capture_output=True, text=True).stdout


def parse_disassembly(dis):
    """llvm-objdump text -> ({symbol: address}, [(address, text, (symbol, offset) branch target or None,
    kernel)]).  The format it relies on: `ADDR <sym>:` symbol lines and instruction lines ending in
    `// ADDR: encoding` with `<sym+0xOFF>` on branches (tests/test_build_guard.py pins it)."""
    base, ins = {}, []
    kernel = None
    for ln in dis.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", ln)
        if m:
            kernel = m.group(2)
            base[kernel] = int(m.group(1), 16)
            continue
        m = re.match(r"^\t(.*?)\s*// ([0-9A-F]+):[0-9A-F ]*(?:<(\S+)\+0x([0-9a-f]+)>)?", ln)
        if m:
            tgt = (m.group(3), int(m.group(4), 16)) if m.group(3) else None
            ins.append((int(m.group(2), 16), m.group(1), tgt, kernel))
    return base, ins


def exec_narrowing_hazards(dis):
    """Vector instructions that run under an exec mask narrowed without a save (`s_and_b64 exec, exec, c`)
    in the blocks its execz branch skips to, before the parent's `s_or_b64 exec, exec, s` restores the
    mask: the lanes turned off never run them, although in the thread-level CFG the register allocator
    sees every lane of the parent region passes through that block (rt_fast_body.h RT_FAST_FAMILY).
    `dis` is llvm-objdump output; returns [(kernel, narrowing address, [instructions])]."""
    base, ins = parse_disassembly(dis)
    at = {a: i for i, (a, _, _, _) in enumerate(ins)}
    out = []
    for i, (addr, text, _, k) in enumerate(ins):
        if not text.startswith("s_and_b64 exec, exec,"):
            continue
        j, target = i + 1, None
        while j < len(ins) and not ins[j][1].startswith("s_or_b64 exec, exec,"):
            if target is None and ins[j][1].startswith("s_cbranch_execz") and ins[j][2]:
                sym, off = ins[j][2]
                target = base.get(sym, -1) + off
            j += 1
        if target is None:
            continue
        if target not in at:
            out.append((k, addr, ["(execz target not found)"]))
            continue
        bad = []
        for _, tx, _, _ in ins[at[target]:]:
            if tx.startswith("s_or_b64 exec, exec,") or tx.startswith("s_endpgm"):
                break
            if _VECTOR_OP.match(tx) and not _LANE_OP.match(tx):
                bad.append(tx)
        if bad:
            out.append((k, addr, bad))
    return out


def check_exec_narrowing(objs):
    """Build guard: no HIP object may carry exec_narrowing_hazards (the miscompile of round 4's 6-wave
    kernel).  Raises RuntimeError naming the kernel and the instructions."""
    problems, flagged = [], []
    for obj in objs:
        dis = disassemble(obj)
        if dis and not parse_disassembly(dis)[1]:
            # device code present but nothing parsed: the objdump format changed, the guard would pass blind
            problems.append(f"{os.path.basename(obj)}: device code but no instruction parsed (llvm-objdump format?)")
            flagged.append(obj)
            continue
        for k, addr, bad in exec_narrowing_hazards(dis):
            problems.append(f"{os.path.basename(obj)}: {k} at 0x{addr:x}: " + "; ".join(bad[:4]))
            flagged.append(obj)
    if problems:
        # drop the flagged objects and their command records so the next build recompiles and re-checks
        # them instead of linking them as up to date
        for obj in set(flagged):
            for f in (obj, obj + ".cmd"):
                if os.path.exists(f):
                    os.remove(f)
        raise RuntimeError("exec narrowed without a save with vector code behind it (tools/exec_narrow_scan.py, "
                           "rt_fast_body.h RT_FAST_FAMILY):\n  " + "\n  ".join(problems))


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
    jobs = [_hip_job(src) for src in HIP_SOURCES]
    for src in HOST_SOURCES:
        obj = os.path.join(BUILD, src + ".o")
        jobs.append((obj, ["g++", "-O2", "-std=c++17", "-fPIC", *FP_FLAGS, "-I", INC, "-I", CSRC,
                           "-c", os.path.join(CSRC, src), "-o", obj]))
    exp_jobs = [_hip_job(src) for src in EXP_SOURCES]
    changed = _compile(jobs + exp_jobs, force)
    objs = [o for o, _ in jobs]
    eobjs = [o for o, _ in exp_jobs]
    relink = changed or not _newer(LIB, objs)
    relink_exp = changed or not _newer(EXP_LIB, eobjs + [LIB])
    if relink or relink_exp:
        # guard every object about to be linked, whether or not this build compiled it (a flagged object
        # is deleted, so it can never be linked by a later build as up to date)
        check_exec_narrowing([o for o, _ in jobs + exp_jobs if o.endswith(".hip.o")])
    if relink:
        tmp = LIB + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-L/opt/rocm/lib", "-lrccl", "-o", tmp])
        os.replace(tmp, LIB)
    if relink_exp:
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
