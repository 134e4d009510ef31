"""Where a render kernel's scalar instructions sit: every instruction of one kernel classified (SALU,
exec-mask bookkeeping, branches, scalar loads, waits, VALU, cross-lane, vector memory, LDS), by the
source line the compiler attributes it to (.loc of a -gline-tables-only build, which emits the same
machine code) and by the loop it sits in.  Static counts: the traversal loops (depth >= 2) are where
the dynamic count is made, so they are listed by loop and by line.

    python tools/salu_map.py [kernel-substring] [asm.s] [--top N]
Without asm.s, rt_fast_prod.hip is compiled here with build.py's flags (+ -gline-tables-only)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytracing_amd"))
import build  # noqa: E402

EXEC_OPS = re.compile(r"s_(and|or|xor|andn2|orn2|nand|nor|xnor|andn1|orn1)_saveexec|s_\w+\s+exec\b|s_mov_b64\s+exec|"
                      r"s_\w+_b64\s+exec,")


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_waitcnt") or op in ("s_nop", "s_setprio", "s_sleep"):
        return "wait"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith(("s_load", "s_buffer_load", "s_memtime", "s_memrealtime", "s_getpc", "s_setpc", "s_swappc")):
        return "smem"
    if op.startswith("s_"):
        return "exec" if EXEC_OPS.search(ins) else "salu"
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        return "xlane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "scratch_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    return "other"


KINDS = ("salu", "exec", "branch", "smem", "xlane", "valu", "vmem", "lds", "wait")


def compile_asm():
    asm = "/tmp/salu_map_prod.s"
    obj, cmd = build._hip_job("rt_fast_prod.hip")
    cmd = [c for c in cmd if c not in ("-fPIC",)]
    i = cmd.index("-c")
    cmd = cmd[:i] + ["--cuda-device-only", "-S", "-gline-tables-only"] + cmd[i:]
    cmd[cmd.index("-o") + 1] = asm
    subprocess.run(cmd, check=True, capture_output=True)
    return asm


def scan(txt, want):
    """-> (kernel symbol, [(kind, source line, loop depth, loop header, text)])."""
    files = {int(m.group(1)): os.path.basename(m.group(2))
             for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', txt, re.M)}
    files.update({int(m.group(1)): os.path.basename(m.group(2))
                  for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', txt, re.M)})
    m = re.search(r"^(_Z\S*" + re.escape(want) + r"\S*):", txt, re.M)
    body = txt[m.start():txt.find(".end_amdhsa_kernel", m.start())]
    loc, depth, header = "?", 0, "-"
    out = []
    for ln in body.split("\n"):
        mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
        if mm:
            loc = f"{files.get(int(mm.group(1)), mm.group(1))}:{mm.group(2)}"
            continue
        mb = re.match(r"^(\.LBB\S+|; %bb\.\d+):", ln)
        if mb:
            name = mb.group(1).lstrip(".").replace("; %bb.", "BB1_")
            mh = re.search(r"Header=(\S+) Depth=(\d+)", ln)
            if mh:
                header, depth = mh.group(1), int(mh.group(2))
            elif "Loop Header: Depth=" in ln or "Inner Loop Header: Depth=" in ln:
                depth = int(re.search(r"Depth=(\d+)", ln).group(1))
                header = name
            else:
                header, depth = "-", 0
            continue
        if ("Loop Header: Depth=" in ln) and ln.strip().startswith(";"):  # continuation line of a header block
            depth = int(re.search(r"Depth=(\d+)", ln).group(1))
            continue
        mi = re.match(r"^\s+([sv]_\S+.*?|global_\S+.*?|buffer_\S+.*?|scratch_\S+.*?|flat_\S+.*?|ds_\S+.*?)\s*(?:;.*)?$", ln)
        if mi and not mi.group(1).startswith(("s_code_end",)):
            ins = mi.group(1)
            out.append((classify(ins), loc, depth, header, ins))
    return m.group(1), out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    top = 25
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
        args = [a for a in args if a != str(top)]
    want = args[0] if args else "render_fast_kernel_w7ILi30ELb0ELi17E"
    asm = args[1] if len(args) > 1 else compile_asm()
    sym, ins = scan(open(asm).read(), want)
    by_depth = collections.defaultdict(collections.Counter)
    by_loop = collections.defaultdict(collections.Counter)
    by_line = collections.defaultdict(collections.Counter)
    for kind, loc, d, hdr, _ in ins:
        by_depth[d][kind] += 1
        if d >= 2:
            by_loop[(d, hdr)][kind] += 1
            by_line[loc][kind] += 1
    print(f"{sym}: {len(ins)} instructions")
    print("by loop depth (static):        " + " ".join(f"{k:>6s}" for k in KINDS))
    for d in sorted(by_depth):
        print(f"  depth {d:<24d}" + " ".join(f"{by_depth[d][k]:6d}" for k in KINDS))
    print("traversal loops (depth >= 2):   " + " ".join(f"{k:>6s}" for k in KINDS))
    for (d, hdr), cnt in sorted(by_loop.items(), key=lambda kv: -(kv[1]["salu"] + kv[1]["exec"])):
        if sum(cnt.values()) < 8:
            continue
        print(f"  {hdr:<18s} depth {d:<3d}" + " ".join(f"{cnt[k]:6d}" for k in KINDS))
    print(f"source lines in the traversal loops, by scalar work (salu + exec + branch + xlane), top {top}:")
    rows = sorted(by_line.items(), key=lambda kv: -(kv[1]["salu"] + kv[1]["exec"] + kv[1]["branch"] + kv[1]["xlane"]))
    for loc, cnt in rows[:top]:
        print(f"  {loc:<28s}" + " ".join(f"{k}={cnt[k]}" for k in KINDS if cnt[k]))


if __name__ == "__main__":
    main()
