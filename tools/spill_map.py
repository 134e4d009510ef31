"""Where a render kernel spills: every scratch load / store of one kernel, by the source line the
compiler attributes it to (.loc of a -gline-tables-only build, which emits the same machine code) and
by the loop nest it sits in.

    python tools/spill_map.py [kernel-substring] [asm.s]
Without asm.s, rt_fast_prod.hip is compiled here with build.py's flags (+ -gline-tables-only)."""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuda-raytracing_amd"))
import build  # noqa: E402

want = sys.argv[1] if len(sys.argv) > 1 else "render_fast_kernel_w7ILi30ELb0ELi17E"
if len(sys.argv) > 2:
    asm = sys.argv[2]
else:
    asm = "/tmp/spill_map_prod.s"
    obj, cmd = build._hip_job("rt_fast_prod.hip")
    cmd = [c for c in cmd if c not in ("-fPIC",)]
    i = cmd.index("-c")
    cmd = cmd[:i] + ["--cuda-device-only", "-S", "-gline-tables-only"] + cmd[i:]
    cmd[cmd.index("-o") + 1] = asm
    subprocess.run(cmd, check=True, capture_output=True)
txt = open(asm).read()
files = {int(m.group(1)): os.path.basename(m.group(2)) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', txt, re.M)}
files.update({int(m.group(1)): os.path.basename(m.group(2)) for m in re.finditer(r'^\s*\.file\s+(\d+)\s+"([^"]+)"\s*$', txt, re.M)})
m = re.search(r"^(_Z\S*" + re.escape(want) + r"\S*):", txt, re.M)
body = txt[m.start():txt.find(".end_amdhsa_kernel", m.start())]
loc, depth = "?", 0
count = collections.Counter()
for ln in body.split("\n"):
    mm = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", ln)
    if mm:
        loc = f"{files.get(int(mm.group(1)), mm.group(1))}:{mm.group(2)}"
        continue
    if re.match(r"^(\.LBB\S+|; %bb\.\d+):", ln):  # a block: its loop depth from the annotation
        mm = re.search(r"Depth=(\d+)", ln)
        depth = int(mm.group(1)) if mm else 0
    mm = re.match(r"\s+(scratch_(load|store)\S*)", ln)
    if mm:
        count[(mm.group(2), loc, depth)] += 1
print(f"{m.group(1)}: {sum(v for (k, _, _), v in count.items() if k == 'store')} scratch stores, "
      f"{sum(v for (k, _, _), v in count.items() if k == 'load')} loads")
for (kind, where, d), n in sorted(count.items(), key=lambda kv: (-kv[0][2], kv[0][1])):
    print(f"  {kind:5s} x{n:3d}  loop depth {d}  {where}")
