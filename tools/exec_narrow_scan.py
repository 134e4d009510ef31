"""Scan HIP objects for exec narrowed without a save with vector code behind it -- the pattern behind
round 4's 6-wave mis-render (rt_fast_body.h RT_FAST_FAMILY).  build.py runs the same check
(check_exec_narrowing) on every object it compiles; this prints every narrowing, hazardous or not.

    python tools/exec_narrow_scan.py cuda-raytracing_amd/build/*.hip.o [/tmp/rtvar/*.o]
Exit status 1 when an object has a hazard."""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-raytracing_amd"))
import build  # noqa: E402

bad = 0
for obj in sys.argv[1:]:
    dis = build.disassemble(obj)
    n = len(re.findall(r"^\ts_and_b64 exec, exec,", dis, re.M))
    hz = build.exec_narrowing_hazards(dis)
    print(f"{obj}: {n} exec narrowings without a save, {len(hz)} with vector code behind them")
    for k, addr, ops in hz:
        print(f"  {k} at 0x{addr:x}: " + "; ".join(ops))
    bad += len(hz)
sys.exit(1 if bad else 0)
