#!/bin/bash
# One PMC pass per --tune value (render kernel instruction mix): AB="0 4096" bash tools/gpu_pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
R="$PWD"
CNT="${CNT:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM}"
for t in ${AB:-0}; do
  cd /tmp
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CNT --output-format csv -d "$R/gpurun_out/pmc_$t" -o run -- python3 "$R/bench.py" --tune $t --no-pmc --steps 1 --warmup 0 --no-cpu-baseline > "$R/gpurun_out/pmc_$t.log" 2>&1
  rc=$?; echo "pmc $t exit $rc"; cd "$R"; case $rc in 0) ;; *) exit $rc;; esac
  python3 - "$t" <<'PY'
import csv, glob, sys, collections
t = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for p in glob.glob(f"gpurun_out/pmc_{t}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "render_fast_kernel" not in k or "false" not in k: continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[(k, r["Counter_Name"])] += 1
for k, cs in acc.items():
    print(t, k.split("(")[0][-60:], {c: round(v / n[(k, c)] / 1e6, 2) for c, v in cs.items()})
PY
done
