#!/bin/bash
# Memory-pipeline counters of the production render kernel (config CFG, default cfg2): one
# rocprofv3 --pmc pass per counter group (block limits: 8 SQ, 4 TCP, 2 TA, 2 TD, 4 TCC), plus the
# list of counters the device offers.  A pass that fails on an unknown counter is reported and
# skipped; a time-out, abort or crash ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/pmc_mem
export TMPDIR=/tmp
R="$PWD"
CFG="${CFG:-cfg2}"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/pmc_mem/avail.txt" 2>&1
rc=$?; echo "list exit $rc"; case $rc in 124|134|137|139) exit $rc;; esac
GROUPS_FILE="${GROUPS_FILE:-$R/tools/pmc_mem_groups.txt}"
i=0
while read -r line; do
  [ -z "$line" ] && continue
  case "$line" in \#*) continue;; esac
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $line --output-format csv -d "$R/gpurun_out/pmc_mem/p$i" -o run -- \
    python3 "$R/bench.py" --config "$CFG" --no-pmc --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/pmc_mem/p$i.log" 2>&1
  rc=$?; echo "pass $i ($line) exit $rc"
  case $rc in 0) ;; 124|134|137|139) exit $rc;; *) continue;; esac
done < "$GROUPS_FILE"
cd "$R"
python3 - <<'PY'
import csv, glob, collections, json, os
acc = collections.defaultdict(float); n = collections.Counter()
for p in glob.glob("gpurun_out/pmc_mem/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if not any(f in k for f in os.environ.get("KFILTER", "render_fast_kernel").split(",")): continue
        if "render_fast_kernel" in k and "false" not in k: continue
        key = (k.split("(")[0].replace("void rtk::", ""), r["Counter_Name"])
        acc[key] += float(r["Counter_Value"]); n[key] += 1
out = collections.defaultdict(dict)
for (k, c), v in sorted(acc.items()):
    out[k][c] = v if os.environ.get("SUM") else v / n[(k, c)]
print(json.dumps(out, indent=1))
PY
