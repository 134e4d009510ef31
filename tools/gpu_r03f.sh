#!/bin/bash
# Round 3: same-box A/B of exact-preserving variants on config 2 (bench --no-pmc): default, the floor
# leaf as a leaf tree walked cooperatively (coop_tree), and a cluster size sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
for opt in ${OPTS:-none leaf_tree_min=300 leaf_tree_min=300,cluster_max=8 leaf_tree_min=200}; do
  a=""; [ "$opt" = none ] || a="--build-options $opt"
  timeout -k 10 240 python bench.py --config ${CFG:-cfg2} --no-pmc --no-cpu-baseline --steps 10 --warmup 2 $a > gpurun_out/bo_$opt.log 2>&1
  rc=$?
  echo "rep $rep $opt exit $rc: $(tail -1 gpurun_out/bo_$opt.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["plan"].get("occupancy",{}).get("probe_ms"))' 2>&1 | tail -1)"
  case $rc in 0) ;; *) exit $rc;; esac
done
done
