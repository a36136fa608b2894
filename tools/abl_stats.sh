# Per-kernel averages of tools/leg_abl.py (unchecked timing diagnostic) under several environments.
# usage (GPU box): bash tools/abl_stats.sh TAG LEG "ENV_A" "ENV_B" ...   (ENV: VAR=value ..., or "-")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
tag=$1; leg=$2; shift 2
i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  d=gpurun_out/$tag/v$i
  mkdir -p $d
  env $e timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
      -- python3 tools/leg_abl.py $leg 200 > $d/abl.log 2>&1 || exit 1
  echo "== v$i: $e  $(tail -1 $d/abl.log | cut -c1-70)"
  python3 - $d/run_kernel_stats.csv <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))[:9]:
    print(f"  {r['Name'].split('(')[0][-34:]:34s} calls {int(r['Calls']):6d} avg_us {float(r['AverageNs'])/1e3:8.2f}")
PY
done
