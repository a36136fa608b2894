# One driver for the GPU box (replaces the per-lease scripts of earlier rounds).
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# Output under gpurun_out/TAG/.  Steps run in order, each under its own time limit; the first failing
# step ends the call (no retries on the GPU).  Steps:
#   tests[:EXPR]   pytest -m gpu (EXPR: a -k expression, ',' for ' or ')
#   smoke          __graft_entry__.smoke()
#   bench[:ARGS]   python bench.py ARGS (',' for ' ') -> bench.json
#   trace[:ARGS]   rocprofv3 --kernel-trace --stats over bench.py ARGS (default: --no-cpu --no-e2e --no-live --steps 10)
#   leg:LEG[,N]    python bench.py --only LEG --steps N (default 200) -> leg_LEG.json
#   legtrace:LEG   rocprofv3 --kernel-trace over bench.py --only LEG --steps 40 -> timeline_LEG.txt
#   steptrace      rocprofv3 --kernel-trace of cfg5 production steps (--tail-steps 3) -> step_timeline.txt, stats csv
#   calib          tools/fetch_calib under FETCH_SIZE / WRITE_SIZE / TCC request-counter passes -> pmc_calib.json
#   ranks          bench.py --total 32768 / 16384 / 8192 / 4096 (one rank's shard of the 1/2/4/8-GPU job on this GPU)
#   pmc            FETCH_SIZE and WRITE_SIZE passes (separate runs) -> pmc_traffic_cfg5.json (stamped)
#   pmcinst        two SQ counter passes (VALU / LDS / waits) over one cfg5 step -> pmc_inst/
#   py:SCRIPT[:ARGS]  python SCRIPT ARGS
set -o pipefail
tag=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$tag
mkdir -p "$out"
python - > "$out/host.txt" 2>&1 <<'PY'
import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
try:
    print("cpu.max", open("/sys/fs/cgroup/cpu.max").read().strip())
except OSError:
    pass
PY
# (--tail-steps 4: the passes average the last 3 steps, production steps after the diagnostic ones:
# early side-stream hashing, records of shadowed blocks dropped, as in the timed steps)
PMC_BENCH="bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --no-decode --no-legs --no-live --tail-steps 4"
die() { echo "$1 failed (rc $2)"; tail -40 "$3"; exit 1; }
for step in "$@"; do
    name=${step%%:*}
    arg=""
    [ "$name" != "$step" ] && arg=${step#*:}
    echo "== $step"
    case $name in
    tests)
        k=()
        [ -n "$arg" ] && k=(-k "${arg//,/ or }")
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
            > "$out/tests.log" 2>&1 || die tests $? "$out/tests.log"
        tail -1 "$out/tests.log" ;;
    smoke)
        timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
            || die smoke $? "$out/smoke.log"
        tail -1 "$out/smoke.log" ;;
    bench)
        timeout -k 10 900 python bench.py ${arg//,/ } > "$out/bench.json" 2> "$out/bench.err" \
            || die bench $? "$out/bench.err"
        python tools/bench_summary.py "$out/bench.json" ;;
    trace)
        a=${arg//,/ }
        [ -z "$a" ] && a="--no-cpu --no-e2e --no-live --steps 10"
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run \
            -- python3 bench.py $a > "$out/trace.log" 2>&1 || die trace $? "$out/trace.log"
        cp "$out/trace/run_kernel_stats.csv" "$out/bench_kernel_stats.csv"
        rm -rf "$out/trace"
        echo "trace ok" ;;
    leg)
        lg=${arg%%,*}
        n=200
        [ "$lg" != "$arg" ] && n=${arg#*,}
        timeout -k 10 300 python bench.py --only $lg --steps $n > "$out/leg_$lg.json" 2> "$out/leg_$lg.err" \
            || die "leg $lg" $? "$out/leg_$lg.err"
        python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d['verified_buffers'])" "$out/leg_$lg.json" $lg ;;
    legtrace)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/lt_$arg" -o run \
            -- python3 bench.py --only $arg --steps 40 > "$out/lt_$arg.log" 2>&1 || die "legtrace $arg" $? "$out/lt_$arg.log"
        python3 tools/timeline.py "$out/lt_$arg/run_kernel_trace.csv" 40 > "$out/timeline_$arg.txt" || die timeline $? "$out/lt_$arg.log"
        echo "legtrace $arg ok" ;;
    steptrace)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/st" -o run \
            -- python3 bench.py --no-cpu --no-e2e --no-live --no-legs --no-decode --steps 6 --tail-steps 3 \
            > "$out/steptrace.log" 2>&1 || die steptrace $? "$out/steptrace.log"
        python3 tools/timeline.py "$out/st/run_kernel_trace.csv" 75 > "$out/step_timeline.txt" || die timeline $? "$out/steptrace.log"
        cp "$out/st/run_kernel_stats.csv" "$out/step_kernel_stats.csv"
        rm -rf "$out/st"
        tail -4 "$out/step_timeline.txt" ;;
    calib)
        /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/fetch_calib.hip -o /tmp/fetch_calib || die calib-build 1 /dev/null
        mkdir -p "$out/calib"
        timeout -k 10 120 /tmp/fetch_calib > "$out/calib/fetch_calib.csv" || die calib-run $? "$out/calib/fetch_calib.csv"
        i=0
        for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"; do
            i=$((i + 1))
            timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/calib/p$i" -o run -- /tmp/fetch_calib \
                > "$out/calib/p$i.log" 2>&1 || die "calib p$i" $? "$out/calib/p$i.log"
        done
        python tools/pmc_calib.py "$out/calib" "$out/pmc_calib.json" || die pmc_calib 1 /dev/null ;;
    ranks)
        for tot in 32768 16384 8192 4096; do
            timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-legs --no-live --no-decode --steps 20 --total $tot \
                > "$out/ranks_$tot.json" 2> "$out/ranks_$tot.err" || die "ranks $tot" $? "$out/ranks_$tot.err"
            python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d['stats']; print('total', sys.argv[2], d['value'], d['ms_per_step'], s['sub_batches'], s['anchor_scans'], s['early_hashed'], d['verified_buffers'])" "$out/ranks_$tot.json" $tot
        done ;;
    pmc)
        # (pmc:--total,S: a rank-sized shard of S buffers on this GPU -> pmc_traffic_cfg5_bS.json)
        a=${arg//,/ }
        sfx=""
        [ -n "$arg" ] && sfx="_b${arg##*,}"
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/pmc$sfx/$c" -o run -- python3 $PMC_BENCH $a \
                > "$out/pmc${sfx}_$c.log" 2>&1 || die "pmc $c" $? "$out/pmc${sfx}_$c.log"
        done
        python tools/pmc_traffic.py "$out/pmc$sfx" "$out/pmc_traffic_cfg5$sfx.json" auto > "$out/pmc_traffic$sfx.log" 2>&1 \
            || die pmc_traffic $? "$out/pmc_traffic$sfx.log"
        tail -3 "$out/pmc_traffic$sfx.log" ;;
    pmcinst)
        i=0
        for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
                 "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA"; do
            i=$((i + 1))
            timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_inst/p$i" -o run -- python3 $PMC_BENCH \
                > "$out/pmc_inst_p$i.log" 2>&1 || die "pmcinst p$i" $? "$out/pmc_inst_p$i.log"
        done
        echo "pmcinst ok" ;;
    py)
        script=${arg%%:*}
        sargs=""
        [ "$script" != "$arg" ] && sargs=${arg#*:}
        timeout -k 10 900 python "$script" ${sargs//,/ } > "$out/$(basename "$script" .py).log" 2>&1 \
            || die "py $script" $? "$out/$(basename "$script" .py).log"
        tail -5 "$out/$(basename "$script" .py).log" ;;
    *)
        echo "unknown step $step"; exit 2 ;;
    esac
done
echo "all steps ok"
