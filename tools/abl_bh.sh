# Block-hashing ablations (XC_ABL_BH, timing only: results wrong in the diagnostic steps) on the cfg5
# step: the side stream's k_blockhash average launch time per variant.  usage (GPU box):
#   bash tools/abl_bh.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/$1
mkdir -p "$out"
for m in 0 2 4 8 12; do
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --no-decode --no-legs --no-live --steps 5 --warmup 1 \
        --diag-env XC_ABL_BH=$m > "$out/abl_bh_$m.json" 2> "$out/abl_bh_$m.err" || { echo "abl $m failed"; tail -5 "$out/abl_bh_$m.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open('$out/abl_bh_$m.json').read().strip().splitlines()[-1]); kr=d['kernel_rooflines'].get('blockhash',{}); print('XC_ABL_BH=$m', 'bh avg ms', kr.get('avg_launch_ms'), 'kernels', d['kernel_ms_per_step'])"
done
