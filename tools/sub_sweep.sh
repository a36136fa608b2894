cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sub
for m in 256 384 512 768; do XC_SUB_MB=$m timeout -k 10 200 python bench.py --no-cpu --no-e2e --verify 0 > gpurun_out/sub/b$m.log 2>&1 || exit 1; done
