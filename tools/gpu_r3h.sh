# round-3: windowed decoder tokenizer: decode tests, A/B against the 1 KiB-window tokenizer (lib b)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3h}
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -k "decode or dec or pipe or fullsize or coss or fuzz" -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests.log; exit 1; }
tail -2 $out/tests.log
bash tools/ab_dec.sh ${1:-r3h}/abdec 3 30
