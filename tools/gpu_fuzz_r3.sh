# round-3: the randomized parity campaign at HEAD (every kind; then every eligible run anchor-scanned)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3fuzz}
mkdir -p $out
FUZZ_KINDS=encode,streams,decode,coss,plan timeout -k 10 560 python -u tools/fuzz_campaign.py 480 7000 > $out/fuzz_all.log 2>&1 || { echo "fuzz rc $?"; tail -30 $out/fuzz_all.log; exit 1; }
tail -3 $out/fuzz_all.log
XC_SCAN=anchor FUZZ_KINDS=encode,streams,decode,plan timeout -k 10 320 python -u tools/fuzz_campaign.py 240 9000 > $out/fuzz_anchor.log 2>&1 || { echo "fuzz anchor rc $?"; tail -30 $out/fuzz_anchor.log; exit 1; }
tail -3 $out/fuzz_anchor.log
echo ok
