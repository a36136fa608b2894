# round-3: cfg3 against caches of 0 / 2 M / 8 M segments, anchor scan (auto) and exact
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3r}
mkdir -p $out
timeout -k 10 500 python tools/bigcache.py 0 2000000 8000000 > $out/bigcache_auto.log 2>&1 || { echo "bigcache auto rc $?"; tail -20 $out/bigcache_auto.log; exit 1; }
grep cache_segments $out/bigcache_auto.log
timeout -k 10 500 python tools/bigcache.py --scan exact 2000000 8000000 > $out/bigcache_exact.log 2>&1 || { echo "bigcache exact rc $?"; tail -20 $out/bigcache_exact.log; exit 1; }
grep cache_segments $out/bigcache_exact.log
