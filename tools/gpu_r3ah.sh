# round-3: multi-sub-batch runs as one HIP graph (XC_GRAPH_MULTI=1): the whole GPU suite with it,
# then cfg5 A/B against direct enqueueing
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${1:-r3ah}
mkdir -p $out
XC_GRAPH_MULTI=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_graph.log 2>&1 || { echo "tests rc $?"; tail -60 $out/tests_graph.log; exit 1; }
tail -1 $out/tests_graph.log
B_ENV="XC_GRAPH_MULTI=1" bash tools/ab.sh ${1:-r3ah}/ab 3 || { echo "ab failed"; exit 1; }
echo ok
