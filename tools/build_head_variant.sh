# Builds wanproxy_amd/libxcodec_hip_b.so (for tools/ab.sh, ab_dec.sh) from the sources of a commit
# (default HEAD), so that a working-tree change can be timed against it.  In a scratch directory.
# usage (here, on the CPU): bash tools/build_head_variant.sh [REV]
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
rev=${1:-HEAD}
out=$(mktemp -d /tmp/xchead.XXXXXX)
mkdir -p "$out"/include "$out"/w/csrc
cd "$root"
for f in $(git ls-tree --name-only "$rev" include/ | grep '\.h$'); do git show "$rev:$f" > "$out/$f"; done
for f in $(git ls-tree --name-only "$rev" wanproxy_amd/csrc/ | grep -E '\.(hip|h|cpp)$'); do
    git show "$rev:$f" > "$out/w/csrc/$(basename $f)"
done
cd "$out"/w/csrc
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value"
for f in xc_encode xc_decode xc_runtime; do /opt/rocm/bin/hipcc $FL -c $f.hip -o $f.o & done
for f in *.cpp; do g++ -O2 -std=c++17 -fPIC -Wall -c $f -o ${f%.cpp}.o; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root"/wanproxy_amd/libxcodec_hip_b.so *.o
cd "$root"
rm -rf "$out"
echo "built wanproxy_amd/libxcodec_hip_b.so from $rev"
