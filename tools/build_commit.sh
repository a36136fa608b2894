# Builds wanproxy_amd/libxcodec_hip_b.so (for tools/ab.sh) from the sources of another commit.
# usage (here, on the CPU): bash tools/build_commit.sh COMMIT
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
out=$(mktemp -d /tmp/xccommit.XXXXXX)
git -C "$root" archive "$1" include wanproxy_amd/csrc | tar -x -C "$out"
cd "$out"/wanproxy_amd/csrc
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value"
for f in xc_encode xc_decode xc_runtime; do /opt/rocm/bin/hipcc $FL -c $f.hip -o $f.o & done
for f in *.cpp; do g++ -O2 -std=c++17 -fPIC -Wall -c $f -o ${f%.cpp}.o; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root"/wanproxy_amd/libxcodec_hip_b.so *.o
rm -rf "$out"
echo "built wanproxy_amd/libxcodec_hip_b.so from $1"
