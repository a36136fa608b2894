# Builds an alternative library wanproxy_amd/libxcodec_hip_b.so (for tools/ab.sh) from the current
# sources with extra compiler flags, in a scratch directory (the in-tree objects stay untouched).
# usage (here, on the CPU): bash tools/build_variant.sh [-DFLAG ...]
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
out=$(mktemp -d /tmp/xcvar.XXXXXX)
mkdir -p "$out"/include "$out"/w/csrc
cp "$root"/include/*.h "$out"/include/
cp "$root"/wanproxy_amd/csrc/*.hip "$root"/wanproxy_amd/csrc/*.h "$root"/wanproxy_amd/csrc/*.cpp "$out"/w/csrc/
cd "$out"/w/csrc
if [ -n "$XC_VARIANT_SED" ]; then sed -i "$XC_VARIANT_SED" ${XC_VARIANT_FILE:-xc_encode.hip}; fi  # (a source edit for the variant)
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-value $*"
for f in xc_encode xc_decode xc_runtime; do /opt/rocm/bin/hipcc $FL -c $f.hip -o $f.o & done
DF=$(printf "%s\n" "$@" | { grep "^-D" || true; } | tr "\n" " ")  # (the -D flags reach the host-only sources too)
for f in *.cpp; do g++ -O2 -std=c++17 -fPIC -Wall $DF -c $f -o ${f%.cpp}.o; done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root"/wanproxy_amd/libxcodec_hip_b.so *.o
rm -rf "$out"
echo "built wanproxy_amd/libxcodec_hip_b.so with: $*"
