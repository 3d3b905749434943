#!/bin/bash
# A/B library variants for tools/gpu.sh ab=NAME:FHESPEAR_LIB=... (built here, on the CPU; the .so travels
# with the gpurun snapshot).
#   tools/build_variant.sh NAME [REV] [-DDEFINE ...]
# REV (a git revision, or "-" for the working tree): its fhs_kernels.hip is compiled with the working
# tree's headers and host code, so the variant differs from the current library in the kernels only.
# DEFINEs are passed to both compilations.  Output: fhe-spear_amd/lib/variants/libfhespear_hip_NAME.so
set -e
name=$1
rev=${2:--}
shift $(( $# >= 2 ? 2 : 1 ))
root=$(cd "$(dirname "$0")/.." && pwd)
d=$root/fhe-spear_amd/build/variants/$name
mkdir -p "$d/csrc" "$root/fhe-spear_amd/lib/variants"
cp "$root"/fhe-spear_amd/csrc/* "$d/csrc/"
mkdir -p "$d/../include" && cp "$root"/include/fhespear.h "$d/../include/"   # fhs_host.hip: ../../include
if [ "$rev" != "-" ]; then
    git -C "$root" show "$rev:fhe-spear_amd/csrc/fhs_kernels.hip" > "$d/csrc/fhs_kernels.hip"
fi
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-variable -Wno-unused-function -Wno-unused-value $*"
/opt/rocm/bin/hipcc $F -I"$d/csrc" -c -o "$d/fhs_kernels.o" "$d/csrc/fhs_kernels.hip" &
/opt/rocm/bin/hipcc $F -I"$d/csrc" -c -o "$d/fhs_host.o" "$d/csrc/fhs_host.hip" &
wait
/opt/rocm/bin/hipcc $F -shared -o "$root/fhe-spear_amd/lib/variants/libfhespear_hip_$name.so" "$d/fhs_kernels.o" "$d/fhs_host.o"
echo "built fhe-spear_amd/lib/variants/libfhespear_hip_$name.so"
