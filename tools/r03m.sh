set -o pipefail
V="FHESPEAR_LIB=$GRAFT_REPO_ROOT/fhe-spear_amd/lib/variants/libfhespear_hip_ntmore.so"
bash tools/gpu_ab.sh r03m "base1" "ntm1 $V" "base2" "ntm2 $V"
