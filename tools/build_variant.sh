# Build an A/B variant of libnngp_hip.so into ab/<name>/ (for tools/gpu_ab.sh / NNGP_LIB).
#   bash tools/build_variant.sh <name> "<extra hipcc flags>" [unit.hip ...]
# Starts from the current in-tree build (pynngp_amd/_build, timestamps kept) and recompiles
# only the listed units (default: the d = 2, m = 14/15 bf_pairb unit) with the extra flags.
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; extra=$2; shift 2
units=("$@")
[ ${#units[@]} -eq 0 ] && units=(bf_pairb_inst_d2_m14_15.hip)
out=ab/$name
rm -rf "$out"; mkdir -p ab
cp -rp pynngp_amd/_build "$out"
touch "$out"/*.o  # only the listed units are recompiled (the copy may predate a header edit)
for u in "${units[@]}"; do rm -f "$out/${u%.hip}.o"; done
make -s -C pynngp_amd/csrc OUT="$(pwd)/$out" EXTRA="$extra" -j8 "$(pwd)/$out/libnngp_hip.so"
echo "$out/libnngp_hip.so"
