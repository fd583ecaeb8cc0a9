# Build an A/B variant of libnngp_hip.so into ab/<name>/ (for tools/gpu_ab.sh / NNGP_LIB).
#   [PATCH=tools/variants/x.patch] bash tools/build_variant.sh <name> "<extra hipcc flags>" [unit.hip ...]
# Starts from the current in-tree build (pynngp_amd/_build, timestamps kept) and recompiles
# only the listed units (default: the d = 2, m = 14/15 bf_pairb unit) with the extra flags.  With PATCH,
# the units are compiled from a copy of the sources with that patch applied (the measured-and-rejected
# designs and the timing probes live as patches under tools/variants/, not as switches in the product).
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
src=pynngp_amd/csrc
if [ -n "${PATCH:-}" ]; then
  tmp=$(mktemp -d)
  mkdir -p "$tmp/pynngp_amd" && cp -rp pynngp_amd/csrc "$tmp/pynngp_amd/" && cp -rp include "$tmp/"
  patch -s -d "$tmp" -p0 < "$PATCH"
  # keep the patched files' timestamps: only the listed units (their objects removed above) recompile
  for f in $(grep '^+++ ' "$PATCH" | awk '{print $2}'); do touch -r "$f" "$tmp/$f"; done
  src=$tmp/pynngp_amd/csrc
fi
make -s -C "$src" OUT="$(pwd)/$out" EXTRA="$extra" -j8 "$(pwd)/$out/libnngp_hip.so"
[ -n "${PATCH:-}" ] && rm -rf "$tmp"
echo "$out/libnngp_hip.so"
