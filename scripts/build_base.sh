#!/bin/bash
# Build lego-loam-sr_amd/libllsr_base.so for scripts/ab_odo.sh: the tree's library with the kernel
# files listed in BASE_FILES taken from git revision BASE_REV (default HEAD), everything else as in
# the working tree (so the A/B isolates the uncommitted kernel changes to those files).
set -eu
cd "$(dirname "$0")/.."
REV=${BASE_REV:-HEAD}
TMP=$(mktemp -d /tmp/llsr_base.XXXXXX)
cp -r lego-loam-sr_amd include "$TMP/"
rm -rf "$TMP/lego-loam-sr_amd/build" "$TMP/lego-loam-sr_amd/"*.so
for f in ${BASE_FILES:?list of lego-loam-sr_amd/csrc files}; do
  git show "$REV:lego-loam-sr_amd/csrc/$f" > "$TMP/lego-loam-sr_amd/csrc/$f"
done
if [ -n "${BASE_SED:-}" ]; then sed -i "$BASE_SED" "$TMP/lego-loam-sr_amd/csrc/${BASE_SED_FILE:?}"; fi
make -s -j8 -C "$TMP/lego-loam-sr_amd" libllsr.so
cp "$TMP/lego-loam-sr_amd/libllsr.so" lego-loam-sr_amd/libllsr_base.so
rm -rf "$TMP"
