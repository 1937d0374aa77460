#!/bin/bash
# Per-kernel times of the IP + feature batch for library variants lego-loam-sr_amd/libllsr_<v>.so
# (VARIANTS, "tree" = the tree's libllsr.so): scripts/phase_profile.py under LLSR_LIB, both lidars.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-variants}
mkdir -p "$OUT"
for v in ${VARIANTS:-base tree}; do
  lib=$PWD/lego-loam-sr_amd/libllsr_$v.so
  [ "$v" = tree ] && lib=$PWD/lego-loam-sr_amd/libllsr.so
  for lid in vlp16:1024 hdl64e:512; do
    LLSR_LIB=$lib PHASES=${PHASES:-7:-2:-1} timeout -k 10 200 python scripts/phase_profile.py ${lid%%:*} ${lid##*:} > "$OUT/$v.${lid%%:*}.json" 2> "$OUT/$v.${lid%%:*}.err" || exit $?
  done
done
