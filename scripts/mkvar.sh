#!/bin/bash
# Build a library variant lego-loam-sr_amd/libllsr_<name>.so: the tree's sources with an edit script
# applied to a copy (python3 EDIT ROOT ARGS...). Usage: bash scripts/mkvar.sh NAME EDIT.py [ARGS...]
set -eu
cd "$(dirname "$0")/.."
name=$1; edit=$2; shift 2
T=$(mktemp -d /tmp/llsr_v.XXXXXX)
cp -r lego-loam-sr_amd include "$T/"
rm -rf "$T/lego-loam-sr_amd/build" "$T/lego-loam-sr_amd/"*.so
python3 "$edit" "$T" "$@" < /dev/null
make -s -j8 -C "$T/lego-loam-sr_amd" libllsr.so
cp "$T/lego-loam-sr_amd/libllsr.so" "lego-loam-sr_amd/libllsr_$name.so"
rm -rf "$T"
