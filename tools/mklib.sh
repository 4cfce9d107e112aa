#!/bin/bash
# Builds libmobilert_amd.so from a git revision (or the working tree with "WT") into ab/<name>.so
# for tools/build_ab.sh.  usage: tools/mklib.sh <rev|WT> <name> [extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
if [ "$rev" = "WT" ]; then
  cp -r mobileraytracer_amd/csrc include "$tmp/"
  mkdir -p "$tmp/mobileraytracer_amd" && mv "$tmp/csrc" "$tmp/mobileraytracer_amd/csrc"
else
  git archive "$rev" mobileraytracer_amd/csrc include | tar -x -C "$tmp"
fi
rm -rf "$tmp/mobileraytracer_amd/csrc/build"
mkdir -p ab
make -s -j8 -C "$tmp/mobileraytracer_amd/csrc" OUT="$(pwd)/ab/$name.so" FLAGS_EXTRA="$*" >/dev/null
rm -rf "$tmp"
echo "ab/$name.so"
