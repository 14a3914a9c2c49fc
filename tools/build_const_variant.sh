#!/bin/bash
# Build an A/B variant of libfia.so with one source edit applied to a copy of csrc/ (e.g. a
# constant): tools/build_const_variant.sh <out.so> <file> <sed expression>
set -eu
cd "$(dirname "$0")/.."
out=$1; f=$2; expr=$3
tmp=$(mktemp -d)
cp -r fia-kdd-19_amd/csrc "$tmp/csrc"
rm -rf "$tmp/csrc/build"
sed -i "$expr" "$tmp/csrc/$f"
if cmp -s "$tmp/csrc/$f" "fia-kdd-19_amd/csrc/$f"; then echo "no change in $f"; exit 1; fi
make -C "$tmp/csrc" -j8 ROOT="$(pwd)" OUT="$tmp/libfia.so" OBJDIR="$tmp/build" >/dev/null
cp "$tmp/libfia.so" "$out"
rm -rf "$tmp"
echo "built $out"
