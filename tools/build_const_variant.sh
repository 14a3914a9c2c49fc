#!/bin/bash
# Build an A/B variant of libfia.so with source edits applied to a copy of csrc/ (e.g. constants):
#   tools/build_const_variant.sh <out.so> <file> <sed expression> [<file> <sed expression> ...]
set -eu
cd "$(dirname "$0")/.."
out=$1; shift
tmp=$(mktemp -d)
cp -r fia-kdd-19_amd/csrc "$tmp/csrc"
rm -rf "$tmp/csrc/build"
while [ $# -ge 2 ]; do
  f=$1; expr=$2; shift 2
  sed -i "$expr" "$tmp/csrc/$f"
  if cmp -s "$tmp/csrc/$f" "fia-kdd-19_amd/csrc/$f"; then echo "no change in $f"; exit 1; fi
done
make -C "$tmp/csrc" -j8 ROOT="$(pwd)" OUT="$tmp/libfia.so" OBJDIR="$tmp/build" >/dev/null
cp "$tmp/libfia.so" "$out"
rm -rf "$tmp"
echo "built $out"
