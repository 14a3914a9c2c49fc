#!/bin/bash
# Fast A/B variant of libfia.so: copies csrc/ with the in-tree objects (timestamps kept), applies
# sed edits, and lets make rebuild only the edited units before linking.
#   tools/build_unit_variant.sh <out.so> <file> <sed expression> [<file> <sed expression> ...]
set -eu
cd "$(dirname "$0")/.."
out=$1; shift
tmp=$(mktemp -d)
cp -rp fia-kdd-19_amd/csrc "$tmp/csrc"
while [ $# -ge 2 ]; do
  f=$1; expr=$2; shift 2
  sed -i "$expr" "$tmp/csrc/$f"
  if cmp -s "$tmp/csrc/$f" "fia-kdd-19_amd/csrc/$f"; then echo "no change in $f ($expr)"; rm -rf "$tmp"; exit 1; fi
done
make -C "$tmp/csrc" -j8 ROOT="$(pwd)" OUT="$tmp/libfia.so" OBJDIR="$tmp/csrc/build" >/dev/null
cp "$tmp/libfia.so" "$out"
rm -rf "$tmp"
echo "built $out"
