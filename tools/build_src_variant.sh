#!/bin/bash
# Build an A/B variant of libfia.so from a copy of csrc/ with whole files replaced and optional
# sed edits:  tools/build_src_variant.sh <out.so> [-f <unit.hip> <replacement>]... [-e <file> <sed expr>]...
set -eu
cd "$(dirname "$0")/.."
out=$1; shift
tmp=$(mktemp -d)
cp -r fia-kdd-19_amd/csrc "$tmp/csrc"
rm -rf "$tmp/csrc/build"
while [ $# -ge 3 ]; do
  case $1 in
    -f) cp "$3" "$tmp/csrc/$2" ;;
    -e) sed -i "$3" "$tmp/csrc/$2"; if cmp -s "$tmp/csrc/$2" "fia-kdd-19_amd/csrc/$2"; then echo "no change in $2"; exit 1; fi ;;
    *) echo "bad option $1"; exit 1 ;;
  esac
  shift 3
done
make -C "$tmp/csrc" -j8 ROOT="$(pwd)" OUT="$tmp/libfia.so" OBJDIR="$tmp/build" >/dev/null
cp "$tmp/libfia.so" "$out"
rm -rf "$tmp"
echo "built $out"
