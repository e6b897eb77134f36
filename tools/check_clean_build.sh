#!/bin/bash
# Pre-commit gate: build the STAGED tree (git index) in a clean directory -- no built artefacts,
# no untracked files -- exactly as a fresh checkout would, then run the CPU ABI checks there.
# Usage: git add -A && tools/check_clean_build.sh && git commit ...
set -eu
cd "$(dirname "$0")/.."
tree=$(git write-tree)
dst=$(mktemp -d /tmp/sdp_clean.XXXXXX)
trap 'rm -rf "$dst"' EXIT
git archive "$tree" | tar -x -C "$dst"
cd "$dst"
echo "[clean-build] tree $tree in $dst"
python __graft_entry__.py build > build.log 2>&1 || { tail -40 build.log; echo "[clean-build] BUILD FAILED"; exit 1; }
python -m pytest tests/test_lib_abi.py -q -p no:cacheprovider 2>&1 | tail -3
echo "[clean-build] OK"
