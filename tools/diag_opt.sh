#!/bin/bash
# Run the diagnostic against device libraries built at several optimisation levels.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for o in -O1 -O2 -O3; do
  cp tools/libs/libpnrt$o.so pnraytracing_amd/libpnrt.so
  echo "== $o"; timeout -k 10 200 python tools/diag.py || exit 1
done
