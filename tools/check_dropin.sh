#!/usr/bin/env bash
# Drop-in check: compiles every band_amd/csrc/backend/hip/*.cc against the
# REFERENCE's own band/ headers (band/interface/*, band/backend_factory.h,
# band/device/cpu.h, band/common.h, band/model_spec.h) - not this repo's
# compat/ stand-ins - plus only the absl status shim, exactly as the files
# would compile after INTEGRATION.md §2's copy into band/backend/hip/.
# Usage: tools/check_dropin.sh [/root/reference]   (exit 0 = every file compiles)
set -uo pipefail
REF=${1:-/root/reference}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/band_amd/csrc
[ -f "$REF/band/interface/model_executor.h" ] || { echo "no reference tree at $REF" >&2; exit 2; }
SHIM=$(mktemp -d)
trap 'rm -rf "$SHIM"' EXIT
ln -s "$CSRC/compat/absl" "$SHIM/absl"   # absl/status/{status,statusor}.h only
fail=0
for f in "$CSRC"/backend/hip/*.cc; do
  # the backend's own headers resolve as "backend/hip/..." (the path they
  # take inside Band); band/... resolves to the reference first
  if ! out=$(g++ -std=c++17 -fsyntax-only -Wall -I"$REF" -I"$SHIM" -I"$ROOT/include" -iquote "$CSRC" "$f" 2>&1); then
    echo "FAIL ${f#$ROOT/}"; echo "$out" | grep -E 'error' | head -5; fail=1
  else
    echo "ok   ${f#$ROOT/}"
  fi
done
# nothing in the backend may reach the harness or the stand-ins
if grep -nE '#include "(engine|compat)/' "$CSRC"/backend/hip/*.cc "$CSRC"/backend/hip/*.h; then
  echo "FAIL backend includes a harness / compat header"; fail=1
fi
exit $fail
